// vw_inv.hip -- launchers (instantiation unit, once per element type) for the kernels in vw_device.h.
#include "vw_launch.h"
#include <algorithm>

namespace vw {

template <typename T, int L, bool FMA, int NV>
static hipError_t run_inverse_fused_nv(const InvArgs<T>& a, int threads, int lds, hipStream_t st) {
  // pairwise sums: k_inverse_fused; sequential sums: two LDS buffers (k_inverse_db) or one (k_inverse_seq)
  static LdsOnce configured_pair, configured_seq, configured_db, configured_blk;
  // register-blocked PERIODIC (host contract; never with NV = 2)
  const bool blk = L > 0 && NV != 2 && a.blk && !a.pair && !a.db;
  auto k = a.pair ? k_inverse_fused<T, L, FMA, NV> : a.db ? k_inverse_db<T, L, FMA, NV> : k_inverse_seq<T, L, FMA, NV>;
  if constexpr (NV != 2) {
    if (blk) k = k_inverse_blk<T, (L > 0 ? L : 2), FMA, NV>;
  }
  hipError_t e = set_lds(k, lds, a.pair ? &configured_pair : a.db ? &configured_db
                                 : blk ? &configured_blk : &configured_seq);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_inverse_fused(const InvArgs<T>& a, int threads, int lds, int nv, hipStream_t st) {
  if constexpr (L > 0 && L <= 8) {  // NV = 2 (1024 threads): short filters at small batches (host policy)
    if (nv == 2) return run_inverse_fused_nv<T, L, FMA, 2>(a, threads, lds, st);
  }
  return nv <= 4 ? run_inverse_fused_nv<T, L, FMA, 4>(a, threads, lds, st) : run_inverse_fused_nv<T, L, FMA, 8>(a, threads, lds, st);
}

template <typename T>
hipError_t launch_inverse_fused(const InvArgs<T>& a, int threads, int lds, bool fma, int nv, hipStream_t st) {
  switch (a.unrolled ? a.taps : 0) {  // unaligned rows / partial slabs: runtime-L kernel
#define VW_CASE(n) \
    case n: return fma ? run_inverse_fused<T, n, true>(a, threads, lds, nv, st) : run_inverse_fused<T, n, false>(a, threads, lds, nv, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return fma ? run_inverse_fused<T, 0, true>(a, threads, lds, nv, st) : run_inverse_fused<T, 0, false>(a, threads, lds, nv, st);
  }
}
template hipError_t launch_inverse_fused<VW_T>(const InvArgs<VW_T>&, int, int, bool, int, hipStream_t);
}  // namespace vw
