#define VW_T float
// vw_inv_f32.hip -- launchers (instantiation unit) for the kernels in vw_device.h.
#include "vw_device.h"
#include <algorithm>

namespace vw {

// Unrolled tap counts; other L use the runtime-L kernels.  Dev builds may restrict the list:
// make DEV_TAPS='X(8)' (the runtime-L kernel still covers every other L).
#ifdef VW_DEV_TAPS
#define VW_TAP_LIST(X) VW_DEV_TAPS(X)
#else
#define VW_TAP_LIST(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(24) X(30)
#endif

// Raise the dynamic-LDS limit once per kernel instantiation (a call per launch costs host time).
// `configured` must be a static of the caller, which is unique per kernel instantiation.
template <typename Kern>
static hipError_t set_lds(Kern k, int lds_bytes, int* configured) {
  if (lds_bytes > *configured) {
    hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize,
                                       kLdsBytes);
    if (e != hipSuccess) return e;
    *configured = kLdsBytes;
  }
  return hipSuccess;
}

template <typename T, int L, bool FMA, int NV>
static hipError_t run_inverse_fused_nv(const InvArgs<T>& a, int threads, int lds, hipStream_t st) {
  // pairwise sums: k_inverse_fused; sequential sums: two LDS buffers (k_inverse_db) or one (k_inverse_seq)
  static int configured_pair = 64 * 1024, configured_seq = 64 * 1024, configured_db = 64 * 1024;
  auto k = a.pair ? k_inverse_fused<T, L, FMA, NV> : a.db ? k_inverse_db<T, L, FMA, NV> : k_inverse_seq<T, L, FMA, NV>;
  hipError_t e = set_lds(k, lds, a.pair ? &configured_pair : a.db ? &configured_db : &configured_seq);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_inverse_fused(const InvArgs<T>& a, int threads, int lds, int nv, hipStream_t st) {
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
