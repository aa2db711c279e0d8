// vw_fwd.hip -- launchers (instantiation unit, once per element type) for the kernels in vw_device.h.
#include "vw_launch.h"
#include <algorithm>

namespace vw {

template <typename T, int L, bool FMA, int NV>
static hipError_t run_forward_fused_nv(const FwdArgs<T>& a, int threads, int lds, hipStream_t st) {
  const bool hist = a.hist[0] != nullptr;
  auto k = hist ? k_forward_fused<T, L, FMA, NV, true> : k_forward_fused<T, L, FMA, NV, false>;
  static LdsOnce configured, configured_h;
  hipError_t e = set_lds(k, lds, hist ? &configured_h : &configured);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_forward_fused(const FwdArgs<T>& a, int threads, int lds, int nv, hipStream_t st) {
  if constexpr (L > 0 && L <= 8) {  // NV = 2 (1024 threads): short filters at small batches (host policy)
    if (nv == 2) return run_forward_fused_nv<T, L, FMA, 2>(a, threads, lds, st);
  }
  return nv <= 4 ? run_forward_fused_nv<T, L, FMA, 4>(a, threads, lds, st) : run_forward_fused_nv<T, L, FMA, 8>(a, threads, lds, st);
}

template <typename T>
hipError_t launch_forward_fused(const FwdArgs<T>& a, int threads, int lds, bool fma, int nv, hipStream_t st) {
  switch (a.unrolled ? a.taps : 0) {  // unaligned rows / partial slabs: runtime-L kernel
#define VW_CASE(n) \
    case n: return fma ? run_forward_fused<T, n, true>(a, threads, lds, nv, st) : run_forward_fused<T, n, false>(a, threads, lds, nv, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return fma ? run_forward_fused<T, 0, true>(a, threads, lds, nv, st) : run_forward_fused<T, 0, false>(a, threads, lds, nv, st);
  }
}
template hipError_t launch_forward_fused<VW_T>(const FwdArgs<VW_T>&, int, int, bool, int, hipStream_t);
// Register-blocked PERIODIC forward (k_forward_blk), unrolled tap counts only.
template <typename T, int L, bool FMA, int NV>
static hipError_t run_forward_blk_nv(const FwdArgs<T>& a, int threads, int lds, hipStream_t st) {
  auto k = k_forward_blk<T, L, FMA, NV>;
  static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_forward_blk(const FwdArgs<T>& a, int threads, int lds, bool fma, int nv, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n)                                                                                       \
    case n:                                                                                              \
      if (nv <= 4) return fma ? run_forward_blk_nv<T, n, true, 4>(a, threads, lds, st)                  \
                              : run_forward_blk_nv<T, n, false, 4>(a, threads, lds, st);                 \
      return fma ? run_forward_blk_nv<T, n, true, 8>(a, threads, lds, st) : run_forward_blk_nv<T, n, false, 8>(a, threads, lds, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return hipErrorNotSupported;
  }
}
template hipError_t launch_forward_blk<VW_T>(const FwdArgs<VW_T>&, int, int, bool, int, hipStream_t);

// Persistent forward (k_forward_persist): as many workgroups as are resident at once, each walking
// signals blockIdx.x + k*gridDim.x.  The resident count comes from the occupancy API (LDS-bound).
template <typename T, int L, bool FMA, int NV>
static hipError_t run_forward_persist(const FwdArgs<T>& a, int threads, int lds, hipStream_t st) {
  auto k = k_forward_persist<T, L, FMA, NV>;
  static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
  }
  // resident workgroups per CU: one occupancy query per (threads, LDS) shape, not one per launch
  static int q_threads = -1, q_lds = -1, q_per_cu = 0;
  if (threads != q_threads || lds != q_lds) {
    int per_cu = 0;
    if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, threads, lds)) != hipSuccess) return e;
    q_threads = threads; q_lds = lds; q_per_cu = per_cu;
  }
  const int per_cu = q_per_cu;
  if (per_cu < 1) return hipErrorInvalidConfiguration;
  const long long grid = std::min<long long>(a.B, (long long)per_cu * cus);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_forward_persist_nv(const FwdArgs<T>& a, int threads, int lds, int nv, hipStream_t st) {
  (void)nv;  // NV = 4 only (host contract)
  return run_forward_persist<T, L, FMA, 4>(a, threads, lds, st);
}

template <typename T>
hipError_t launch_forward_persist(const FwdArgs<T>& a, int threads, int lds, bool fma, int nv, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n) \
    case n: return fma ? run_forward_persist_nv<T, n, true>(a, threads, lds, nv, st) : run_forward_persist_nv<T, n, false>(a, threads, lds, nv, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return hipErrorNotSupported;
  }
}
template hipError_t launch_forward_persist<VW_T>(const FwdArgs<VW_T>&, int, int, bool, int, hipStream_t);
}  // namespace vw
