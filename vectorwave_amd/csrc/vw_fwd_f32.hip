#define VW_T float
// vw_fwd_f32.hip -- launchers (instantiation unit) for the kernels in vw_device.h.
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
static hipError_t run_forward_fused_nv(const FwdArgs<T>& a, int threads, int lds, hipStream_t st) {
  auto k = k_forward_fused<T, L, FMA, NV>;
  static int configured = 64 * 1024;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_forward_fused(const FwdArgs<T>& a, int threads, int lds, int nv, hipStream_t st) {
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
// Persistent forward (k_forward_persist): as many workgroups as are resident at once, each walking
// signals blockIdx.x + k*gridDim.x.  The resident count comes from the occupancy API (LDS-bound).
template <typename T, int L, bool FMA>
static hipError_t run_forward_persist(const FwdArgs<T>& a, int threads, int lds, hipStream_t st) {
  auto k = k_forward_persist<T, L, FMA, 4>;
  static int configured = 64 * 1024;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  static int cus = 0;
  if (!cus) {
    int dev = 0;
    if ((e = hipGetDevice(&dev)) != hipSuccess) return e;
    if ((e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev)) != hipSuccess) return e;
  }
  int per_cu = 0;
  if ((e = hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, threads, lds)) != hipSuccess) return e;
  if (per_cu < 1) return hipErrorInvalidConfiguration;
  const long long grid = std::min<long long>(a.B, (long long)per_cu * cus);
  hipLaunchKernelGGL(k, dim3((unsigned)grid), dim3(threads), lds, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_forward_persist(const FwdArgs<T>& a, int threads, int lds, bool fma, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n) \
    case n: return fma ? run_forward_persist<T, n, true>(a, threads, lds, st) : run_forward_persist<T, n, false>(a, threads, lds, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return hipErrorNotSupported;
  }
}
template hipError_t launch_forward_persist<VW_T>(const FwdArgs<VW_T>&, int, int, bool, hipStream_t);
}  // namespace vw
