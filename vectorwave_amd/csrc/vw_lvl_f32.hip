#define VW_T float
// vw_lvl_f32.hip -- launchers (instantiation unit) for the kernels in vw_device.h.
#include "vw_device.h"

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

template <typename T, int L, bool FMA, bool INV>
static hipError_t run_level(const LevelArgs<T>& a, int lds, hipStream_t st) {
  const unsigned tiles = (unsigned)((a.N + a.tile - 1) / a.tile);
  if constexpr (INV) {
    auto k = k_inverse_level<T, L, FMA>;
    static int configured = 64 * 1024;
  hipError_t e = set_lds(k, lds, &configured);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(tiles, (unsigned)a.B), dim3(256), lds, st, a);
  } else {
    auto k = k_forward_level<T, L, FMA>;
    static int configured = 64 * 1024;
  hipError_t e = set_lds(k, lds, &configured);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(tiles, (unsigned)a.B), dim3(256), lds, st, a);
  }
  return hipGetLastError();
}

template <typename T, bool INV>
static hipError_t dispatch_level(const LevelArgs<T>& a, int lds, bool fma, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n) \
    case n: return fma ? run_level<T, n, true, INV>(a, lds, st) : run_level<T, n, false, INV>(a, lds, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return fma ? run_level<T, 0, true, INV>(a, lds, st) : run_level<T, 0, false, INV>(a, lds, st);
  }
}

// Column sweeps (k_forward_sweep / k_inverse_sweep): one thread per (signal, column, q-chunk).
template <typename T>
static unsigned sweep_blocks(const LevelArgs<T>& a) {
  const long long s = a.lv.s, qn = (a.N + s - 1) / s, chunks = (qn + a.tile - 1) / a.tile;
  return (unsigned)((a.B * s * chunks + 255) / 256);
}

template <typename T, int L, bool FMA>
static hipError_t run_forward_sweep(const LevelArgs<T>& a, hipStream_t st) {
  hipLaunchKernelGGL((k_forward_sweep<T, L, FMA>), dim3(sweep_blocks(a)), dim3(256), 0, st, a);
  return hipGetLastError();
}

template <typename T, int L, bool FMA>
static hipError_t run_inverse_sweep(const LevelArgs<T>& a, hipStream_t st) {
  const dim3 g(sweep_blocks(a)), blk(256);
  const int da = a.lv.dir_a > 0, dd = a.lv.dir_d > 0;
  if (da && dd) hipLaunchKernelGGL((k_inverse_sweep<T, L, FMA, 1, 1>), g, blk, 0, st, a);
  else if (da) hipLaunchKernelGGL((k_inverse_sweep<T, L, FMA, 1, -1>), g, blk, 0, st, a);
  else if (dd) hipLaunchKernelGGL((k_inverse_sweep<T, L, FMA, -1, 1>), g, blk, 0, st, a);
  else hipLaunchKernelGGL((k_inverse_sweep<T, L, FMA, -1, -1>), g, blk, 0, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_forward_sweep(const LevelArgs<T>& a, bool fma, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n) \
    case n: return fma ? run_forward_sweep<T, n, true>(a, st) : run_forward_sweep<T, n, false>(a, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default: return hipErrorInvalidValue;  // runtime-L filters use the tiled kernel
  }
}
template <typename T>
hipError_t launch_inverse_sweep(const LevelArgs<T>& a, bool fma, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n) \
    case n: return fma ? run_inverse_sweep<T, n, true>(a, st) : run_inverse_sweep<T, n, false>(a, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default: return hipErrorInvalidValue;
  }
}
template hipError_t launch_forward_sweep<VW_T>(const LevelArgs<VW_T>&, bool, hipStream_t);
template hipError_t launch_inverse_sweep<VW_T>(const LevelArgs<VW_T>&, bool, hipStream_t);

template <typename T>
hipError_t launch_forward_level(const LevelArgs<T>& a, int lds, bool fma, hipStream_t st) {
  return dispatch_level<T, false>(a, lds, fma, st);
}
template <typename T>
hipError_t launch_inverse_level(const LevelArgs<T>& a, int lds, bool fma, hipStream_t st) {
  return dispatch_level<T, true>(a, lds, fma, st);
}
template hipError_t launch_forward_level<VW_T>(const LevelArgs<VW_T>&, int, bool, hipStream_t);
template hipError_t launch_inverse_level<VW_T>(const LevelArgs<VW_T>&, int, bool, hipStream_t);
}  // namespace vw

#include "vw_multi.inc"
