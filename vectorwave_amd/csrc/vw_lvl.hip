// vw_lvl.hip -- launchers (instantiation unit, once per element type) for the kernels in vw_device.h.
#include "vw_launch.h"

namespace vw {

template <typename T, int L, bool FMA, bool INV>
static hipError_t run_level(const LevelArgs<T>& a, int lds, hipStream_t st) {
  const unsigned tiles = (unsigned)((a.N + a.tile - 1) / a.tile);
  if constexpr (INV) {
    auto k = k_inverse_level<T, L, FMA>;
    static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k, dim3(tiles, (unsigned)a.B), dim3(256), lds, st, a);
  } else {
    auto k = k_forward_level<T, L, FMA>;
    static LdsOnce configured;
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

// Two / three inverse levels per launch (k_inverse_sweep2 / k_inverse_sweep3): one workgroup per (signal,
// R-residue block, u-chunk) of 4R / 12R threads.  KA = 8 or 16 outputs per thread and step; a block
// (G*KA positions) must cover the reach of the levels below the top, and the rings must fit LDS
// (the host applies the same rule: vw_capi.cpp sweepg_plan).
template <typename T, int L, bool FMA, int KA, int R, int G>
static hipError_t run_inverse_sweepg(const LevelArgs<T>& a, hipStream_t st) {
  constexpr int KMIN = (G == 2 ? 1 : 2) * (L - 1);
  constexpr bool fits = (G == 2 ? 1 : 2) * 3 * G * KA * R * (int)sizeof(T) <= kLdsBytes;
  if constexpr (G * KA >= KMIN && fits) {
    const long long h = a.lv.s / G, nu = a.N / h, nch = (nu + a.tile - 1) / a.tile;
    const long long groups = a.B * (h / R) * nch;
    if constexpr (G == 2)
      hipLaunchKernelGGL((k_inverse_sweep2<T, L, FMA, KA, R>), dim3((unsigned)groups), dim3(4 * R), 0, st, a);
    else
      hipLaunchKernelGGL((k_inverse_sweep3<T, L, FMA, KA, R>), dim3((unsigned)groups), dim3(12 * R), 0, st, a);
    return hipGetLastError();
  } else {
    return hipErrorInvalidValue;
  }
}

template <typename T, int L, bool FMA, int G>
static hipError_t run_inverse_sweepg_k(const LevelArgs<T>& a, int ka, int R, hipStream_t st) {
  if (ka == 8) return R == 64 ? run_inverse_sweepg<T, L, FMA, 8, 64, G>(a, st) : run_inverse_sweepg<T, L, FMA, 8, 32, G>(a, st);
  return R == 64 ? run_inverse_sweepg<T, L, FMA, 16, 64, G>(a, st) : run_inverse_sweepg<T, L, FMA, 16, 32, G>(a, st);
}

template <typename T>
hipError_t launch_inverse_sweepg(const LevelArgs<T>& a, int levels, int ka, int R, bool fma, hipStream_t st) {
  if (R != 64 && R != 32) return hipErrorInvalidValue;
  switch (a.taps) {
#define VW_CASE(n)                                                                                   \
    case n:                                                                                          \
      if (levels == 2) return fma ? run_inverse_sweepg_k<T, n, true, 2>(a, ka, R, st) : run_inverse_sweepg_k<T, n, false, 2>(a, ka, R, st); \
      return fma ? run_inverse_sweepg_k<T, n, true, 4>(a, ka, R, st) : run_inverse_sweepg_k<T, n, false, 4>(a, ka, R, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default: return hipErrorInvalidValue;
  }
}
template hipError_t launch_inverse_sweepg<VW_T>(const LevelArgs<VW_T>&, int, int, int, bool, hipStream_t);

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
