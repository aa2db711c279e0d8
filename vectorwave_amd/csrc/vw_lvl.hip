// vw_lvl.hip -- launchers (instantiation unit, once per element type) for the kernels in vw_device.h.
#include "vw_launch.h"

namespace vw {

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

// Two inverse levels per launch (k_inverse_sweep2): one workgroup per (signal, 64-residue block,
// u-chunk).  KA = 8 or 16 outputs per stage-A thread and step.
template <typename T, int L, bool FMA, int KA>
static hipError_t run_inverse_sweep2(const LevelArgs<T>& a, hipStream_t st) {
  const long long h = a.lv.s / 2, nu = a.N / h, nch = (nu + a.tile - 1) / a.tile;
  const long long groups = a.B * (h / 64) * nch;
  hipLaunchKernelGGL((k_inverse_sweep2<T, L, FMA, KA>), dim3((unsigned)groups), dim3(kSweep2Threads), 0, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_inverse_sweep2(const LevelArgs<T>& a, int ka, bool fma, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n)                                                                                  \
    case n:                                                                                         \
      if constexpr (n <= 17) {                                                                      \
        if (ka == 8) return fma ? run_inverse_sweep2<T, n, true, 8>(a, st) : run_inverse_sweep2<T, n, false, 8>(a, st); \
      }                                                                                             \
      return fma ? run_inverse_sweep2<T, n, true, 16>(a, st) : run_inverse_sweep2<T, n, false, 16>(a, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default: return hipErrorInvalidValue;
  }
}
template hipError_t launch_inverse_sweep2<VW_T>(const LevelArgs<VW_T>&, int, bool, hipStream_t);

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
