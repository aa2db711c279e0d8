// vw_misc.hip -- launchers (instantiation unit) for the kernels in vw_device.h.
#define VW_MISC_UNIT 1
#include "vw_device.h"
#include "vw_sigma.h"

namespace vw {

// Unrolled tap counts; other L use the runtime-L kernels.  Dev builds may restrict the list:
// make DEV_TAPS='X(8)' (the runtime-L kernel still covers every other L).
#ifdef VW_DEV_TAPS
#define VW_TAP_LIST(X) VW_DEV_TAPS(X)
#else
#define VW_TAP_LIST(X) X(2) X(4) X(6) X(8) X(10) X(12) X(14) X(16) X(18) X(20) X(24) X(30)
#endif


bool has_unrolled_taps(int L) {
  switch (L) {
#define VW_CASE(n) case n: return true;
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default: return false;
  }
}

int fused_max_threads() { return kMaxThreads; }

template <typename T>
hipError_t launch_history_update(const T* in, long long ld_in, const T* old_hist, T* new_hist, long long B, int n,
                                 int hist_len, hipStream_t st) {
  if (hist_len <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_history_update<T>, dim3((unsigned)((hist_len + 255) / 256), (unsigned)B), dim3(256), 0, st,
                     in, ld_in, old_hist, new_hist, n, hist_len);
  return hipGetLastError();
}

static hipError_t run_sigma(const double* x, long long ld, long long B, int N, double scale_c, double* sigma_out,
                            double* thr_out, const double* center, double* median_out, hipStream_t st) {
  hipLaunchKernelGGL(k_noise_sigma, dim3((unsigned)B), dim3(kSigmaThreads), 0, st, x, ld, N, scale_c, sigma_out,
                     thr_out, center, median_out);
  return hipGetLastError();
}

hipError_t launch_noise_sigma(const double* coeffs, long long ld, long long B, int N, double scale_c,
                              double* sigma_out, double* thr_out, hipStream_t st) {
  return run_sigma(coeffs, ld, B, N, scale_c, sigma_out, thr_out, (const double*)nullptr, (double*)nullptr, st);
}

hipError_t launch_median(const double* x, long long ld, long long B, int N, const double* center, double* median_out,
                         hipStream_t st) {
  return run_sigma(x, ld, B, N, 0.0, (double*)nullptr, (double*)nullptr, center, median_out, st);
}

__global__ void __launch_bounds__(256) k_abs_center(const double* __restrict__ x, long long ld, int N,
                                                    const double* __restrict__ center, double* __restrict__ out) {
  const long long b = blockIdx.y;
  const double c = center[b];
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < N; i += gridDim.x * blockDim.x)
    out[b * (long long)N + i] = __builtin_fabs(x[b * ld + i] - c);  // Math.abs(values[i] - median)
}

hipError_t launch_abs_center(const double* x, long long ld, long long B, int N, const double* center, double* out,
                             hipStream_t st) {
  if (B > 65535) return hipErrorInvalidConfiguration;
  const unsigned gx = (unsigned)std::min(std::max((N + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(k_abs_center, dim3(gx, (unsigned)B), dim3(256), 0, st, x, ld, N, center, out);
  return hipGetLastError();
}

hipError_t launch_seq_std(const double* x, int n, double* out, hipStream_t st) {
  hipLaunchKernelGGL(k_seq_std, dim3(1), dim3(64), 0, st, x, n, out);
  return hipGetLastError();
}

hipError_t launch_gather_abs(const double* src, const int* idx, int count, double* window, int wsize, int start,
                             hipStream_t st) {
  if (count <= 0) return hipSuccess;
  hipLaunchKernelGGL(k_gather_abs, dim3((unsigned)((count + 255) / 256)), dim3(256), 0, st, src, idx, count, window,
                     wsize, start);
  return hipGetLastError();
}

// WaveletDenoiser thresholds, one per (level, signal): SURE by the sort + exact-tie kernel, the others
// by k_level_threshold.
hipError_t launch_level_threshold(const double* coeffs, long long level_stride, const double* sigma,
                                  const DenoiseConsts& k, long long B, int levels, double* thr, hipStream_t st) {
  if (B <= 0 || levels <= 0) return hipSuccess;
  const dim3 grid((unsigned)B, (unsigned)levels);
  if (k.method == kThrSure) {
    int npow2 = 1;
    while (npow2 < k.n) npow2 <<= 1;
    const int lds = npow2 * (int)sizeof(unsigned long long);
    static LdsOnce configured;  // (this kernel also has static LDS: raise the limit to what it asks)
    hipError_t e = set_lds(k_sure_threshold, lds, &configured, lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_sure_threshold, grid, dim3(kSureThreads), lds, st, coeffs, level_stride, sigma, k, B, thr);
  } else {
    hipLaunchKernelGGL(k_level_threshold, grid, dim3(64), 0, st, coeffs, level_stride, sigma, k, B, thr);
  }
  return hipGetLastError();
}

template <typename T>
hipError_t launch_threshold(T* c, long long B, long long N, const T* thr, int soft, hipStream_t st) {
  const long long total = B * N;
  const unsigned grid = (unsigned)std::min<long long>((total + 255) / 256, 65536);
  hipLaunchKernelGGL(k_threshold<T>, dim3(grid), dim3(256), 0, st, c, B, N, thr, soft);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_fill_uniform(T* x, long long count, unsigned long long seed, long long offset, hipStream_t st) {
  const unsigned grid = (unsigned)std::min<long long>((count + 255) / 256, 65536);
  hipLaunchKernelGGL(k_fill_uniform<T>, dim3(grid), dim3(256), 0, st, x, count, seed, offset);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_single_haar_batch(const T* x, long long ldx, long long B, int N, T* approx, T* detail,
                                    hipStream_t st) {
  const unsigned gx = (unsigned)std::min(std::max((N + 255) / 256, 1), 1024);
  hipLaunchKernelGGL(k_single_haar_batch<T>, dim3(gx, (unsigned)B), dim3(256), 0, st, x, ldx, N, approx, detail);
  return hipGetLastError();
}

// AoS <-> SoA layout change (BatchSIMDMODWT.convertToSoA / convertFromSoA, ext/extensions/modwt/
// BatchSIMDMODWT.java:282-308): out[c][r] = in[r][c] for a rows x cols matrix, through 64 x 64 LDS
// tiles (one padding column: conflict-free column reads), coalesced on both sides.  HBM-bound: 2 x
// sizeof(T) bytes per element.
constexpr int kTrTile = 64;
template <typename T>
__global__ void __launch_bounds__(256) k_transpose(const T* __restrict__ in, long long rows, long long cols,
                                                   T* __restrict__ out) {
  __shared__ T tile[kTrTile][kTrTile + 1];
  const long long r0 = (long long)blockIdx.y * kTrTile, c0 = (long long)blockIdx.x * kTrTile;
  const int tx = threadIdx.x & 63, ty = threadIdx.x >> 6;  // 64 x 4 threads
#pragma unroll
  for (int k = 0; k < kTrTile; k += 4) {
    const long long r = r0 + ty + k, c = c0 + tx;
    if (r < rows && c < cols) tile[ty + k][tx] = in[r * cols + c];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < kTrTile; k += 4) {
    const long long c = c0 + ty + k, r = r0 + tx;  // output row c, column r
    if (r < rows && c < cols) out[c * rows + r] = tile[tx][ty + k];
  }
}

template <typename T>
hipError_t launch_transpose(const T* in, long long rows, long long cols, T* out, hipStream_t st) {
  const dim3 grid((unsigned)((cols + kTrTile - 1) / kTrTile), (unsigned)((rows + kTrTile - 1) / kTrTile));
  if (grid.y > 65535u) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(k_transpose<T>, grid, dim3(256), 0, st, in, rows, cols, out);
  return hipGetLastError();
}

#define VW_INST(T)                                                                                              \
  template hipError_t launch_history_update<T>(const T*, long long, const T*, T*, long long, int, int,         \
                                               hipStream_t);                                                    \
  template hipError_t launch_threshold<T>(T*, long long, long long, const T*, int, hipStream_t);               \
  template hipError_t launch_fill_uniform<T>(T*, long long, unsigned long long, long long, hipStream_t);       \
  template hipError_t launch_single_haar_batch<T>(const T*, long long, long long, int, T*, T*, hipStream_t); \
  template hipError_t launch_transpose<T>(const T*, long long, long long, T*, hipStream_t);
VW_INST(double)
VW_INST(float)
#undef VW_INST

}  // namespace vw
