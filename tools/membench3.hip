// membench3.hip -- store-policy calibration for the forward's write-heavy pattern (calibration, not product).
// Questions: (1) does the store cache policy (default / nt / sc1 / sc0|sc1 / nt|sc1) change the HBM
// write ceiling of the 1 -> 7 rows fan-out?  (2) how long is the boundary to a dependent kernel after
// each policy (dirty L2 lines must be written back at the end of a kernel)?
// Buffer stores with an explicit aux field: 1 = sc0, 2 = nt, 16 = sc1.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d2 __attribute__((ext_vector_type(2)));
typedef int i4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

template <int AUX>
__device__ __forceinline__ void st(__amdgpu_buffer_rsrc_t r, int off, d2 v) {
  __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4, v), r, off, 0, AUX);
}

// fan-out: one WG per 4096-sample row: read x row (nt), write J rows of the [J][B][N] planes.
template <int AUX>
__global__ __launch_bounds__(512) void fanout(const double* __restrict__ x, double* __restrict__ out, int N,
                                              long long plane, int J) {
  const long long b = blockIdx.x;
  d2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(x + b * N) + threadIdx.x + k * 512);
  for (int j = 0; j < J; ++j) {
    const auto r = rsrc(out + j * plane + b * N);
#pragma unroll
    for (int k = 0; k < 4; ++k) st<AUX>(r, (threadIdx.x + k * 512) * 16, v[k] * (double)(j + 1));
  }
}

// fan-out shaped like k_forward_fused: dynamic LDS (occupancy), a workgroup barrier per plane, the
// plane's values round-tripped through LDS (the level ping-pong) when RT
template <int AUX, bool BAR, bool RT>
__global__ __launch_bounds__(512) void fanout_lvl(const double* __restrict__ x, double* __restrict__ out, int N,
                                                  long long plane, int J) {
  extern __shared__ d2 lds[];
  const long long b = blockIdx.x;
  d2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(x + b * N) + threadIdx.x + k * 512);
  for (int j = 0; j < J; ++j) {
    if (RT) {
#pragma unroll
      for (int k = 0; k < 4; ++k) lds[threadIdx.x + k * 512] = v[k];
    }
    if (BAR) { __builtin_amdgcn_s_waitcnt(0xC07F); __builtin_amdgcn_s_barrier(); }
    if (RT) {
#pragma unroll
      for (int k = 0; k < 4; ++k) v[k] = lds[(threadIdx.x + k * 512 + 1) & 2047] * 0.5 + v[k];
    }
    const auto r = rsrc(out + j * plane + b * N);
#pragma unroll
    for (int k = 0; k < 4; ++k) st<AUX>(r, (threadIdx.x + k * 512) * 16, v[k] * (double)(j + 1));
    if (BAR) { __builtin_amdgcn_s_waitcnt(0xC07F); __builtin_amdgcn_s_barrier(); }
  }
}

// fan-out, signal-major output layout [B][J][N] (each WG writes one contiguous 7-row block)
template <int AUX>
__global__ __launch_bounds__(512) void fanout_sm(const double* __restrict__ x, double* __restrict__ out, int N,
                                                 long long plane, int J) {
  const long long b = blockIdx.x;
  d2 v[4];
#pragma unroll
  for (int k = 0; k < 4; ++k)
    v[k] = __builtin_nontemporal_load(reinterpret_cast<const d2*>(x + b * N) + threadIdx.x + k * 512);
  for (int j = 0; j < J; ++j) {
    const auto r = rsrc(out + (b * J + j) * N);
#pragma unroll
    for (int k = 0; k < 4; ++k) st<AUX>(r, (threadIdx.x + k * 512) * 16, v[k] * (double)(j + 1));
  }
}

// write-only, one WG per row chunk of 32 KB, contiguous
template <int AUX>
__global__ __launch_bounds__(512) void fill_rows(double* __restrict__ y) {
  const auto r = rsrc(y + blockIdx.x * 4096ll);
#pragma unroll
  for (int k = 0; k < 4; ++k) st<AUX>(r, (threadIdx.x + k * 512) * 16, d2{1.0, 2.0});
}

// reader after writer: fan-in read of the 7 planes (to time the dependent boundary)
__global__ __launch_bounds__(512) void fanin(const double* __restrict__ in, double* __restrict__ y, int N,
                                             long long plane, int J) {
  const long long b = blockIdx.x;
  d2 acc[4] = {};
  for (int j = 0; j < J; ++j)
#pragma unroll
    for (int k = 0; k < 4; ++k)
      acc[k] += __builtin_nontemporal_load(reinterpret_cast<const d2*>(in + j * plane + b * N) + threadIdx.x + k * 512);
#pragma unroll
  for (int k = 0; k < 4; ++k)
    __builtin_nontemporal_store(acc[k], reinterpret_cast<d2*>(y + b * N) + threadIdx.x + k * 512);
}

int main() {
  const int B = 4096, N = 4096, J = 7;
  const long long plane = (long long)B * N;
  const long long total = plane * J;
  double *x, *o;
  if (hipMalloc(&x, total * 8) != hipSuccess || hipMalloc(&o, total * 8) != hipSuccess) return 1;
  hipMemset(x, 0, total * 8);
  hipMemset(o, 0, total * 8);
  hipEvent_t a, bb;
  hipEventCreate(&a);
  hipEventCreate(&bb);
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 5; ++i) launch();
    hipDeviceSynchronize();
    const int reps = 50;
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(bb);
    hipEventSynchronize(bb);
    float ms = 0;
    hipEventElapsedTime(&ms, a, bb);
    ms /= reps;
    printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
    fflush(stdout);
  };
  const double b8 = plane * 8.0 * 8;
  const double b7 = plane * 8.0 * 7;
#define FO(AUX)                                                                                           \
  timeit("fanout aux" #AUX, b8, [&] { hipLaunchKernelGGL((fanout<AUX>), dim3(B), dim3(512), 0, 0, x, o, N, plane, J); }); \
  timeit("fanout-sm aux" #AUX, b8, [&] { hipLaunchKernelGGL((fanout_sm<AUX>), dim3(B), dim3(512), 0, 0, x, o, N, plane, J); }); \
  timeit("fill aux" #AUX, b7, [&] { hipLaunchKernelGGL((fill_rows<AUX>), dim3(B * J), dim3(512), 0, 0, o); }); \
  timeit("fanout+fanin aux" #AUX, 2 * b8, [&] {                                                      \
    hipLaunchKernelGGL((fanout<AUX>), dim3(B), dim3(512), 0, 0, x, o, N, plane, J);                     \
    hipLaunchKernelGGL(fanin, dim3(B), dim3(512), 0, 0, o, x, N, plane, J);                             \
  });
  FO(0) FO(2) FO(16)
#define FL(AUX, BAR, RT, LDSB)                                                                              \
  timeit("fanout-lvl aux" #AUX " bar" #BAR " rt" #RT " lds" #LDSB, b8, [&] {                               \
    hipLaunchKernelGGL((fanout_lvl<AUX, BAR, RT>), dim3(B), dim3(512), LDSB, 0, x, o, N, plane, J); });
  hipFuncSetAttribute(reinterpret_cast<const void*>(fanout_lvl<2, true, true>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute(reinterpret_cast<const void*>(fanout_lvl<2, false, false>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  hipFuncSetAttribute(reinterpret_cast<const void*>(fanout_lvl<2, true, false>), hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
  FL(2, false, false, 0) FL(2, false, false, 34816) FL(2, false, false, 69632)
  FL(2, true, false, 0) FL(2, true, false, 34816) FL(2, true, false, 69632)
  FL(2, true, true, 34816) FL(2, true, true, 69632)
  timeit("fanin alone", b8, [&] { hipLaunchKernelGGL(fanin, dim3(B), dim3(512), 0, 0, o, x, N, plane, J); });
  hipFree(x);
  hipFree(o);
  return 0;
}
