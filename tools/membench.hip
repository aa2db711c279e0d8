// membench.hip -- HBM ceilings for the MODWT traffic patterns on this GPU (calibration, not product).
//   fan-out : read 1 row, write 7 rows   (forward: x -> d_1..d_6, a_6)
//   fan-in  : read 7 rows, write 1 row   (inverse: a_6, d_6..d_1 -> y)
//   copy, read-only, write-only; nt vs default cache policy; vectors per thread
// One workgroup per 4096-sample fp64 row (like the fused kernels) unless noted.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

template <bool NT>
__device__ __forceinline__ void st(d2* p, d2 v) {
  if constexpr (NT) __builtin_nontemporal_store(v, p); else *p = v;
}
template <bool NT>
__device__ __forceinline__ d2 ld(const d2* p) {
  if constexpr (NT) return __builtin_nontemporal_load(p); else return *p;
}

// fan-out: each thread owns VPT vectors of the row (loaded up front), then writes them to J planes
template <bool NT, int VPT>
__global__ void fanout(const double* __restrict__ x, double* __restrict__ out, int N, long long plane, int J) {
  const long long b = blockIdx.x;
  const int nv = N / 2;
  d2 v[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int w = threadIdx.x + k * blockDim.x;
    v[k] = w < nv ? ld<true>(reinterpret_cast<const d2*>(x + b * N) + w) : d2{0, 0};
  }
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int w = threadIdx.x + k * blockDim.x;
      if (w < nv) st<NT>(reinterpret_cast<d2*>(out + j * plane + b * N) + w, v[k] * (double)(j + 1));
    }
  }
}

// fan-in: each thread sums J rows into VPT vectors (loads of one plane issued together)
template <bool NT, int VPT>
__global__ void fanin(const double* __restrict__ in, double* __restrict__ y, int N, long long plane, int J) {
  const long long b = blockIdx.x;
  const int nv = N / 2;
  d2 acc[VPT];
#pragma unroll
  for (int k = 0; k < VPT; ++k) acc[k] = d2{0, 0};
  for (int j = 0; j < J; ++j) {
#pragma unroll
    for (int k = 0; k < VPT; ++k) {
      const int w = min((int)threadIdx.x + k * (int)blockDim.x, nv - 1);
      acc[k] += ld<NT>(reinterpret_cast<const d2*>(in + j * plane + b * N) + w);
    }
  }
#pragma unroll
  for (int k = 0; k < VPT; ++k) {
    const int w = threadIdx.x + k * blockDim.x;
    if (w < nv) st<true>(reinterpret_cast<d2*>(y + b * N) + w, acc[k]);
  }
}

template <bool NT>
__global__ void fill(double* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 2; i += (long long)gridDim.x * blockDim.x)
    st<NT>(reinterpret_cast<d2*>(y) + i, d2{1.0, 2.0});
}

template <bool NT>
__global__ void readsum(const double* __restrict__ x, double* out, long long n) {
  d2 acc = {0, 0};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 2; i += (long long)gridDim.x * blockDim.x)
    acc += ld<NT>(reinterpret_cast<const d2*>(x) + i);
  if (acc[0] == 12345.0) out[0] = acc[1];
}

int main() {
  const int B = 4096, N = 4096, J = 7;
  const long long plane = (long long)B * N;
  const long long total = plane * J;  // elements in each buffer
  double *x, *o;
  // both buffers hold J = 7 planes; every pattern below stays inside them
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
  const double b8 = plane * 8.0 * 8;  // 1 + 7 planes
  timeit("fanout nt vpt4 t512", b8, [&] { hipLaunchKernelGGL((fanout<true, 4>), dim3(B), dim3(512), 0, 0, x, o, N, plane, J); });
  timeit("fanout def vpt4 t512", b8, [&] { hipLaunchKernelGGL((fanout<false, 4>), dim3(B), dim3(512), 0, 0, x, o, N, plane, J); });
  timeit("fanout nt vpt8 t256", b8, [&] { hipLaunchKernelGGL((fanout<true, 8>), dim3(B), dim3(256), 0, 0, x, o, N, plane, J); });
  timeit("fanout nt vpt2 t1024", b8, [&] { hipLaunchKernelGGL((fanout<true, 2>), dim3(B), dim3(1024), 0, 0, x, o, N, plane, J); });
  timeit("fanin nt vpt4 t512", b8, [&] { hipLaunchKernelGGL((fanin<true, 4>), dim3(B), dim3(512), 0, 0, o, x, N, plane, J); });
  timeit("fanin def vpt4 t512", b8, [&] { hipLaunchKernelGGL((fanin<false, 4>), dim3(B), dim3(512), 0, 0, o, x, N, plane, J); });
  timeit("fanin nt vpt8 t256", b8, [&] { hipLaunchKernelGGL((fanin<true, 8>), dim3(B), dim3(256), 0, 0, o, x, N, plane, J); });
  timeit("fanin nt vpt2 t1024", b8, [&] { hipLaunchKernelGGL((fanin<true, 2>), dim3(B), dim3(1024), 0, 0, o, x, N, plane, J); });
  timeit("write-only 7 planes nt", plane * 8.0 * 7,
         [&] { hipLaunchKernelGGL((fill<true>), dim3(8192), dim3(256), 0, 0, o, total); });
  timeit("write-only 7 planes def", plane * 8.0 * 7,
         [&] { hipLaunchKernelGGL((fill<false>), dim3(8192), dim3(256), 0, 0, o, total); });
  timeit("read-only 7 planes nt", plane * 8.0 * 7,
         [&] { hipLaunchKernelGGL((readsum<true>), dim3(8192), dim3(256), 0, 0, o, x, total); });
  timeit("read-only 7 planes def", plane * 8.0 * 7,
         [&] { hipLaunchKernelGGL((readsum<false>), dim3(8192), dim3(256), 0, 0, o, x, total); });
  timeit("copy 1->1 nt", plane * 8.0 * 2,
         [&] { hipLaunchKernelGGL((fanout<true, 4>), dim3(B), dim3(512), 0, 0, x, o, N, plane, 1); });
  hipFree(x);
  hipFree(o);
  return 0;
}
