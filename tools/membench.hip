// membench.hip -- HBM ceilings for the MODWT traffic patterns on this GPU (calibration, not product).
//   fan-out : read 1 row, write 7 rows   (forward: x -> d_1..d_6, a_6)
//   fan-in  : read 7 rows, write 1 row   (inverse: a_6, d_6..d_1 -> y)
//   copy, read-only, write-only
// One workgroup per 4096-sample fp64 row, 16-byte accesses, like the fused kernels.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef double d2 __attribute__((ext_vector_type(2)));

__global__ void fanout(const double* __restrict__ x, double* __restrict__ out, int N, long long plane, int J) {
  const long long b = blockIdx.x;
  for (int w = threadIdx.x; w < N / 2; w += blockDim.x) {
    d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2*>(x + b * N) + w);
    for (int j = 0; j < J; ++j) {
      d2 o = v * (double)(j + 1);
      __builtin_nontemporal_store(o, reinterpret_cast<d2*>(out + j * plane + b * N) + w);
    }
  }
}

__global__ void fanin(const double* __restrict__ in, double* __restrict__ y, int N, long long plane, int J) {
  const long long b = blockIdx.x;
  for (int w = threadIdx.x; w < N / 2; w += blockDim.x) {
    d2 acc = {0, 0};
    for (int j = 0; j < J; ++j) acc += __builtin_nontemporal_load(reinterpret_cast<const d2*>(in + j * plane + b * N) + w);
    __builtin_nontemporal_store(acc, reinterpret_cast<d2*>(y + b * N) + w);
  }
}

__global__ void fill(double* __restrict__ y, long long n) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 2; i += (long long)gridDim.x * blockDim.x)
    __builtin_nontemporal_store(d2{1.0, 2.0}, reinterpret_cast<d2*>(y) + i);
}

__global__ void readsum(const double* __restrict__ x, double* out, long long n) {
  d2 acc = {0, 0};
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < n / 2; i += (long long)gridDim.x * blockDim.x)
    acc += __builtin_nontemporal_load(reinterpret_cast<const d2*>(x) + i);
  if (acc[0] == 12345.0) out[0] = acc[1];
}

int main() {
  const int B = 4096, N = 4096, J = 7;
  const long long plane = (long long)B * N;
  double *x, *o;
  // both buffers hold J = 7 planes; every pattern below stays inside them
  hipMalloc(&x, plane * 8 * J);
  hipMalloc(&o, plane * 8 * J);
  hipMemset(x, 0, plane * 8 * J);
  hipMemset(o, 0, plane * 8 * J);
  hipEvent_t a, bb;
  hipEventCreate(&a);
  hipEventCreate(&bb);
  auto timeit = [&](const char* name, double bytes, auto launch) {
    for (int i = 0; i < 3; ++i) launch();
    hipDeviceSynchronize();
    const int reps = 20;
    hipEventRecord(a);
    for (int i = 0; i < reps; ++i) launch();
    hipEventRecord(bb);
    hipEventSynchronize(bb);
    float ms = 0;
    hipEventElapsedTime(&ms, a, bb);
    ms /= reps;
    printf("{\"pattern\": \"%s\", \"ms\": %.4f, \"GBps\": %.1f}\n", name, ms, bytes / (ms * 1e-3) / 1e9);
  };
  for (int th : {256, 512}) {
    char nm[64];
    snprintf(nm, sizeof nm, "fanout 1->7 (threads %d)", th);
    timeit(nm, plane * 8.0 * 8, [&] { hipLaunchKernelGGL(fanout, dim3(B), dim3(th), 0, 0, x, o, N, plane, J); });
    snprintf(nm, sizeof nm, "fanin 7->1 (threads %d)", th);
    timeit(nm, plane * 8.0 * 8, [&] { hipLaunchKernelGGL(fanin, dim3(B), dim3(th), 0, 0, o, x, N, plane, J); });
  }
  timeit("copy-like fanout 1->1", plane * 8.0 * 2,
         [&] { hipLaunchKernelGGL(fanout, dim3(B), dim3(512), 0, 0, x, o, N, plane, 1); });
  timeit("write-only 7 planes", plane * 8.0 * 7, [&] { hipLaunchKernelGGL(fill, dim3(8192), dim3(256), 0, 0, o, plane * 7); });
  timeit("read-only 7 planes", plane * 8.0 * 7,
         [&] { hipLaunchKernelGGL(readsum, dim3(8192), dim3(256), 0, 0, o, x, plane * 7); });
  return 0;
}
