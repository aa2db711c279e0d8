// valubench.hip -- vector-ALU FMA issue rates on this GPU (calibration, not product): the compute
// roof of the long-filter configs (coif5 fp32: 60 FMA per sample per level and pass).
//   f32    : v_fma_f32 chains (one FMA per lane per instruction)
//   pk_f32 : v_pk_fma_f32 chains (two FMAs per lane per instruction)
//   f64    : v_fma_f64 chains
// Each lane runs ACC independent chains (enough to cover the FMA latency at W waves per SIMD), so
// the kernel is issue-bound.  Prints achieved TFLOP/s (2 flop per FMA).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f2 __attribute__((ext_vector_type(2)));

#define CHECK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP error %s at %d\n", hipGetErrorString(e_), __LINE__); return 1; } } while (0)

constexpr int ACC = 16;

template <typename T>
__global__ void __launch_bounds__(256) k_fma(T* out, int iters, T a, T b) {
  T acc[ACC];
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = T(threadIdx.x + i);
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) {
      // inline asm: the compiler would otherwise pair adjacent f32 chains into v_pk_fma_f32
      if constexpr (sizeof(T) == 4) asm volatile("v_fma_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
      else asm volatile("v_fma_f64 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(a), "v"(b));
    }
  }
  T s = T(0);
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

__global__ void __launch_bounds__(256) k_pk_fma(float* out, int iters, float a, float b) {
  f2 acc[ACC];
  const f2 va = {a, a}, vb = {b, b};
#pragma unroll
  for (int i = 0; i < ACC; ++i) acc[i] = f2{float(threadIdx.x + i), float(i)};
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int i = 0; i < ACC; ++i) asm volatile("v_pk_fma_f32 %0, %0, %1, %2" : "+v"(acc[i]) : "v"(va), "v"(vb));
  }
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < ACC; ++i) s += acc[i].x + acc[i].y;
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <typename K>
static int timeit(const char* name, K launch, double flop, int reps) {
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  launch();
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < reps; ++r) launch();
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms = 0.f;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double s = ms * 1e-3 / reps;
  printf("%-8s %8.3f ms  %7.1f TFLOP/s\n", name, s * 1e3, flop / s / 1e12);
  return 0;
}

int main() {
  int cus = 0;
  CHECK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  const int threads = 256, blocks = cus * 8;  // 8 waves per SIMD
  const int iters = 4096;
  void* out = nullptr;
  CHECK(hipMalloc(&out, (size_t)blocks * threads * sizeof(double)));
  const double lanes = (double)blocks * threads;
  const double fmas = lanes * iters * ACC;
  printf("CUs %d, %d workgroups x %d threads, %d chains x %d iterations per lane\n", cus, blocks, threads, ACC, iters);
  int rc = 0;
  rc |= timeit("f32", [&] { hipLaunchKernelGGL(k_fma<float>, dim3(blocks), dim3(threads), 0, 0, (float*)out, iters, 0.999f, 1e-3f); },
               2 * fmas, 5);
  rc |= timeit("pk_f32", [&] { hipLaunchKernelGGL(k_pk_fma, dim3(blocks), dim3(threads), 0, 0, (float*)out, iters, 0.999f, 1e-3f); },
               4 * fmas, 5);
  rc |= timeit("f64", [&] { hipLaunchKernelGGL(k_fma<double>, dim3(blocks), dim3(threads), 0, 0, (double*)out, iters, 0.999, 1e-3); },
               2 * fmas, 5);
  CHECK(hipFree(out));
  return rc;
}
