// mfmabench.hip -- issue rate of the Toeplitz MFMA pattern of vw_mfma.hip (calibration, not product).
// Per wave: R rounds of (2 tiles x KS = 12 k-steps x {lo, hi}) v_mfma_f32_16x16x4_f32, i.e. four independent
// accumulation chains; the B operand either from registers (pure issue) or read from LDS each round with
// the forward's s = 1 address pattern (ds_read_b32, base(n) = 16 n, reversed k).  Prints cycles per MFMA per
// SIMD and TFLOP/s; the guide's figure is 32 cycles (155 TF).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));
constexpr int KS = 12;

template <bool LDS>
__global__ void __launch_bounds__(256) k(float* out, int rounds, float seed) {
  __shared__ float X[9216];
  const int tid = threadIdx.x, lane = tid & 63, row = lane & 15, kk = lane >> 4, wave = tid >> 6;
  for (int i = tid; i < 9216; i += 256) X[i] = seed * (float)(i & 63);
  __syncthreads();
  float A[KS], Bv[2][KS];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    A[q] = seed + (float)(row + q);
    Bv[0][q] = seed * (float)(kk + q);
    Bv[1][q] = seed * (float)(kk - q);
  }
  f4 lo[2] = {}, hi[2] = {};
  for (int r = 0; r < rounds; ++r) {
    if constexpr (LDS) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int base = 1024 + 256 * ((wave * 2 + h + r) & 31) + 16 * row + 15 - kk;
#pragma unroll
        for (int q = 0; q < KS; ++q) Bv[h][q] = X[base - 4 * q];
      }
      __builtin_amdgcn_sched_barrier(0);
    }
#pragma unroll
    for (int q = 0; q < KS; ++q)
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        lo[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q], Bv[h][q], lo[h], 0, 0, 0);
        hi[h] = __builtin_amdgcn_mfma_f32_16x16x4f32(A[q] * 0.5f, Bv[h][q], hi[h], 0, 0, 0);
      }
  }
  f4 s = lo[0] + lo[1] + hi[0] + hi[1];
  if (s[0] + s[1] + s[2] + s[3] == 1234.5f) out[0] = s[0];
}

int main() {
  float* out;
  hipMalloc(&out, 16);
  hipEvent_t a, b;
  hipEventCreate(&a);
  hipEventCreate(&b);
  const int rounds = 2000;
  for (int wgs_per_cu : {1, 2, 4}) {
    for (int lds = 0; lds < 2; ++lds) {
      const int grid = 256 * wgs_per_cu;
      auto launch = [&] {
        if (lds) hipLaunchKernelGGL(k<true>, dim3(grid), dim3(256), 0, 0, out, rounds, 1e-3f);
        else hipLaunchKernelGGL(k<false>, dim3(grid), dim3(256), 0, 0, out, rounds, 1e-3f);
      };
      launch();
      hipDeviceSynchronize();
      hipEventRecord(a);
      launch();
      hipEventRecord(b);
      hipEventSynchronize(b);
      float ms = 0;
      hipEventElapsedTime(&ms, a, b);
      const double mfmas_per_simd = (double)rounds * 48 * wgs_per_cu;  // one wave per SIMD per workgroup
      const double cyc = ms * 1e-3 * 2.4e9 / mfmas_per_simd;
      const double tf = (double)grid * 4 * rounds * 48 * 2048 / (ms * 1e-3) / 1e12;
      printf("{\"wgs_per_cu\": %d, \"B_from\": \"%s\", \"ms\": %.3f, \"cycles_per_mfma_per_simd\": %.1f, \"TFLOPs\": %.1f}\n",
             wgs_per_cu, lds ? "LDS" : "registers", ms, cyc, tf);
    }
  }
  return 0;
}
