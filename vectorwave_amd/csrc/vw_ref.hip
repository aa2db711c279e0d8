// vw_ref.hip -- the reference's own arithmetic for the rows that hold non-finite values, on the
// unvalidated callers (VW_FLAG_REF_NONFINITE, include/vectorwave_amd.h).
//
// The fast kernels read only the L non-zero taps of an upsampled filter.  For finite data that is
// exact (a zero tap adds +-0 to a sum that is never -0), but the reference multiplies every one of the
// L_j = (L-1)*2^(j-1)+1 taps, zeros included, and 0 * Inf = 0 * NaN = NaN.  Where a caller does not
// validate its input first --
//   BatchMODWT.multiLevelAoS -> BatchSIMDMODWT.generalBatchMODWTSoAWithScaledFilters
//                                 ext/extensions/modwt/BatchSIMDMODWT.java:384-424 (no finite check,
//                                 BatchMODWT.java:201-212)
//   BatchMODWT.inverseMultiLevelAoS -> MultiLevelMODWTTransform.reconstruct (K4, :339-349, :576-589)
//   VectorWaveSwtAdapter.forwardParallel  core/swt/VectorWaveSwtAdapter.java:210-335 (N >= 4096, J > 2)
//   VectorWaveSwtAdapter.inverse / reconstructPeriodic  :435-487, and core reconstruct K5 / K6 :590-642
//   BatchStreamingMODWT ZERO / SYMMETRIC blocks -> BatchSIMDMODWT
//                                 .generalBatchMODWTSoAWithScaledFiltersAndHistory :447-507 (and its flush)
// -- a non-finite sample turns every output whose window reaches it through a zero tap into NaN.
// The engine keeps its fast kernels for every row and then recomputes, with the reference's loops
// (every tap, zeros included, separate multiply and add in the reference's order: bit-identical to it,
// NaN and +-Inf included), exactly the rows whose results can differ: those where some level input --
// x or an intermediate approximation in the forward; a_J, a kept d_j or an intermediate approximation in
// the inverse; a streaming history -- holds a NaN / +-Inf.  Such a value reaches the final output of the
// cascade through the non-zero taps (every filter's end taps are non-zero, and a sum with a non-finite
// term never turns finite), so one look at the final output finds them: a_J of the forward, y of the
// inverse -- in registers by the kernels that write it (FwdArgs / InvArgs nf_flag: v * 0 + z is NaN iff
// v is not finite, one FMA per value), else by k_flag_nonfinite over that one plane.  (A finite row that
// overflows to Inf there is recomputed too: harmless.)  Flagged rows are rare (they are invalid input to
// every validated entry point), so the fix-up is one persistent launch of one workgroup per row, reading
// the level input from global memory (L2).  Flags stay zero between calls: these kernels clear every row
// they recompute.
#include <hip/hip_runtime.h>
#include "vw_internal.h"

#pragma clang fp contract(off)

namespace vw {

// MathUtils.symmetricBoundaryExtension  core/util/MathUtils.java:30-51
__device__ __forceinline__ int ref_sym(int idx, int n) {
  if (idx >= 0 && idx < n) return idx;
  const int period = 2 * n;
  idx = ((idx % period) + period) % period;
  if (idx >= n) idx = period - idx - 1;
  return idx;
}

// MutableMultiLevelMODWTResult.applyThresholdToArray  core/modwt/MutableMultiLevelMODWTResult.java:97-114
template <typename T>
__device__ __forceinline__ T ref_threshold(T c, T thr, int soft) {
  const T av = c < T(0) ? -c : c;  // Math.abs
  if (soft) {
    if (av > thr) {
      const T sg = c > T(0) ? T(1) : (c < T(0) ? T(-1) : c);  // Math.signum
      return sg * (av - thr);
    }
    return T(0);
  }
  return av <= thr ? T(0) : c;
}

// flag[b] = 1 when row b of any plane holds a NaN or +-Inf.  One workgroup per (row, 4096-element chunk).
constexpr int kScanThreads = 256;
constexpr int kScanChunk = 4096;
template <typename T>
__global__ void __launch_bounds__(kScanThreads) k_flag_nonfinite(RefScan<T> a) {
  const long long b = blockIdx.x / a.chunks;
  const int c0 = (int)(blockIdx.x % a.chunks) * kScanChunk;
  const int c1 = min(a.N, c0 + kScanChunk);
  bool bad = false;
  for (int p = 0; p < a.np; ++p) {
    const T* row = a.p[p] + b * a.ld[p];
    const int e = min(c1, a.len[p] ? a.len[p] : a.N);
    for (int i = c0 + (int)threadIdx.x; i < e; i += kScanThreads) bad |= !__builtin_isfinite(row[i]);
  }
  // one store per wave that saw one (a plain vector store: every writer stores the same 1)
  if (__any(bad) && (threadIdx.x & 63) == 0) a.flag[b] = 1;
}

// Forward cascade of one flagged row, the reference's loop per level (level input from global memory):
//   PERIODIC  idx = t - l, if idx < 0: ((idx % n) + n) % n        forwardParallel :282-300 (== K7's
//             (t - l + N) % N wherever BatchSIMDMODWT can run, L_j <= N + 1)
//   ZERO      terms with idx < 0 skipped                            convolveZeroPadChunk :303-318
//   SYMMETRIC idx mirrored                                          convolveSymmetricChunk :321-335
//   history   idx < 0 reads the level's history at hl + idx        BatchSIMDMODWT
//             (BatchStreamingMODWT blocks)                          .generalBatchMODWTSoAWithScaledFiltersAndHistory
//                                                                   :447-507; history initialised / updated as
//                                                                   BatchStreamingMODWT :131-147, :326-352
// a += f_lo[l] * x[idx], d += f_hi[l] * x[idx], l = 0 .. L_j - 1 ascending, f[l] = 0 off the 2^(j-1) grid.
template <typename T>
__global__ void __launch_bounds__(512) k_ref_forward(RefArgs<T> a) {
  const int N = a.N;
  T* s0 = a.scratch + (size_t)blockIdx.x * 2 * (size_t)N;
  T* s1 = s0 + N;
  for (long long b = blockIdx.x; b < a.B; b += gridDim.x) {
    if (!a.flag[b]) continue;
    const T* cur = a.x + b * a.ldx;
    for (int j = 1; j <= a.J; ++j) {
      const int s = 1 << (j - 1);
      T* out_a = (j == a.J) ? a.approx + b * (long long)N : ((j & 1) ? s0 : s1);
      T* out_d = a.details + ((size_t)(j - 1) * (size_t)a.B + (size_t)b) * (size_t)N;
      const int hl = a.hist_mode ? a.hist_len[j - 1] : 0;
      const T* ho = (a.hist_mode && !a.hist_first) ? a.hist_old[j - 1] + b * (long long)hl : nullptr;
      // history position p (sample p - hl of the stream): the snapshot, or the one the first block creates
      auto hist = [&](int p) -> T {
        if (ho) return ho[p];
        return a.mode == kHaloZero ? T(0) : cur[ref_sym(p - hl, N)];  // fillSymmetricHistoryFromSoA :326-335
      };
      for (int t = threadIdx.x; t < N; t += blockDim.x) {
        T sa = T(0), sd = T(0);
        for (int i = 0; i < a.L; ++i) {
          const int reps = (i < a.L - 1) ? s : 1;  // the zeros between tap i and tap i + 1
          for (int r = 0; r < reps; ++r) {
            const int l = i * s + r;
            int idx = t - l;
            T v;
            if (idx >= 0) {
              v = cur[idx];
            } else if (a.hist_mode) {
              v = hist(hl + idx);
            } else {
              if (a.mode == kHaloZero) continue;
              idx = a.mode == kHaloSymmetric ? ref_sym(idx, N) : ((idx % N) + N) % N;
              v = cur[idx];
            }
            const T fl = r == 0 ? a.lo[i] : T(0), fh = r == 0 ? a.hi[i] : T(0);
            sa = sa + fl * v;
            sd = sd + fh * v;
          }
        }
        out_a[t] = sa;
        out_d[t] = sd;
      }
      // updateHistoryFromSoA :337-352: the last hl samples of the level input, or (n < hl) the old
      // history shifted by n followed by the whole input
      if (a.hist_mode && a.hist_new[j - 1]) {
        T* hn = a.hist_new[j - 1] + b * (long long)hl;
        for (int p = threadIdx.x; p < hl; p += blockDim.x)
          hn[p] = N >= hl ? cur[N - hl + p] : (p < hl - N ? hist(p + N) : cur[p - (hl - N)]);
      }
      __syncthreads();  // the level's approximation is the next level's input (same workgroup, same CU)
      cur = out_a;
    }
    if (threadIdx.x == 0) a.flag[b] = 0;  // read by every thread before the levels' barriers
  }
}

// Inverse cascade of one flagged row, levels J .. 1 (MultiLevelMODWTTransform.applyScaledInverseMODWT
// :554-645; VectorWaveSwtAdapter.reconstructPeriodic :444-474).  Per level j with a = running
// approximation, d = thresholded d_j (or the zero row of a masked level):
//   PERIODIC  sum += h[l] * a[(t + l) % n] for every l, then sum += g[l] * d[(t + l) % n]  (K4)
//   ZERO      for l with t + l < n: sum += h[l] * a[t + l] + g[l] * d[t + l]            (K5, pairwise)
//   SYMMETRIC approx branch idx = t + dir_a*l + off_a, detail branch t + dir_d*l + off_d, mirrored (K6)
template <typename T>
__global__ void __launch_bounds__(512) k_ref_inverse(RefArgs<T> a) {
  const int N = a.N;
  T* s0 = a.scratch + (size_t)blockIdx.x * 2 * (size_t)N;
  T* s1 = s0 + N;
  for (long long b = blockIdx.x; b < a.B; b += gridDim.x) {
    if (!a.flag[b]) continue;
    const T* cur = a.x ? a.x + b * (long long)N : nullptr;  // nullptr: zero approximation
    for (int j = a.J; j >= 1; --j) {
      const LevelDesc& lv = a.lv[j - 1];
      const int s = 1 << (j - 1);
      const T* d = lv.use_d ? a.det_in + ((size_t)(j - 1) * (size_t)a.B + (size_t)b) * (size_t)N : nullptr;
      const T th = a.thr ? a.thr[(size_t)(j - 1) * (size_t)a.thr_ld + (size_t)b] : T(0);
      auto dval = [&](int idx) {
        if (!d) return T(0);
        const T v = d[idx];
        return a.thr ? ref_threshold(v, th, a.soft) : v;
      };
      auto aval = [&](int idx) { return cur ? cur[idx] : T(0); };
      T* out = (j == 1) ? a.y + b * (long long)N : ((j & 1) ? s0 : s1);
      for (int t = threadIdx.x; t < N; t += blockDim.x) {
        T sum = T(0);
        if (a.mode == kHaloZero) {
          for (int i = 0; i < a.L; ++i) {
            const int reps = (i < a.L - 1) ? s : 1;
            for (int r = 0; r < reps; ++r) {
              const int idx = t + i * s + r;
              if (idx >= N) continue;
              const T h = r == 0 ? a.lo[i] : T(0), g = r == 0 ? a.hi[i] : T(0);
              sum = sum + (h * aval(idx) + g * dval(idx));
            }
          }
        } else {
          for (int br = 0; br < 2; ++br) {
            const T* f = br == 0 ? a.lo : a.hi;
            const int dir = br == 0 ? lv.dir_a : lv.dir_d, off = br == 0 ? lv.off_a : lv.off_d;
            for (int i = 0; i < a.L; ++i) {
              const int reps = (i < a.L - 1) ? s : 1;
              for (int r = 0; r < reps; ++r) {
                const int l = i * s + r;
                int idx;
                if (a.mode == kHaloSymmetric) idx = ref_sym(t + dir * l + off, N);
                else idx = (int)(((long long)t + l) % N);
                const T v = br == 0 ? aval(idx) : dval(idx);
                sum = sum + (r == 0 ? f[i] : T(0)) * v;
              }
            }
          }
        }
        out[t] = sum;
      }
      __syncthreads();
      cur = out;
    }
    if (threadIdx.x == 0) a.flag[b] = 0;
  }
}

template <typename T>
hipError_t launch_flag_nonfinite(const RefScan<T>& a, hipStream_t st) {
  const long long grid = a.B * (long long)a.chunks;
  if (grid <= 0) return hipSuccess;
  if (grid > 0x7fffffffLL) return hipErrorInvalidConfiguration;
  hipLaunchKernelGGL(k_flag_nonfinite<T>, dim3((unsigned)grid), dim3(kScanThreads), 0, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_ref_cascade(const RefArgs<T>& a, int grid, bool inverse, hipStream_t st) {
  if (inverse) hipLaunchKernelGGL(k_ref_inverse<T>, dim3((unsigned)grid), dim3(512), 0, st, a);
  else hipLaunchKernelGGL(k_ref_forward<T>, dim3((unsigned)grid), dim3(512), 0, st, a);
  return hipGetLastError();
}

int ref_scan_chunks(int N) { return (N + kScanChunk - 1) / kScanChunk; }

template hipError_t launch_flag_nonfinite<double>(const RefScan<double>&, hipStream_t);
template hipError_t launch_flag_nonfinite<float>(const RefScan<float>&, hipStream_t);
template hipError_t launch_ref_cascade<double>(const RefArgs<double>&, int, bool, hipStream_t);
template hipError_t launch_ref_cascade<float>(const RefArgs<float>&, int, bool, hipStream_t);

}  // namespace vw
