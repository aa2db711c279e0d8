// vw_sigma.h -- per-signal noise estimate for the SWT denoise path (included by vw_misc.hip only).
#pragma once
#include "vw_device.h"

namespace vw {

// ---------------------------------------------------------------------------------------------
// VectorWaveSwtAdapter.estimateNoiseSigma (:627-645): exact median of |c| by MSB-first radix
// selection on the IEEE bit patterns (non-negative doubles order as unsigned integers), then
// sigma = median / 0.6745 and the universal threshold T = sigma * sqrt(2 ln N) (:514).
constexpr int kSigmaThreads = 1024;
constexpr int kSigmaKeys = 16;

__device__ __forceinline__ unsigned long long abs_bits(double v) {
  return (unsigned long long)__double_as_longlong(v) & 0x7FFFFFFFFFFFFFFFull;
}

// Exact order statistics k1 = (N even ? N/2 - 1 : N/2) and k2 = N/2 of |c| by MSB-first radix selection (8-bit
// digits).  Robust for any distribution (ties, zeros, non-finite values: NaN orders above +Inf as in
// Arrays.sort), but a digit shared by most keys (the exponent byte) makes every key add into one LDS bin.
__device__ __forceinline__ void radix_median(const double* __restrict__ c, int N, const unsigned long long (&keys)[kSigmaKeys],
                                          bool in_regs, double* v1_out, double* v2_out) {
  __shared__ unsigned int hist[2][256];
  __shared__ unsigned int wsum[2][kSigmaThreads / 64];
  __shared__ unsigned long long prefix[2];
  __shared__ long long krem[2];
  const int tid = threadIdx.x;
  const int nsel = (N % 2 == 0) ? 2 : 1;
  if (tid == 0) {
    prefix[0] = prefix[1] = 0ull;
    krem[0] = (N % 2 == 0) ? N / 2 - 1 : N / 2;
    krem[1] = N / 2;
  }
  for (int shift = 56; shift >= 0; shift -= 8) {
    for (int q = tid; q < 512; q += kSigmaThreads) hist[q >> 8][q & 255] = 0u;
    lds_barrier();
    const unsigned long long hm = (shift == 56) ? 0ull : (~0ull << (shift + 8));
    const unsigned long long p0 = prefix[0], p1 = prefix[1];
    if (in_regs) {
#pragma unroll
      for (int k = 0; k < kSigmaKeys; ++k) {
        const int i = tid + k * kSigmaThreads;
        if (i < N) {
          const unsigned long long key = keys[k];
          const unsigned d = (unsigned)(key >> shift) & 255u;
          if (((key ^ p0) & hm) == 0) atomicAdd(&hist[0][d], 1u);
          if (nsel == 2 && ((key ^ p1) & hm) == 0) atomicAdd(&hist[1][d], 1u);
        }
      }
    } else {
      for (int i = tid; i < N; i += kSigmaThreads) {
        const unsigned long long key = abs_bits(c[i]);
        const unsigned d = (unsigned)(key >> shift) & 255u;
        if (((key ^ p0) & hm) == 0) atomicAdd(&hist[0][d], 1u);
        if (nsel == 2 && ((key ^ p1) & hm) == 0) atomicAdd(&hist[1][d], 1u);
      }
    }
    lds_barrier();
    // exclusive scan of 2 x 256 bins by threads 0..511 (wave-level shuffles)
    const int r = tid >> 8, bin = tid & 255, lane = tid & 63, wv = (tid >> 6) & 3;
    unsigned incl = 0;
    if (tid < 512) {
      const unsigned h = hist[r][bin];
      incl = h;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (lane == 63) wsum[r][wv] = incl;
    }
    lds_barrier();
    if (tid < 512 && r < nsel) {
      unsigned base = 0;
      for (int q = 0; q < wv; ++q) base += wsum[r][q];
      const unsigned h = hist[r][bin];
      const unsigned long long excl = (unsigned long long)(base + incl - h);
      const long long k = krem[r];
      if ((long long)excl <= k && k < (long long)(excl + h)) {
        prefix[r] |= ((unsigned long long)bin) << shift;
        krem[r] = k - (long long)excl;
      }
    }
    lds_barrier();
  }
  *v1_out = __longlong_as_double((long long)prefix[0]);
  *v2_out = __longlong_as_double((long long)prefix[1]);
}

// Block-wide min / max over 1024 threads (16 waves): wave butterflies, then the 16 partials via LDS.
__device__ __forceinline__ double block_minmax(double v, bool is_max, double* red) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    const double t = __shfl_xor(v, o, 64);
    v = is_max ? (t > v ? t : v) : (t < v ? t : v);
  }
  lds_barrier();  // red[] free (previous use complete)
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  lds_barrier();
  double r = red[0];
#pragma unroll
  for (int q = 1; q < kSigmaThreads / 64; ++q) r = is_max ? (red[q] > r ? red[q] : r) : (red[q] < r ? red[q] : r);
  return r;
}

constexpr int kSelBins = 2048;  // value buckets per refinement pass
constexpr int kSelCand = 1024;  // a bucket this small is finished by exact ranking (one candidate per thread)

// VectorWaveSwtAdapter.estimateNoiseSigma (:627-645) for N <= 16384, keys held in registers.
// Selection by value-range refinement: bucket(v) = min(B-1, floor((v - lo) * B / (hi - lo))) is monotone
// in v, so the keys of one bucket form a contiguous value interval; the bucket holding rank k is either
// small (its keys are ranked exactly, in LDS) or becomes the next [lo, hi].  Two ranks in adjacent
// buckets are the max of the first and the min of the second.  The result is the exact order statistic
// (the same as sorting); anything unusual (non-finite keys, a range too narrow to scale, no
// convergence in 6 passes) falls back to radix_median.  Two histogram atomics per key per pass on a
// spread-out digit, instead of eight radix passes whose first digits every key shares.
// center (optional, [B]): the keys are |c - center[b]| (MathUtils.medianAbsoluteDeviation's second
// pass; N <= 16384, keys in registers); median_out (optional): the raw median.
// One row b: keys from ck, fallback re-reads from c (both the row in HBM).  The barriers wait for LDS only
// (lds_barrier): nothing here reads global memory a barrier must order.  (A persistent form that copied the
// next row into LDS by DMA during the selection measured slower: profiles/r03/ab_sigma_pf_blkfwd8.log.)
__device__ __forceinline__ void noise_sigma_row(long long b, const double* __restrict__ c, const double* ck, bool vec,
                                                int N, double scale_c, double* sigma_out, double* thr_out,
                                                const double* __restrict__ center, double* median_out) {
  __shared__ int bad_any;
  __shared__ unsigned int hist[kSelBins];
  __shared__ double cand[kSelCand];
  __shared__ double red[kSigmaThreads / 64];
  __shared__ unsigned int wsum[kSigmaThreads / 64];
  __shared__ long long sel[2][3];  // per rank: bucket, exclusive count, count
  __shared__ double res[2];
  __shared__ int ncand;
  const int tid = threadIdx.x;
  const bool in_regs = N <= kSigmaThreads * kSigmaKeys;
  const double ctr = center ? center[b] : 0.0;
  auto key_of = [&](double v) { return abs_bits(center ? v - ctr : v); };
  const long long k1 = (N % 2 == 0) ? N / 2 - 1 : N / 2, k2 = N / 2;
  unsigned long long keys[kSigmaKeys];
  double v1 = 0.0, v2 = 0.0;
  bool done = false;
  if (in_regs) {
    if (vec) {
      typedef double d2 __attribute__((ext_vector_type(2)));
#pragma unroll
      for (int k = 0; k < kSigmaKeys / 2; ++k) {
        const int w = min(tid + k * kSigmaThreads, N / 2 - 1);
        const d2 v = __builtin_nontemporal_load(reinterpret_cast<const d2*>(ck) + w);
        keys[2 * k] = key_of(v[0]);
        keys[2 * k + 1] = key_of(v[1]);
      }
    } else {
#pragma unroll
      for (int k = 0; k < kSigmaKeys / 2; ++k) {
        const int i = 2 * (tid + k * kSigmaThreads);
        keys[2 * k] = i < N ? key_of(ck[i]) : 0ull;
        keys[2 * k + 1] = i + 1 < N ? key_of(ck[i + 1]) : 0ull;
      }
    }
    // key slot 2k+e holds element 2*(tid + k*1024) + e
    auto valid = [&](int q) { return 2 * (tid + (q >> 1) * kSigmaThreads) + (q & 1) < N; };
    auto val = [&](int q) { return __longlong_as_double((long long)keys[q]); };
    bool bad = false;
    double lo = __builtin_inf(), hi = -__builtin_inf();
#pragma unroll
    for (int q = 0; q < kSigmaKeys; ++q) {
      if (valid(q)) {
        const double v = val(q);
        bad |= !__builtin_isfinite(v);
        lo = v < lo ? v : lo;
        hi = v > hi ? v : hi;
      }
    }
    if (tid == 0) bad_any = 0;
    lds_barrier();  // bad_any cleared
    if (bad) bad_any = 1;
    lds_barrier();
    bad = bad_any != 0;
    lo = block_minmax(lo, false, red);
    hi = block_minmax(hi, true, red);
    long long r1 = k1, r2 = k2;  // ranks within the active keys [lo, hi]
    for (int pass = 0; !bad && !done && pass < 6; ++pass) {
      if (!(lo < hi)) { v1 = v2 = lo; done = true; break; }  // every active key equal
      const double scale = (double)kSelBins / (hi - lo);
      if (!__builtin_isfinite(scale)) break;
      auto bucket = [&](double v) { return min(kSelBins - 1, (int)((v - lo) * scale)); };
      for (int q = tid; q < kSelBins; q += kSigmaThreads) hist[q] = 0u;
      lds_barrier();
#pragma unroll
      for (int q = 0; q < kSigmaKeys; ++q) {
        const double v = val(q);
        if (valid(q) && v >= lo && v <= hi) atomicAdd(&hist[bucket(v)], 1u);
      }
      lds_barrier();
      // scan: thread t owns bins 2t, 2t+1
      const unsigned h0 = hist[2 * tid], h1 = hist[2 * tid + 1];
      unsigned incl = h0 + h1;
      const int lane = tid & 63, wv = tid >> 6;
#pragma unroll
      for (int o = 1; o < 64; o <<= 1) {
        const unsigned t = __shfl_up(incl, o, 64);
        if (lane >= o) incl += t;
      }
      if (lane == 63) wsum[wv] = incl;
      lds_barrier();
      unsigned base = 0;
      for (int q = 0; q < wv; ++q) base += wsum[q];
      const long long e0 = (long long)(base + incl - h0 - h1), e1 = e0 + h0;
#pragma unroll
      for (int r = 0; r < 2; ++r) {
        const long long rk = r ? r2 : r1;
        if (e0 <= rk && rk < e1) { sel[r][0] = 2 * tid; sel[r][1] = e0; sel[r][2] = h0; }
        if (e1 <= rk && rk < e1 + h1) { sel[r][0] = 2 * tid + 1; sel[r][1] = e1; sel[r][2] = h1; }
      }
      if (tid == 0) ncand = 0;
      lds_barrier();
      const int b1 = (int)sel[0][0], b2 = (int)sel[1][0];
      const long long ex1 = sel[0][1], cnt1 = sel[0][2];
      auto in_bucket = [&](int q, int bk) {
        const double v = val(q);
        return valid(q) && v >= lo && v <= hi && bucket(v) == bk;
      };
      if (b1 != b2) {  // r2 = r1 + 1: the last key of bucket b1 and the first of bucket b2
        double m1 = -__builtin_inf(), m2 = __builtin_inf();
#pragma unroll
        for (int q = 0; q < kSigmaKeys; ++q) {
          const double v = val(q);
          if (in_bucket(q, b1)) m1 = v > m1 ? v : m1;
          if (in_bucket(q, b2)) m2 = v < m2 ? v : m2;
        }
        v1 = block_minmax(m1, true, red);
        v2 = block_minmax(m2, false, red);
        done = true;
        break;
      }
      if (cnt1 <= kSelCand) {  // exact ranks inside the bucket
#pragma unroll
        for (int q = 0; q < kSigmaKeys; ++q)
          if (in_bucket(q, b1)) cand[atomicAdd(&ncand, 1)] = val(q);
        lds_barrier();
        const int n = ncand;
        if (tid < n) {
          const double x = cand[tid];
          int lt = 0, le = 0;
          for (int j = 0; j < n; ++j) {
            const double y = cand[j];
            lt += y < x;
            le += y <= x;
          }
          if (lt <= r1 - ex1 && r1 - ex1 < le) res[0] = x;
          if (lt <= r2 - ex1 && r2 - ex1 < le) res[1] = x;
        }
        lds_barrier();
        v1 = res[0];
        v2 = res[1];
        done = true;
        break;
      }
      // refine: the next active range is bucket b1's [min, max]
      double m1 = __builtin_inf(), m2 = -__builtin_inf();
#pragma unroll
      for (int q = 0; q < kSigmaKeys; ++q) {
        const double v = val(q);
        if (in_bucket(q, b1)) { m1 = v < m1 ? v : m1; m2 = v > m2 ? v : m2; }
      }
      const double nlo = block_minmax(m1, false, red);
      const double nhi = block_minmax(m2, true, red);
      lo = nlo;
      hi = nhi;
      r1 -= ex1;
      r2 -= ex1;
    }
  }
  if (!done) {
    // radix fallback (also N > 16384): key slots hold element tid + k*1024 there
    if (in_regs) {
#pragma unroll
      for (int k = 0; k < kSigmaKeys; ++k) {
        const int i = tid + k * kSigmaThreads;
        keys[k] = i < N ? key_of(c[i]) : 0ull;
      }
    }
    radix_median(c, N, keys, in_regs, &v1, &v2);
  }
  if (tid == 0) {
    const double median = (N % 2 == 0) ? (v1 + v2) / 2.0 : v1;  // odd N: k1 = N/2
    const double sigma = median / 0.6745;
    if (sigma_out) sigma_out[b] = sigma;
    if (thr_out) thr_out[b] = sigma * scale_c;
    if (median_out) median_out[b] = median;
  }
}

__global__ void __launch_bounds__(kSigmaThreads) k_noise_sigma(const double* __restrict__ coeffs, long long ld, int N,
                                                               double scale_c, double* sigma_out, double* thr_out,
                                                               const double* __restrict__ center, double* median_out) {
  const long long b = blockIdx.x;
  const double* c = coeffs + b * ld;
  const bool vec = (N % 2 == 0) && (ld % 2 == 0) && ((reinterpret_cast<uintptr_t>(coeffs) & 15) == 0);
  noise_sigma_row(b, c, c, vec, N, scale_c, sigma_out, thr_out, center, median_out);
}

// MathUtils.standardDeviation (core/util/MathUtils.java:233-257): sequential sum -> mean, sequential
// sum of squared deviations, sqrt(ssd / (n - 1)).  One lane: the reference's summation order.
__global__ void k_seq_std(const double* __restrict__ x, int n, double* out) {
  if (threadIdx.x != 0 || blockIdx.x != 0) return;
  double sum = 0.0;
  for (int i = 0; i < n; ++i) sum += x[i];
  const double mean = sum / n;
  double ssd = 0.0;
  for (int i = 0; i < n; ++i) {
    const double d = x[i] - mean;
    ssd += d * d;
  }
  out[0] = __builtin_sqrt(ssd / (n - 1));
}

// window[(start + k) % wsize] = |src[idx[k]]|, k < count (distinct ring slots: count <= wsize).
__global__ void k_gather_abs(const double* __restrict__ src, const int* __restrict__ idx, int count,
                             double* window, int wsize, int start) {
  for (int k = blockIdx.x * blockDim.x + threadIdx.x; k < count; k += gridDim.x * blockDim.x) {
    const double v = src[idx[k]];
    window[(start + k) % wsize] = __builtin_fabs(v);  // Math.abs: clears the sign bit (-0.0 -> 0.0)
  }
}



// ---------------------------------------------------------------------------------------------
// WaveletDenoiser thresholds (core/denoising/WaveletDenoiser.java:394-549), one per (level, signal):
// grid (B, levels).  sigma[b] is the MAD estimate of d_1 (k_noise_sigma); level j uses
// sigma / Math.sqrt(1 << j) (:225; 1 for the single-level denoise).  Host-side constants (the logs,
// square roots) come from the host libm, as in the C restatement.
//
// UNIVERSAL / MINIMAX: closed forms.  BAYES: the reference's sequential mean and variance sums in
// coefficient order, by one lane (bit-identical; rows are independent, so many waves run at once).
__global__ void __launch_bounds__(64) k_level_threshold(const double* __restrict__ coeffs, long long level_stride,
                                                        const double* __restrict__ sigma, const DenoiseConsts k,
                                                        long long B, double* __restrict__ thr) {
  if (threadIdx.x != 0) return;
  const long long b = blockIdx.x;
  const int lev = blockIdx.y;
  const int n = k.n;
  const double sig = sigma[b] / k.level_scale[lev];
  double T = 0.0;
  if (k.method == kThrUniversal) {
    T = sig * k.univ_c;
  } else if (k.method == kThrMinimax) {  // :497-509
    if (n <= 32) T = 0;
    else if (n <= 64) T = sig * 0.3936 + 0.1829 * sig * k.log_n;
    else T = sig * (0.4745 + 0.1148 * k.log_n);
  } else if (k.method == kThrBayes) {  // :521-549
    const double* c = coeffs + (size_t)lev * (size_t)level_stride + (size_t)b * (size_t)n;
    const double sigma2 = sig * sig;
    double mean = 0.0;
    for (int i = 0; i < n; ++i) mean += c[i];
    mean /= n;
    double variance = 0.0;
    for (int i = 0; i < n; ++i) {
      const double diff = c[i] - mean;
      variance += diff * diff;
    }
    variance /= n;
    const double sigmaX2 = variance - sigma2 > 0.0 ? variance - sigma2 : 0.0;  // Math.max(0.0, .)
    const double sigmaX = __builtin_sqrt(sigmaX2 + 1e-10);                   // BAYES_EPSILON :62
    T = sigma2 / sigmaX;
  }
  thr[(size_t)lev * (size_t)B + (size_t)b] = T;
}

// SURE (calculateSUREThreshold :441-472 + calculateSURERisk :477-492).  The reference tries every
// sorted |c_k| as the threshold and evaluates the risk in O(n) each (O(n^2) per row), keeping the
// first minimum.  Here, one workgroup per (signal, level):
//   1. |c| bit patterns sorted in LDS (bitonic; non-negative doubles order as unsigned integers);
//   2. the risk of every distinct t = a_k from prefix sums (one pass, O(n)):
//        n * risk(t) = -n s^2 + sum_{a<=t} a^2 + sum_{a>t} (s^2 + (a - t)^2)
//      (ties share t and the same risk, so only the last index of each run is scored);
//   3. this approximation differs from the reference's sequential sum by at most a few n*eps*(s^2 +
//      max a^2) (both sides' rounding); every t within kSureTol of that bound of the minimum is a
//      candidate.  One candidate decides the threshold by itself; otherwise each candidate's risk is
//      re-evaluated exactly as the reference does (sequential sum in coefficient order, one lane per
//      candidate) and the smallest risk with the smallest t wins -- the reference's strict-< scan.
//   4. the result is capped at the universal threshold (:466-469).
// The threshold is therefore the reference's value bit for bit.  n <= kSureMaxN (LDS: the sorted keys).
constexpr int kSureThreads = 1024;
constexpr int kSureMaxChunks = kSureMaxN / kSureThreads;

__device__ __forceinline__ double sure_exact_risk(const double* __restrict__ c, int n, double t, double s2) {
  double risk = -n * s2;
  for (int i = 0; i < n; ++i) {
    const double x = c[i];
    const double a = __builtin_fabs(x);
    if (a <= t) risk += x * x;
    else risk += s2 + (a - t) * (a - t);
  }
  return risk / n;
}

// inclusive block scan of (x, y) over 1024 threads; returns the block totals
__device__ __forceinline__ void block_scan2(double& x, double& y, double* wx, double* wy, double* tx, double* ty) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const double px = __shfl_up(x, o, 64), py = __shfl_up(y, o, 64);
    if (lane >= o) { x += px; y += py; }
  }
  __syncthreads();  // wx / wy free
  if (lane == 63) { wx[wv] = x; wy[wv] = y; }
  __syncthreads();
  double bx = 0.0, by = 0.0, sx = 0.0, sy = 0.0;
  for (int q = 0; q < kSureThreads / 64; ++q) {
    if (q < wv) { bx += wx[q]; by += wy[q]; }
    sx += wx[q];
    sy += wy[q];
  }
  x += bx;
  y += by;
  *tx = sx;
  *ty = sy;
}

__global__ void __launch_bounds__(kSureThreads) k_sure_threshold(const double* __restrict__ coeffs, long long level_stride,
                                                                 const double* __restrict__ sigma, const DenoiseConsts k,
                                                                 long long B, double* __restrict__ thr) {
  extern __shared__ unsigned long long key[];
  __shared__ double wx[kSureThreads / 64], wy[kSureThreads / 64];
  __shared__ double red[kSureThreads / 64];
  __shared__ int ired[kSureThreads / 64];
  const int tid = threadIdx.x;
  const long long b = blockIdx.x;
  const int lev = blockIdx.y;
  const int n = k.n;
  const double* c = coeffs + (size_t)lev * (size_t)level_stride + (size_t)b * (size_t)n;
  const double sig = sigma[b] / k.level_scale[lev];
  const double s2 = sig * sig;
  int npow2 = 1;
  while (npow2 < n) npow2 <<= 1;
  for (int i = tid; i < npow2; i += kSureThreads) key[i] = i < n ? abs_bits(c[i]) : 0x7FF0000000000000ull;
  __syncthreads();
  for (int size = 2; size <= npow2; size <<= 1) {  // bitonic sort, ascending
    for (int stride = size >> 1; stride > 0; stride >>= 1) {
      for (int i = tid; i < npow2 / 2; i += kSureThreads) {
        const int lo = 2 * i - (i & (stride - 1));
        const int hi = lo + stride;
        const unsigned long long x = key[lo], y = key[hi];
        if ((x > y) == ((lo & size) == 0)) { key[lo] = y; key[hi] = x; }
      }
      __syncthreads();
    }
  }
  auto val = [&](int i) { return __longlong_as_double((long long)key[i]); };
  // totals
  double s1 = 0.0, sq = 0.0;
  for (int i = tid; i < n; i += kSureThreads) { const double a = val(i); s1 += a; sq += a * a; }
  double S1, S2;
  {
    double x = s1, y = sq;
    block_scan2(x, y, wx, wy, &S1, &S2);
  }
  const double amax = val(n - 1);
  const double tol = 32.0 * n * 2.220446049250313e-16 * (s2 + amax * amax);
  // approximate risk of every run's last index
  const int nch = (n + kSureThreads - 1) / kSureThreads;
  double risk[kSureMaxChunks];
  double c1 = 0.0, c2 = 0.0;
#pragma unroll
  for (int ch = 0; ch < kSureMaxChunks; ++ch) {
    risk[ch] = __builtin_inf();
    if (ch < nch) {
      const int kk = ch * kSureThreads + tid;
      const double a = kk < n ? val(kk) : 0.0;
      double p1 = a, p2 = a * a, t1, t2;
      block_scan2(p1, p2, wx, wy, &t1, &t2);
      p1 += c1;
      p2 += c2;
      c1 += t1;
      c2 += t2;
      if (kk < n && (kk == n - 1 || key[kk + 1] != key[kk])) {
        const double up = (double)(n - kk - 1);
        const double x = -n * s2 + p2 + up * s2 + (S2 - p2) - 2.0 * a * (S1 - p1) + up * a * a;
        risk[ch] = x / n;
      }
    }
  }
  // minimum approximate risk
  double m = __builtin_inf();
#pragma unroll
  for (int ch = 0; ch < kSureMaxChunks; ++ch) m = risk[ch] < m ? risk[ch] : m;
  m = block_minmax(m, false, red);
  // candidates
  int cnt = 0, first = 0x7FFFFFFF;
#pragma unroll
  for (int ch = 0; ch < kSureMaxChunks; ++ch)
    if (risk[ch] <= m + tol && risk[ch] < __builtin_inf()) { ++cnt; first = min(first, ch * kSureThreads + tid); }
  // count and (for a single candidate) its index
  int total = cnt;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) total += __shfl_xor(total, o, 64);
  __syncthreads();
  if ((tid & 63) == 0) ired[tid >> 6] = total;
  __syncthreads();
  total = 0;
  for (int q = 0; q < kSureThreads / 64; ++q) total += ired[q];
  int best_k = -1;
  if (total == 1) {
    best_k = (int)block_minmax((double)first, false, red);
  } else if (total > 1) {
    // exact risks of the candidates (a lane per candidate, chunk by chunk), then (risk, index) minimum
    double em = __builtin_inf();
    int ek = 0x7FFFFFFF;
#pragma unroll
    for (int ch = 0; ch < kSureMaxChunks; ++ch) {
      if (risk[ch] <= m + tol && risk[ch] < __builtin_inf()) {
        const int kk = ch * kSureThreads + tid;
        const double r = sure_exact_risk(c, n, val(kk), s2);
        if (r < em) { em = r; ek = kk; }  // kk ascends with ch: ties keep the smaller index
      }
    }
    const double emin = block_minmax(em, false, red);
    const double kd = em == emin ? (double)ek : 1e300;
    const double kmin = block_minmax(kd, false, red);
    best_k = kmin < 1e300 ? (int)kmin : -1;
  }
  if (tid == 0) {
    double best = best_k >= 0 ? val(best_k) : 0.0;
    const double universal = sig * k.univ_c;
    if (best > universal) best = universal;
    thr[(size_t)lev * (size_t)B + (size_t)b] = best;
  }
}

}  // namespace vw
