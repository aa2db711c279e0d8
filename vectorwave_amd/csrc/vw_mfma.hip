// vw_mfma.hip -- the à-trous convolutions of the fp32 FMA path on the matrix cores (v_mfma_f32_16x16x4_f32).
//
// Why: the long-filter fp32 configuration (coif5, 30 taps, BASELINE config 5) is VALU-issue-bound, not
// HBM-bound (1,440 flop/sample against a 19.7 flop/B ridge; the VALU kernels issued 1.18
// instructions per FMA and shared the CU with their LDS reads).  The f32-input MFMA runs at the fp32 vector
// peak (MI355X guide: 155 TF measured) and holds the SIMD's vector issue for 8 of its 32 cycles, so the
// address arithmetic, LDS reads and stores run beside it.
//
// Formulation.  A level with spacing s is, in each residue class mod s, an ordinary convolution along the
// class coordinate u (sample t = r + s*u).  Sixteen consecutive class positions of a class form a column;
// sixteen columns form a 16 x 16 output tile O = T * X with
//   forward  out[t] = sum_i f[i] x[t - s*i]      T[m][k] = f[m + k - 15], X[k][n] = x[base(n) + s*(15 - k)]
//   inverse  y[t]   = sum_i h[i] a[t + s*i] (+) sum_i g[i] d[t + s*i]
//                                                T[m][k] = f[k - m],      X[k][n] = a[base(n) + s*k]
// (rows m, columns n, output t = base(n) + s*m; k = 0 .. 4*KS - 1, KS = ceil((L + 15) / 4) MFMA k-steps,
// T zero outside the band).  T depends only on the lane: it is held in registers for the whole kernel (A
// operand, one VGPR per k-step and filter); X is one ds_read_b32 per lane and k-step from the level row in
// LDS (B operand), shared by the low- and high-pass MFMAs of the forward.  The forward reads X backwards so
// that k ascends with the tap index: each output is then accumulated tap by tap in the reference's order
// (the inverse: the approximation branch's taps, then the detail branch's), one rounding per tap -- the
// VALU FMA kernels' sums.  Useful work: L / (4*KS) of the MFMA's (30 / 48 = 62.5 % for coif5).
//
// Columns: s < 16: n = c + s*b, base(n) = 256*tile + c + 16*s*b (c < s: 16/s blocks of 16 class positions
// in each of the s classes -- a tile is 256 consecutive samples); s >= 16: base(n) = 16*g + n + 16*s*cb (16
// consecutive residues of group g, class block cb).  Lane l holds O[4*(l>>4) + v][l & 15], v = 0..3.
//
// Scope: PERIODIC, fp32, VW_FLAG_FMA (EXACT keeps the VALU kernels: separate multiply and add), one signal
// per workgroup (NT threads, N = 4 * NT * TPW samples, TPW tiles per wave), every level's halo (4*KS - 16)*s
// within the row.  Host policy: vw_capi.cpp (VW_MFMA).
#include "vw_device.h"

namespace vw {

// D += A * B on the matrix core: 16 x 16 x 4, f32 in, f32 accumulate.
typedef float f4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ f4 mfma4(float a, float b, f4 c) { return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0); }

// base(n) of this lane's column in tile `tile` at spacing s (see the header)
__device__ __forceinline__ int mfma_base(int tile, int s, int n) {
  if (s < 16) {
    const int sh = __builtin_ctz(s);
    return 256 * tile + (n & (s - 1)) + 16 * s * (n >> sh);
  }
  const int G = s >> 4;  // residue groups of 16
  return 16 * (tile & (G - 1)) + n + 16 * s * (tile >> __builtin_ctz(G));
}

// Four outputs of a lane, t = base + s*(4*kk + v): one 16-byte store when they are consecutive.  Write-back
// policy: at s > 1 a lane's values are s apart and a wave writes pieces of every line -- L2 merges them
// before HBM (the VALU kernels' small-stride stores, profiles/hbm_traffic_coif5-f32.json).
__device__ __forceinline__ void store4(float* __restrict__ row, int t, int s, f4 v) {
  if (s == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(row + t));
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) row[t + e * s] = v[e];
  }
}

// A tile's four outputs per lane (t = base + s*(4*kk + v)) to a row: s = 1 one 16-byte store; 2 <= s < 16
// through the wave's scratch (sc, 256 floats) so that lane l stores samples 256*tile + 4l .. 4l+3; s >= 16
// four scattered stores (16 consecutive residues: 64-byte pieces).
__device__ __forceinline__ void put_tile(float* sc, int lane, float* __restrict__ row, int tile, int t, int s, f4 v) {
  if (s == 1) {
    __builtin_nontemporal_store(v, reinterpret_cast<f4*>(row + t));
  } else if (s < 16) {
    const int o = t - 256 * tile;
#pragma unroll
    for (int e = 0; e < 4; ++e) sc[o + e * s] = v[e];
    __builtin_amdgcn_wave_barrier();  // one wave's LDS accesses run in order; keep the compiler's order too
    const f4 w = *reinterpret_cast<const f4*>(sc + 4 * lane);
    __builtin_amdgcn_wave_barrier();
    __builtin_nontemporal_store(w, reinterpret_cast<f4*>(row + 256 * tile + 4 * lane));
  } else {
#pragma unroll
    for (int e = 0; e < 4; ++e) row[t + e * s] = v[e];
  }
}

// Workgroup: NT threads (NT / 64 waves of TPW tiles each, N = 4 * NT * TPW).  N = 8192 runs 512 threads of
// four tiles (the inverse's registers at eight tiles per wave -- its row prefetch alone is 2 x 32 VGPRs --
// left two waves per SIMD); VW_MFMA_NT8K=256 restores one workgroup of 256 threads x 8 tiles.
#ifndef VW_MFMA_NT8K
#define VW_MFMA_NT8K 512
#endif

// LDS layout: element i at slot ph(i) = i + (i >> S), one pad per 2^S elements (S = 3 by default).  The 16
// columns of a tile sit 16*s elements apart, i.e. on 2 of a half wave's 32 banks unpadded (8-way at s = 1, 2);
// padded, the modelled B reads are conflict-free at s <= 4 and 2-way above, and -- what keeps them one
// ds_read at an offset -- the slot distance ph(i0 -+ 4*s*q) - ph(i0) of k-step q is the same for every lane
// and tile of a level (dq below, computed once per level).
#ifndef VW_MFMA_PAD_SHIFT
#define VW_MFMA_PAD_SHIFT 3
#endif
__device__ __forceinline__ int ph(int i) { return i + (i >> VW_MFMA_PAD_SHIFT); }

// Forward, PERIODIC, fp32 FMA: all J levels of one signal per workgroup.  One LDS level buffer X: element t
// at X[H + t] for t in [-H, N) (left wrap images; H = p.hlpad >= (4*KS - 16) * s_J); taps at p.tap_lds.
// Per level: every tile of the wave computed (approximations kept in registers, details stored), barrier,
// approximations written back as the next level's input, barrier.  (Two level buffers -- write-back straight
// after each tile pair, one barrier per level -- measured slower: one 1024-thread workgroup per CU,
// profiles/r06/ab_coif5_mfma_v3_two_level_buffers.log.)
template <int L, int TPW, int NT>
__global__ void __launch_bounds__(NT) k_forward_mfma(const FwdArgs<float> p) {
  constexpr int KS = (L + 15 + 3) / 4;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* X = reinterpret_cast<float*>(smem);
  float* taps = reinterpret_cast<float*>(smem) + p.tap_lds;
  // per-wave transpose scratch (256 floats after the taps): at 2 <= s < 16 a tile is the 256 consecutive
  // samples [256*tile, +256) in the MFMA's lane order, four per lane s apart; through the scratch every lane
  // stores 16 contiguous bytes (whole lines) instead of four scattered floats
  float* const SC = reinterpret_cast<float*>(smem) + ((p.tap_lds + 2 * L + 3) & ~3) + 256 * (threadIdx.x >> 6);
  const int N = p.N, H = p.hlpad;
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kk = lane >> 4;
  const long long b = blockIdx.x;
  for (int i = tid; i < 2 * L; i += NT) taps[i] = i < L ? p.lo[i] : p.hi[i - L];
  {
    const f4* xr = reinterpret_cast<const f4*>(p.x + b * p.ldx);
    for (int w = tid; w < N / 4; w += NT) {
      const f4 v = __builtin_nontemporal_load(xr + w);
      const int o = ph(H + 4 * w);  // an aligned 4-group stays contiguous (pads fall between 8-groups)
#pragma unroll
      for (int e = 0; e < 4; ++e) X[o + e] = v[e];
      if (4 * w >= N - H) {
        const int oi = ph(H + 4 * w - N);
#pragma unroll
        for (int e = 0; e < 4; ++e) X[oi + e] = v[e];
      }
    }
  }
  __syncthreads();
  float Alo[KS], Ahi[KS];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int i = row + 4 * q + kk - 15;  // T[row][k] = f[row + k - 15]
    const bool in = i >= 0 && i < L;
    Alo[q] = in ? taps[i] : 0.f;
    Ahi[q] = in ? taps[L + i] : 0.f;
  }
  for (int j = 1; j <= p.J; ++j) {
    const int s = 1 << (j - 1);
    const bool last = j == p.J;
    const unsigned xb = lds_base(X);
    int dq[KS];  // slot distance of k-step q (lane- and tile-uniform)
    {
      const int r0 = H + mfma_base(0, s, 0) + 15 * s;
#pragma unroll
      for (int q = 0; q < KS; ++q) dq[q] = ph(r0 - 4 * s * q) - ph(r0);
    }
    float* dout = p.details + ((size_t)(j - 1) * (size_t)p.B + (size_t)b) * (size_t)N;
    float* aout = p.approx + b * (size_t)N;
    f4 keep[TPW];
    // two tiles at a time: their 2*KS B values read first (one wait), then four independent accumulation
    // chains (lo / hi of each tile) interleaved, so neither the LDS latency nor the MFMA's dependent-issue
    // latency is exposed
#pragma unroll
    for (int i = 0; i < TPW; i += 2) {
      int base[2];
      float xv[2][KS];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        base[h] = mfma_base(wave * TPW + i + h, s, row);
        // B operand of k-step q: X[k = 4q + kk][n] = x[base + s*(15 - 4q - kk)]
        const unsigned a0 = xb + 4u * (unsigned)ph(H + base[h] + s * (15 - kk));
#pragma unroll
        for (int q = 0; q < KS; ++q) xv[h][q] = lds_vec_at<float>(a0 + 4u * (unsigned)dq[q]);
      }
      __builtin_amdgcn_sched_barrier(0);
      f4 lo[2] = {}, hi[2] = {};
#pragma unroll
      for (int q = 0; q < KS; ++q)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          lo[h] = mfma4(Alo[q], xv[h][q], lo[h]);
          hi[h] = mfma4(Ahi[q], xv[h][q], hi[h]);
        }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const int t = base[h] + 4 * s * kk;  // this lane's outputs: t + s*v
        const int tile = wave * TPW + i + h;
        put_tile(SC, lane, dout, tile, t, s, hi[h]);
        if (last) put_tile(SC, lane, aout, tile, t, s, lo[h]);
        keep[i + h] = lo[h];
      }
    }
    if (last) break;
    __syncthreads();  // every read of this level's input done
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = mfma_base(wave * TPW + i, s, row) + 4 * s * kk;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int te = t + e * s;
        X[ph(H + te)] = keep[i][e];
        if (te >= N - H) X[ph(H + te - N)] = keep[i][e];
      }
    }
    __syncthreads();
  }
}

// Inverse, PERIODIC, sequential sums (K4: the approximation branch, then the detail branch, in one
// accumulator per output), fp32 FMA.  One LDS region R time-shared by a_j and d_j: element t at R[t] for t in
// [0, N + H) (right wrap images, H = p.hlpad_a >= (4*KS - 16) * s_J); the tiles' accumulators stay in
// registers across the swap; d_{j-1} is prefetched into registers while level j computes.
template <int L, int TPW, int NT>
__global__ void __launch_bounds__(NT) k_inverse_mfma(const InvArgs<float> p) {
  constexpr int KS = (L + 15 + 3) / 4;
  constexpr int RV = TPW;  // float4 row vectors per thread: N / 4 / 256 = TPW
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  float* R = reinterpret_cast<float*>(smem);
  float* taps = R + p.tap_lds;
  const int N = p.N;  // the right images reach (4*KS - 16)*s_j: p.hlpad_a covers level J
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int row = lane & 15, kk = lane >> 4;
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const size_t plane = (size_t)p.B * (size_t)N;
  const unsigned rb = lds_base(R);
  for (int i = tid; i < 2 * L; i += NT) taps[i] = i < L ? p.lo[i] : p.hi[i - L];
  // a row (standard mapping: vector tid + k*256) into R with the right images of the level's reach
  auto stage = [&](const f4 (&r)[RV], int reach, int mode, float thr) {
#pragma unroll
    for (int k = 0; k < RV; ++k) {
      const int t = 4 * (tid + k * NT);
      f4 v = r[k];
      if (mode == 1) v = f4{0.f, 0.f, 0.f, 0.f};
      if (mode == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = threshold_t(v[e], thr, p.soft);
      }
      const int o = ph(t);
#pragma unroll
      for (int e = 0; e < 4; ++e) R[o + e] = v[e];
      if (t < reach) {
        const int oi = ph(N + t);
#pragma unroll
        for (int e = 0; e < 4; ++e) R[oi + e] = v[e];
      }
    }
  };
  auto load = [&](f4 (&r)[RV], const float* src) {
#pragma unroll
    for (int k = 0; k < RV; ++k) r[k] = __builtin_nontemporal_load(reinterpret_cast<const f4*>(src) + tid + k * NT);
  };
  auto reach_of = [&](int j) { return (4 * KS - 16) << (j - 1); };
  auto thr_of = [&](int j) { return p.thr ? load_uniform(p.thr + (size_t)(j - 1) * (size_t)p.thr_ld + (size_t)b) : 0.f; };
  f4 rA[RV], rD[RV];
  if (!p.approx_zero) load(rA, p.approx + b * (size_t)N);
  if (p.lv[p.J - 1].use_d) load(rD, p.details + (size_t)(p.J - 1) * plane + b * (size_t)N);
  __syncthreads();  // taps
  float Alo[KS], Ahi[KS];
#pragma unroll
  for (int q = 0; q < KS; ++q) {
    const int i = 4 * q + kk - row;  // T[row][k] = f[k - row]
    const bool in = i >= 0 && i < L;
    Alo[q] = in ? taps[i] : 0.f;
    Ahi[q] = in ? taps[L + i] : 0.f;
  }
  stage(rA, reach_of(p.J), p.approx_zero ? 1 : 0, 0.f);
  for (int j = p.J; j >= 1; --j) {
    const int s = 1 << (j - 1);
    const LevelDesc& lv = p.lv[j - 1];
    int dq[KS];  // slot distance of k-step q (lane- and tile-uniform)
    {
      const int r0 = mfma_base(0, s, 0);
#pragma unroll
      for (int q = 0; q < KS; ++q) dq[q] = ph(r0 + 4 * s * q) - ph(r0);
    }
    __syncthreads();  // R = a_j + images
    f4 acc[TPW];
    // one branch over the wave's tiles, two at a time: B values first, then two interleaved chains
    auto branch = [&](const float (&A)[KS], bool first) __attribute__((always_inline)) {
#pragma unroll
      for (int i = 0; i < TPW; i += 2) {
        float xv[2][KS];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const unsigned a0 = rb + 4u * (unsigned)ph(mfma_base(wave * TPW + i + h, s, row) + s * kk);
#pragma unroll
          for (int q = 0; q < KS; ++q) xv[h][q] = lds_vec_at<float>(a0 + 4u * (unsigned)dq[q]);
        }
        __builtin_amdgcn_sched_barrier(0);
        f4 c[2];
#pragma unroll
        for (int h = 0; h < 2; ++h) c[h] = first ? f4{0.f, 0.f, 0.f, 0.f} : acc[i + h];
#pragma unroll
        for (int q = 0; q < KS; ++q)
#pragma unroll
          for (int h = 0; h < 2; ++h) c[h] = mfma4(A[q], xv[h][q], c[h]);
#pragma unroll
        for (int h = 0; h < 2; ++h) acc[i + h] = c[h];
      }
    };
    branch(Alo, true);
    __syncthreads();  // every approximation-branch read done
    stage(rD, reach_of(j), lv.use_d ? (p.thr ? 2 : 0) : 1, thr_of(j));
    if (j > 1 && p.lv[j - 2].use_d) load(rD, p.details + (size_t)(j - 2) * plane + b * (size_t)N);
    __syncthreads();  // R = d_j + images
    branch(Ahi, false);
    if (j == 1) {
#pragma unroll
      for (int i = 0; i < TPW; ++i)
        store4(p.y + b * (size_t)N, mfma_base(wave * TPW + i, s, row) + 4 * s * kk, s, acc[i]);
      break;
    }
    __syncthreads();  // every detail-branch read done
    const int reach = reach_of(j - 1);
#pragma unroll
    for (int i = 0; i < TPW; ++i) {
      const int t = mfma_base(wave * TPW + i, s, row) + 4 * s * kk;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const int te = t + e * s;
        R[ph(te)] = acc[i][e];
        if (te < reach) R[ph(N + te)] = acc[i][e];
      }
    }
  }
}

// Host side: FwdArgs / InvArgs as the fused kernels; p.hlpad (forward) / p.hlpad_a (inverse) = the halo,
// p.tap_lds = the tap table's element offset.  L = 30 (coif5) and 16 (db8 / sym8) are instantiated.
template <int L, int TPW, int NT>
static hipError_t run_fwd(const FwdArgs<float>& a, int lds, hipStream_t st) {
  auto k = k_forward_mfma<L, TPW, NT>;
  static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(NT), lds, st, a);
  return hipGetLastError();
}

template <int L, int TPW, int NT>
static hipError_t run_inv(const InvArgs<float>& a, int lds, hipStream_t st) {
  auto k = k_inverse_mfma<L, TPW, NT>;
  static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(k, dim3((unsigned)a.B), dim3(NT), lds, st, a);
  return hipGetLastError();
}

#define VW_MFMA_DISPATCH(RUN, a, lds, st)                                    \
  switch (a.taps * 100 + a.N / 1024) {                                       \
    case 3002: return RUN<30, 2, 256>(a, lds, st);                           \
    case 3004: return RUN<30, 4, 256>(a, lds, st);                           \
    case 3008: return RUN<30, 8192 / 4 / VW_MFMA_NT8K, VW_MFMA_NT8K>(a, lds, st); \
    case 1602: return RUN<16, 2, 256>(a, lds, st);                           \
    case 1604: return RUN<16, 4, 256>(a, lds, st);                           \
    case 1608: return RUN<16, 8192 / 4 / VW_MFMA_NT8K, VW_MFMA_NT8K>(a, lds, st); \
    default: return hipErrorNotSupported;                                    \
  }

bool mfma_supported(int L, long long N) {
  return (L == 30 || L == 16) && (N == 2048 || N == 4096 || N == 8192);
}

int mfma_halo(int L, int J) { return (4 * ((L + 15 + 3) / 4) - 16) << (J - 1); }

// LDS floats of the padded level region of elements [0, n) (the tap table follows it)
int mfma_region(int n) { return n == 0 ? 0 : (n - 1) + ((n - 1) >> VW_MFMA_PAD_SHIFT) + 1; }

hipError_t launch_forward_mfma(const FwdArgs<float>& a, int lds, hipStream_t st) { VW_MFMA_DISPATCH(run_fwd, a, lds, st) }
hipError_t launch_inverse_mfma(const InvArgs<float>& a, int lds, hipStream_t st) { VW_MFMA_DISPATCH(run_inv, a, lds, st) }

}  // namespace vw
