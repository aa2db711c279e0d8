// vw_deep.hip -- streaming deep-level kernels (instantiation unit, once per element type).
//
// The deep PERIODIC levels j0..J of a long signal (BatchStreamingMODWT's 2^20-sample blocks at db8
// J = 10: levels 6..10) in ONE launch each way, each input read from HBM once and each output written
// once.  Level j0's spacing P = 2^(j0-1) divides N, so from level j0 on the cascade never mixes the
// residue classes mod P: in the decimated coordinate q (sample t = q*P + r) level j0+k is a dense
// L-tap filter with spacing 2^k (MultiLevelMODWTTransform.java:243-251 forward, :339-349 / :576-589
// inverse; ScalarOps.java:700-723 circular convolution).
//
// A workgroup owns C consecutive residues (64 contiguous bytes per decimated position) of one signal
// and STREAMS along q in tiles of kDeepT positions.  Every level keeps, in an LDS ring, the part of its
// input that the coming tiles still read (its history of (L-1)*2^k positions) plus the current tile,
// so nothing is re-read or recomputed between tiles -- the column sweeps read and write three rows per
// level (2.1x the group's algorithmic bytes at db8 levels 6..10), the earlier column-group tiles
// re-read their whole reach per tile.  The next tile's input arrives by LDS-DMA
// (global_load_lds_dwordx4) `depth` tiles ahead of the computing one: one tile of 4 KiB in flight per
// workgroup left every tile waiting for its load (measured: slower than the sweeps).
//
// Periodic boundary: the stream starts `warm` positions before the segment (wrapping mod N/P) and
// stores nothing there; after that warm-up every ring holds exactly the values the reference's
// modulo index would read (the group's reach is sum_k (L-1)*2^k positions).  Outputs computed from
// the not-yet-valid start of a ring are never stored (the reach argument), so uninitialised LDS is
// harmless.  Per output the taps run in the reference's order (forward: i ascending, both filters
// from one read; inverse: approximation branch then detail branch) -> bit-exact in EXACT mode.
#include "vw_launch.h"
#include "vw_deep.h"
#include <algorithm>

namespace vw {

constexpr int kDeepNP = 2;                // positions per thread
constexpr int kDeepT = 64 * kDeepNP;      // decimated positions per tile (256 threads = 64 x 4 chunks)

// Global stores of the deep kernels (experiment builds: -DVW_DEEP_STORE=0 none, 1 non-temporal).  Default
// 2, plain write-back stores: four residue-block workgroups write 64-byte pieces of each 256-byte span, and
// L2 merges a line's pieces before it goes to HBM (non-temporal: 7.0 rows written for 6 on db8-stream;
// write-back forward 8.70-8.74 vs 8.80-8.84 ms, profiles/r03/ab_deep_store_db8.log)
#ifndef VW_DEEP_STORE
#define VW_DEEP_STORE 2
#endif
template <typename vec, typename T>
__device__ __forceinline__ void deep_store(T* dst, const vec& v) {
  if constexpr (VW_DEEP_STORE == 1) __builtin_nontemporal_store(v, reinterpret_cast<vec*>(dst));
  else if constexpr (VW_DEEP_STORE == 2) *reinterpret_cast<vec*>(dst) = v;
}
constexpr int kDeepThreads = 256;
// Forward levels 0..4 of a deep group with compile-time spacing (immediate LDS offsets); 0: runtime form only
#ifndef VW_DEEP_CK
#define VW_DEEP_CK 1
#endif
#ifndef VW_DEEP_TC
#define VW_DEEP_TC 8   // taps whose LDS reads the no-wrap forward loop issues before their FMAs
#endif
constexpr int kDeepTC = VW_DEEP_TC;
#ifndef VW_DEEP_PAIR
#define VW_DEEP_PAIR 1  // forward levels with spacing >= 4: output pairs P0, P0 + SK share their reads
#endif


// One wave's LDS-DMA of 16 positions x 64 bytes (1 KiB): lane -> position lane / 4, 16-byte chunk lane % 4.
template <typename T>
__device__ __forceinline__ void deep_dma(T* lds_dst, const T* __restrict__ gsrc) {
  const unsigned lds = (unsigned)(uintptr_t)lds_dst;
  unsigned keep;
  asm volatile(
      "s_mov_b32 %0, m0\n\t"
      "s_mov_b32 m0, %2\n\t"
      "s_nop 0\n\t"
      "global_load_lds_dwordx4 %1, off\n\t"
      "s_mov_b32 m0, %0"
      : "=&s"(keep)
      : "v"(gsrc), "s"(__builtin_amdgcn_readfirstlane(lds))
      : "memory");
}

// Prefetch bookkeeping (per wave; every quantity is wave-uniform).  Event order: the prologue issues the
// DMA batches of tiles 0..D-1; tile tau issues the batch of tile tau + D (if it exists), then st(tau)
// stores.  Before tile tn computes, its batch must have landed: the wave waits until at most the
// vector-memory operations issued AFTER that batch are outstanding (vmcnt retires in issue order).
struct DeepPf {
  int D, nt, ndma, nst, warm_tiles;
  __device__ __forceinline__ int st(int tau) const { return tau >= warm_tiles ? nst : 0; }
  __device__ __forceinline__ int after(int tn, int t) const {  // ops issued after tile tn's batch, by the end of tile t
    int n = 0, tau0;
    if (tn < D) {
      n += (min(D, nt) - 1 - tn) * ndma;  // later prologue batches
      tau0 = 0;
    } else {
      n += st(tn - D);                    // the stores of the tile that issued it
      tau0 = tn - D + 1;
    }
    for (int tau = tau0; tau <= t; ++tau) n += (tau + D < nt ? ndma : 0) + st(tau);
    return n;
  }
};

// Workgroup -> (signal b, residue block rb, segment sg).  The nb residue blocks of one (b, sg) read and
// write interleaved 64-byte pieces of the same 128-byte lines: they go to the same XCD (blockIdx % 8)
// so those lines meet in one L2.  Returns false for the padding workgroups of the rounded grid.
struct DeepWork {
  long long b;
  int rb, sg;
};

__device__ __forceinline__ bool deep_work(long long B, int nb, int seg, DeepWork* w) {
  const long long id = blockIdx.x;
  const long long xcd = id & 7, slot = id >> 3;
  const long long gi = (slot / nb) * 8 + xcd;  // (b, sg) group
  if (gi >= B * seg) return false;
  w->rb = (int)(slot % nb);
  w->b = gi / seg;
  w->sg = (int)(gi % seg);
  return true;
}

__device__ __forceinline__ int ring_wrap(int s, int cap) { return s < 0 ? s + cap : (s >= cap ? s - cap : s); }

// ---------------------------------------------------------------------------------------------------
// Thread mapping: thread tid owns the 16-byte chunk (tid & 3) of the C residues at the kDeepNP
// positions pi + 64 r (pi = tid >> 2) of a tile: kDeepNP independent accumulators per branch and
// element keep the dependent FMA chains of the few resident waves overlapped.  Ring slots are derived
// from a workgroup-uniform base per tile and level (one compare per tap, no integer division).

// Forward: level j0+k reads its input at q - i*2^k (left reach), so the stream runs q ascending.
// Ring k holds level j0+k's input; ring 0 is fed by LDS-DMA, `depth` tiles ahead (capacity >= history +
// (depth + 1) tiles, a multiple of 16), ring k+1 by level k's approximation.
template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(kDeepThreads) k_forward_deep(const DeepArgs<T> p) {
  constexpr int V = VT<T>::V;
  constexpr int C = 64 / (int)sizeof(T);
  constexpr int NP = kDeepNP;
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* const lds = reinterpret_cast<T*>(smem);
  DeepWork wk;
  if (!deep_work(p.B, p.nb, p.seg, &wk)) return;
  const int P = p.P, nq = p.nq, g = p.g;
  const int tid = threadIdx.x;
  const int pi = tid >> 2;                  // first position within the tile
  const int ce = (tid & 3) * V;             // element offset within the C residues
  const int wave = tid >> 6, lane = tid & 63;
  const long long rowoff = wk.b * (long long)p.N + (long long)wk.rb * C;
  const T* __restrict__ src = p.src + wk.b * p.lda + (long long)wk.rb * C;
  T nf = T(0);  // VW_FLAG_REF_NONFINITE (p.nf_flag: out = a_J): the probe of the stored approximation
  const int qs = wk.sg * p.seglen;
  const int qe = min(qs + p.seglen, nq);
  const int total = p.warm + (qe - qs);     // positions streamed
  const int nt = (total + kDeepT - 1) / kDeepT;
  int qst = (qs - p.warm) % nq;             // q of stream position 0
  if (qst < 0) qst += nq;
  auto qwrap = [&](int q) { return q >= nq ? q - nq : q; };
  auto q_tile = [&](int u0) { return (int)(((long long)qst + u0) % nq); };  // uniform
  // this wave's share of a tile's DMA: 16-position chunks wave + 4m, lane -> position lane / 4
  auto dma_tile = [&](int u0) {
    const int s0 = u0 % p.cap[0], q0 = q_tile(u0);
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const int c16 = 16 * (wave + 4 * m);
      const int q = qwrap(q0 + c16 + (lane >> 2));
      const int sl = s0 + c16 >= p.cap[0] ? s0 + c16 - p.cap[0] : s0 + c16;  // caps are multiples of 16
      deep_dma<T>(lds + p.off[0] + sl * C, src + (long long)q * P + (lane & 3) * V);
    }
  };
  DeepPf pf{p.depth, nt, NP, NP * (g + 1), p.warm / kDeepT};
  for (int i = 0; i < min(pf.D, nt); ++i) dma_tile(i * kDeepT);  // prologue: D tiles in flight
  wait_vmcnt_rt(pf.after(0, -1));
  lds_barrier();
  for (int t = 0; t < nt; ++t) {
    const int u0 = t * kDeepT;
    if (t + pf.D < nt) dma_tile(u0 + pf.D * kDeepT);  // ring 0: tile t + D, in flight across D tiles
    const bool store = u0 >= p.warm;                   // tile-uniform; the last tile's tail is masked
    const int q0 = q_tile(u0);
    for (int k = 0; k < g; ++k) {
      if (k > 0) lds_barrier();  // ring k holds level k-1's approximation of this tile
      const int cap = p.cap[k], sk = 1 << k;
      const T* ring = lds + p.off[k] + ce;
      const int s0 = u0 % cap;
      // One level of this tile.  KC >= 0: compile-time spacing 2^KC (immediate LDS offsets); -1: runtime.
      auto level = [&](auto kc) __attribute__((always_inline)) {
        constexpr int KC = decltype(kc)::value;
        // Output pairs (spacing SK >= 4, VW_DEEP_PAIR): a thread's two positions are P0 and P0 + SK, so
        // they share L - 1 of their inputs -- L + 1 LDS reads instead of 2L.  Consecutive threads take
        // consecutive residues of the block (P0 = (pi / SK) * 2SK + pi % SK), so a quarter-wave still
        // reads four consecutive positions (256 contiguous bytes, conflict-free).  Below SK = 4 that
        // mapping would put two lanes of a quarter-wave on one bank group: those levels keep pi, pi + 64.
        constexpr bool PAIR = VW_DEEP_PAIR && KC >= 2;
        constexpr int KP = PAIR ? KC : 0;
        int pos[NP];
#pragma unroll
        for (int r = 0; r < NP; ++r)
          pos[r] = PAIR ? ((pi >> KP) << (KP + 1)) + (pi & ((1 << KP) - 1)) + (r << KP) : pi + 64 * r;
        int br[NP];
#pragma unroll
        for (int r = 0; r < NP; ++r) {
          const int v = s0 + pos[r];
          br[r] = v >= cap ? v - cap : v;
        }
        T al[NP][V], ah[NP][V];
#pragma unroll
        for (int r = 0; r < NP; ++r)
#pragma unroll
          for (int e = 0; e < V; ++e) { al[r][e] = T(0); ah[r][e] = T(0); }
        // tap i of output r reads slot br[r] - i*sk (mod cap), i ascending; the same products in every form
        auto fma2 = [&](int r, int i, const vec& x) __attribute__((always_inline)) {
#pragma unroll
          for (int e = 0; e < V; ++e) {
            al[r][e] = madd<FMA>(al[r][e], x[e], p.lo[i]);
            ah[r][e] = madd<FMA>(ah[r][e], x[e], p.hi[i]);
          }
        };
        if constexpr (PAIR) {
          // reads t = 0..L at slot br[1] - t*SK: tap t of P0 + SK (t < L), tap t - 1 of P0 (t >= 1)
          constexpr int SK = 1 << KP;
          const T* a0 = ring + (br[1] - L * SK) * C;
          const T* a1 = a0 + cap * C;
          auto use = [&](int t, const vec& x) __attribute__((always_inline)) {
            if (t < L) fma2(1, t, x);
            if (t >= 1) fma2(0, t - 1, x);
          };
          if (__all(br[1] >= L * SK)) {
            const unsigned ab = lds_base(a0);
            static_for<0, (L + 1 + kDeepTC - 1) / kDeepTC>([&](auto c) __attribute__((always_inline)) {
              constexpr int T0 = decltype(c)::value * kDeepTC;
              constexpr int T1 = (T0 + kDeepTC < L + 1) ? T0 + kDeepTC : L + 1;
              vec xs[T1 - T0];
#pragma unroll
              for (int t = T0; t < T1; ++t)
                xs[t - T0] = lds_vec_at<vec>(ab + (unsigned)((L - t) * SK * C * (int)sizeof(T)));
#pragma unroll
              for (int t = T0; t < T1; ++t) use(t, xs[t - T0]);
            });
          } else {
#pragma unroll
            for (int t = 0; t <= L; ++t) {
              const T* a = br[1] >= t * SK ? a0 : a1;
              use(t, *reinterpret_cast<const vec*>(a + (L - t) * SK * C));
            }
          }
        } else if constexpr (KC >= 0) {
          // Compile-time spacing: the reads of a lane sit at fixed distances (L-1-i)*SK positions above
          // a0 = slot br - (L-1)*SK, so each is ONE ds_read at an immediate offset from a0 -- or from
          // a1 = a0 + cap where that slot wrapped (br < i*SK: one compare and select per read).  A wave
          // whose lanes never wrap at this level takes the select-free loop.  The runtime form (wrap
          // arithmetic per read: sub, compare, select, address) measured ~1 INT32 VALU per FMA on
          // db8-stream's levels 6..10 (profiles/r05/pmc_mix_db8_a0b973e.txt).
          constexpr int SK = 1 << (KC >= 0 ? KC : 0);
          const T* a0[NP];
          const T* a1[NP];
          bool nowrap = true;
#pragma unroll
          for (int r = 0; r < NP; ++r) {
            a0[r] = ring + (br[r] - (L - 1) * SK) * C;
            a1[r] = a0[r] + cap * C;
            nowrap = nowrap && br[r] >= (L - 1) * SK;
          }
          if (__all(nowrap)) {
            // 32-bit LDS base per lane (laundered: the immediate offsets stay positive); the reads of a
            // chunk of kDeepTC taps are issued together (VGPRs to spare at two workgroups per CU)
            unsigned ab[NP];
#pragma unroll
            for (int r = 0; r < NP; ++r) ab[r] = lds_base(a0[r]);
            static_for<0, (L + kDeepTC - 1) / kDeepTC>([&](auto c) __attribute__((always_inline)) {
              constexpr int I0 = decltype(c)::value * kDeepTC;
              constexpr int I1 = (I0 + kDeepTC < L) ? I0 + kDeepTC : L;
              vec xs[I1 - I0][NP];
#pragma unroll
              for (int i = I0; i < I1; ++i)
#pragma unroll
                for (int r = 0; r < NP; ++r)
                  xs[i - I0][r] = lds_vec_at<vec>(ab[r] + (unsigned)((L - 1 - i) * SK * C * (int)sizeof(T)));
#pragma unroll
              for (int i = I0; i < I1; ++i)
#pragma unroll
                for (int r = 0; r < NP; ++r) fma2(r, i, xs[i - I0][r]);
            });
          } else {
#pragma unroll
            for (int i = 0; i < L; ++i)
#pragma unroll
              for (int r = 0; r < NP; ++r) {
                const T* a = br[r] >= i * SK ? a0[r] : a1[r];
                fma2(r, i, *reinterpret_cast<const vec*>(a + (L - 1 - i) * SK * C));
              }
          }
        } else {
#pragma unroll
          for (int i = 0; i < L; ++i) {
#pragma unroll
            for (int r = 0; r < NP; ++r) {
              int sl = br[r] - i * sk;
              sl = sl < 0 ? sl + cap : sl;
              fma2(r, i, *reinterpret_cast<const vec*>(ring + sl * C));
            }
          }
        }
#pragma unroll
        for (int r = 0; r < NP; ++r)
#pragma unroll
          for (int e = 0; e < V; ++e) {  // both chains computed here, not sunk into the store branch
            asm volatile("" : "+v"(al[r][e]));
            asm volatile("" : "+v"(ah[r][e]));
          }
        const int cap1 = k + 1 < g ? p.cap[k + 1] : 1;
        const int s1 = u0 % cap1;
#pragma unroll
        for (int r = 0; r < NP; ++r) {
          vec od, oa;
#pragma unroll
          for (int e = 0; e < V; ++e) { od[e] = ah[r][e]; oa[e] = al[r][e]; }
          // every tile issues the same number of stores per wave (DeepPf); only the last tile's tail is masked
          const bool live = store && u0 + pos[r] < total;
          const long long gofs = rowoff + (long long)qwrap(q0 + pos[r]) * P + ce;
          if (live) deep_store<vec>(p.out_d[k] + gofs, od);
          if (k + 1 < g) {
            const int v = s1 + pos[r];
            *reinterpret_cast<vec*>(lds + p.off[k + 1] + (v >= cap1 ? v - cap1 : v) * C + ce) = oa;
          } else if (live) {
            deep_store<vec>(p.out + gofs, oa);
            if (p.nf_flag)
#pragma unroll
              for (int e = 0; e < V; ++e) nf = nf_step<T>(oa[e], nf);
          }
        }
      };
      switch (VW_DEEP_CK ? k : -1) {
        case 0: level(std::integral_constant<int, 0>{}); break;
        case 1: level(std::integral_constant<int, 1>{}); break;
        case 2: level(std::integral_constant<int, 2>{}); break;
        case 3: level(std::integral_constant<int, 3>{}); break;
        case 4: level(std::integral_constant<int, 4>{}); break;
        default: level(std::integral_constant<int, -1>{}); break;
      }
    }
    // tile t+1's batch has landed once at most the operations issued after it are outstanding
    if (t + 1 < nt) wait_vmcnt_rt(pf.after(t + 1, t));
    lds_barrier();
  }
  if (p.nf_flag) nf_flag_row<T>(p.nf_flag, wk.b, nf);
}

// ---------------------------------------------------------------------------------------------------
// Inverse: level j0+k reads a and d at q + i*2^k (right reach), so the stream runs q DESCENDING:
// stream position u = 0, 1, ... is q = qe - 1 + warm - u, and "history" is the larger q.  Rings:
// A_k (approximation input of level j0+k; A_{g-1} = a_J fed by DMA, A_k for k < g-1 by level k+1's
// output) and D_k (d of level j0+k, fed by DMA `depth` tiles ahead).  DMA-fed rings have capacity >=
// history + (depth + 1) tiles.  A descending chunk of 16 positions is still written to 16 ascending
// slots by the DMA, so positions map to slots through u (not q).
template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(kDeepThreads) k_inverse_deep(const DeepArgs<T> p) {
  constexpr int V = VT<T>::V;
  constexpr int C = 64 / (int)sizeof(T);
  constexpr int NP = kDeepNP;
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* const lds = reinterpret_cast<T*>(smem);
  DeepWork wk;
  if (!deep_work(p.B, p.nb, p.seg, &wk)) return;
  const int P = p.P, nq = p.nq, g = p.g;
  const int tid = threadIdx.x;
  const int pi = tid >> 2;
  const int ce = (tid & 3) * V;
  const int wave = tid >> 6, lane = tid & 63;
  const long long cofs = wk.b * (long long)p.N + (long long)wk.rb * C;
  const int qs = wk.sg * p.seglen;
  const int qe = min(qs + p.seglen, nq);
  const int total = p.warm + (qe - qs);
  const int nt = (total + kDeepT - 1) / kDeepT;
  const int qst = (int)(((long long)qe - 1 + p.warm) % nq);   // q of stream position 0
  auto qdown = [&](int q) { return q < 0 ? q + nq : q; };
  auto q_tile = [&](int u0) { return (int)((((long long)qst - u0) % nq + nq) % nq); };
  auto dma_ring = [&](int rg, const T* row, int u0, int s0, int q0) {
#pragma unroll
    for (int m = 0; m < NP; ++m) {
      const int c16 = 16 * (wave + 4 * m);
      const int q = qdown(q0 - c16 - (lane >> 2));
      const int sl = s0 + c16 >= p.cap[rg] ? s0 + c16 - p.cap[rg] : s0 + c16;  // caps are multiples of 16
      deep_dma<T>(lds + p.off[rg] + sl * C, row + cofs + (long long)q * P + (lane & 3) * V);
    }
  };
  // ring indices: A_k = k, D_k = g + k
  auto dma_tile = [&](int u0) {
    const int q0 = q_tile(u0);
    if (p.src) dma_ring(g - 1, p.src, u0, u0 % p.cap[g - 1], q0);
    for (int k = 0; k < g; ++k)
      if (p.src_d[k]) dma_ring(g + k, p.src_d[k], u0, u0 % p.cap[g + k], q0);
  };
  int nring = p.src ? 1 : 0;
  for (int k = 0; k < g; ++k) nring += p.src_d[k] ? 1 : 0;
  DeepPf pf{p.depth, nt, NP * nring, NP, p.warm / kDeepT};
  for (int i = 0; i < min(pf.D, nt); ++i) dma_tile(i * kDeepT);
  wait_vmcnt_rt(pf.after(0, -1));
  lds_barrier();
  for (int t = 0; t < nt; ++t) {
    const int u0 = t * kDeepT;
    if (t + pf.D < nt) dma_tile(u0 + pf.D * kDeepT);
    const bool store = u0 >= p.warm;
    const int q0 = q_tile(u0);
    for (int k = g - 1; k >= 0; --k) {
      if (k < g - 1) lds_barrier();  // A_k holds level k+1's output of this tile
      const int sk = 1 << k;
      T acc[NP][V];
#pragma unroll
      for (int r = 0; r < NP; ++r)
#pragma unroll
        for (int e = 0; e < V; ++e) acc[r][e] = T(0);
      // approximation branch (all taps), then detail branch: MultiLevelMODWTTransform.java:576-589
      auto branch = [&](int rg, const T* f, bool thr_on, T thr_b) {
        const int cap = p.cap[rg];
        const T* ring = lds + p.off[rg] + ce;
        const int s0 = u0 % cap;
        int br[NP];
#pragma unroll
        for (int r = 0; r < NP; ++r) {
          const int v = s0 + pi + 64 * r;
          br[r] = v >= cap ? v - cap : v;
        }
#pragma unroll
        for (int i = 0; i < L; ++i) {
#pragma unroll
          for (int r = 0; r < NP; ++r) {
            int sl = br[r] - i * sk;
            sl = sl < 0 ? sl + cap : sl;
            const vec x = *reinterpret_cast<const vec*>(ring + sl * C);
#pragma unroll
            for (int e = 0; e < V; ++e)
              acc[r][e] = madd<FMA>(acc[r][e], thr_on ? threshold_t(x[e], thr_b, p.soft) : x[e], f[i]);
          }
        }
      };
      if (k < g - 1 || p.src) branch(k, p.lo, false, T(0));
      if (p.src_d[k]) {
        if (p.thr[k]) branch(g + k, p.hi, true, load_uniform(p.thr[k] + wk.b));
        else branch(g + k, p.hi, false, T(0));
      }
      if (k > 0) {
        const int cap1 = p.cap[k - 1];
        const int s1 = u0 % cap1;
#pragma unroll
        for (int r = 0; r < NP; ++r) {
          vec o;
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] = acc[r][e];
          const int v = s1 + pi + 64 * r;
          *reinterpret_cast<vec*>(lds + p.off[k - 1] + (v >= cap1 ? v - cap1 : v) * C + ce) = o;
        }
      } else if (store) {
#pragma unroll
        for (int r = 0; r < NP; ++r) {
          vec o;
#pragma unroll
          for (int e = 0; e < V; ++e) o[e] = acc[r][e];
          if (u0 + pi + 64 * r < total) deep_store<vec>(p.out + cofs + (long long)qdown(q0 - pi - 64 * r) * P + ce, o);
        }
      }
    }
    if (t + 1 < nt) wait_vmcnt_rt(pf.after(t + 1, t));
    lds_barrier();
  }
}

template <typename T, int L, bool FMA, bool INV>
static hipError_t run_deep(const DeepArgs<T>& a, int lds, hipStream_t st) {
  auto k = INV ? k_inverse_deep<T, L, FMA> : k_forward_deep<T, L, FMA>;
  static LdsOnce configured;
  hipError_t e = set_lds(k, lds, &configured);
  if (e != hipSuccess) return e;
  const long long groups = (a.B * a.seg + 7) / 8 * 8;
  hipLaunchKernelGGL(k, dim3((unsigned)(groups * a.nb)), dim3(kDeepThreads), lds, st, a);
  return hipGetLastError();
}

template <typename T>
hipError_t launch_deep(const DeepArgs<T>& a, int lds_bytes, bool fma, bool inverse, hipStream_t st) {
  switch (a.taps) {
#define VW_CASE(n)                                                                                    \
    case n:                                                                                           \
      if (inverse) return fma ? run_deep<T, n, true, true>(a, lds_bytes, st) : run_deep<T, n, false, true>(a, lds_bytes, st); \
      return fma ? run_deep<T, n, true, false>(a, lds_bytes, st) : run_deep<T, n, false, false>(a, lds_bytes, st);
    VW_TAP_LIST(VW_CASE)
#undef VW_CASE
    default:
      return hipErrorNotSupported;
  }
}
template hipError_t launch_deep<VW_T>(const DeepArgs<VW_T>&, int, bool, bool, hipStream_t);

}  // namespace vw
