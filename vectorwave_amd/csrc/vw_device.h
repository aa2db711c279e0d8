#pragma once
// vw_device.h -- hand-written CDNA4 (gfx950) HIP kernels for VectorWave's MODWT / SWT hot path.
//
// The hot loop of the reference is the a-trous convolution of one level:
//   forward  (K1-K3)  out[t] = sum_{l=0}^{L_j-1} f_j[l] * x[g(t - l)]           ScalarOps.java:700-835
//   inverse  (K4-K6)  y[t]   = sum_l h_j[l] * a[g(t +/- l - tau)] (+) sum_l g_j[l] * d[...]
//                                                                  MultiLevelMODWTTransform.java:554-645
// with f_j the base taps * 1/sqrt(2) upsampled by 2^(j-1) (ScalarOps.java:909-916).  Only the L
// non-zero taps at spacing s = 2^(j-1) contribute; the zero taps add +/-0.0 to a sum that is never
// -0.0, so skipping them is exact.
//
// MI355X design:
//  * One workgroup per signal.  The whole level input lives in LDS with its boundary "halo"
//    materialised around it, so the inner loop is boundary-agnostic: the reference's index map g
//    (periodic wrap, zero padding, half-sample mirror, FFT zero-pad, streaming history) is applied
//    once per level when the halo is filled, not once per tap.
//  * The J-level cascade is fused: x is read from HBM once, each detail level is written once,
//    the running approximation never leaves LDS / VGPRs (forward); the inverse reads each detail
//    level once (prefetched into VGPRs while the previous level computes) and writes y once.
//  * Each lane owns 16-byte vectors of consecutive outputs (2 x fp64 / 4 x fp32): global loads
//    and stores are dwordx4 and fully coalesced; LDS reads are ds_read_b128 at spacing s, or one
//    register window for s < vector width (level 1), conflict-free (consecutive lanes, consecutive
//    16-byte slots).
//  * EXACT variant: separate v_mul_f64 / v_add_f64 in the reference's tap order (file compiled with
//    -ffp-contract=off): bit-identical to vectorwave-core.  FMA variant: v_fma_f64, ~1 ulp/tap.
//  * Bandwidth-bound stencil: no MFMA.
#include <hip/hip_runtime.h>
#include <cstdint>
#include <type_traits>
#include "vw_internal.h"

#pragma clang fp contract(off)

namespace vw {

template <typename T> struct VT;
template <> struct VT<double> { typedef double v __attribute__((ext_vector_type(2))); static constexpr int V = 2; };
template <> struct VT<float>  { typedef float  v __attribute__((ext_vector_type(4))); static constexpr int V = 4; };

__device__ __forceinline__ double fma_t(double a, double b, double c) { return __builtin_fma(a, b, c); }
__device__ __forceinline__ float fma_t(float a, float b, float c) { return __builtin_fmaf(a, b, c); }

// acc + x*f : EXACT = rounded product then rounded sum (Java semantics); FMA = one rounding.
template <bool FMA, typename T>
__device__ __forceinline__ T madd(T acc, T x, T f) {
  if constexpr (FMA) return fma_t(x, f, acc);
  else return acc + x * f;
}

// acc_e (+)= x_e * f over one 16-byte vector of outputs, per element.  PK (fp32 only): two packed
// operations per pair (v_pk_fma_f32; EXACT v_pk_mul_f32 + v_pk_add_f32, the same rounding per
// element).  Measured on coif5 fp32, same box (profiles/r03/ab_coif5_pk_cinv.log): packed forward
// 6.46 -> 5.88 ms; packed inverse 7.05 -> 7.23 ms.  So the forward kernels pack (VW_PK_F32_FWD,
// default 1) and the inverse ones do not (VW_PK_F32, default 0).  tools/valubench.hip: v_fma_f32
// issues 95 TFLOP/s, v_pk_fma_f32 117 on this GPU.
#ifndef VW_PK_F32
#define VW_PK_F32 0
#endif
#ifndef VW_PK_F32_FWD
#define VW_PK_F32_FWD 1
#endif
constexpr bool kPkFwd = VW_PK_F32_FWD != 0;
template <bool FMA, bool PK = (VW_PK_F32 != 0), typename T, typename X>
__device__ __forceinline__ void vmadd(T* acc, const X& x, T f) {
  if constexpr (PK && std::is_same<T, float>::value) {
    typedef float f2 __attribute__((ext_vector_type(2)));
    const f2 fv = {f, f};
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      f2 a = {acc[2 * h], acc[2 * h + 1]};
      const f2 xv = {x[2 * h], x[2 * h + 1]};
      if constexpr (FMA) a = __builtin_elementwise_fma(xv, fv, a);
      else a = a + xv * fv;
      acc[2 * h] = a[0];
      acc[2 * h + 1] = a[1];
    }
  } else {
#pragma unroll
    for (int e = 0; e < VT<T>::V; ++e) acc[e] = madd<FMA>(acc[e], x[e], f);
  }
}

// Workgroup-uniform read of data written before the launch (thresholds, per-signal constants)
// through the constant address space: a scalar (SMEM) load.  A vector load of it inside a level loop
// would make the waitcnt pass, which cannot count across the loop's conditional load, wait vmcnt(0)
// at the loop head -- i.e. for the detail-row prefetch that is meant to stay in flight.
template <typename T>
__device__ __forceinline__ T load_uniform(const T* q) {
  typedef const __attribute__((address_space(4))) T* cptr;
  return *(cptr)(q);
}

__device__ __forceinline__ bool finite_t(double v) { return __builtin_isfinite(v); }
__device__ __forceinline__ bool finite_t(float v) { return __builtin_isfinite(v); }

// MathUtils.symmetricBoundaryExtension  core/util/MathUtils.java:30-51
__device__ __forceinline__ int sym_index(int idx, int n) {
  if (idx >= 0 && idx < n) return idx;
  int period = 2 * n;
  idx = ((idx % period) + period) % period;
  if (idx >= n) idx = period - idx - 1;
  return idx;
}

// Workgroup barrier that orders LDS only: waits for this wave's LDS operations (lgkmcnt(0)) and
// lets global stores and prefetch loads stay in flight across it.  (__syncthreads() also waits
// vmcnt(0), which would expose the latency of every detail-level store at every level.)  Values
// loaded from global memory are waited for by the compiler at their first use, as usual.
// 16-byte LDS read at a 32-bit LDS byte address.  With the base laundered (lds_base) the compiler keeps
// base + constant as ONE ds_read with the constant in its offset field, instead of re-basing on the
// highest address of a run of reads and paying a v_add per read.
#pragma clang diagnostic push
#pragma clang diagnostic ignored "-Wint-to-pointer-cast"
template <typename vec>
__device__ __forceinline__ vec lds_vec_at(unsigned a) {
  return *(const __attribute__((address_space(3))) vec*)a;
}
#pragma clang diagnostic pop
template <typename T>
__device__ __forceinline__ unsigned lds_base(const T* p) {
  unsigned a = (unsigned)(uintptr_t)p;
  asm volatile("" : "+v"(a));
  return a;
}

__device__ __forceinline__ void lds_barrier() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0); vmcnt / expcnt untouched
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Wait for this wave's outstanding global loads (and stores) explicitly.  Used where every
// outstanding op is one we need anyway: the waitcnt pass models exec-masked (skippable) blocks
// conservatively, and without this it keeps the prologue loads "pending" into the level loop, where
// it then waits for the detail stores of the previous level before touching those registers.
__device__ __forceinline__ void wait_vmem() { __builtin_amdgcn_s_waitcnt(0x0F70); }  // vmcnt(0)

// Value of a level input at signal index idx outside [0, N), read from the LDS copy `buf`
// (element 0 at buf[0]).  The reference's index maps; see HaloMode.
template <typename T>
__device__ __forceinline__ T halo_value_lds(const T* buf, int idx, int N, int mode, int npow2,
                                            const T* hist_b, int hist_len) {
  switch (mode) {
    case kHaloPeriodic: { int r = idx % N; if (r < 0) r += N; return buf[r]; }
    case kHaloSymmetric: return buf[sym_index(idx, N)];
    case kHaloFftPad: { int r = idx < 0 ? idx + npow2 : idx; return (r >= 0 && r < N) ? buf[r] : T(0); }
    case kHaloHistory: return (idx < 0 && idx >= -hist_len) ? hist_b[hist_len + idx] : T(0);
    default: return T(0);
  }
}

// Fill positions [-hl, 0) and [N, N+hr) of the LDS level buffer.  The streaming-history fill is a
// separate loop: it is the only global load inside the level loop, and vmcnt is in order (stores
// count too), so waiting for it would also wait for every detail store still in flight.
template <typename T>
__device__ __forceinline__ void fill_halo(T* buf, int N, int hl, int hr, int mode, int npow2,
                                          const T* hist_b, int hist_len) {
  const int total = hl + hr;
  if (mode == kHaloHistory) {
    for (int q = threadIdx.x; q < total; q += blockDim.x) {
      const int idx = q < hl ? q - hl : N + (q - hl);
      buf[idx] = (idx < 0 && idx >= -hist_len) ? hist_b[hist_len + idx] : T(0);
    }
    return;
  }
  for (int q = threadIdx.x; q < total; q += blockDim.x) {
    const int idx = q < hl ? q - hl : N + (q - hl);
    buf[idx] = halo_value_lds(buf, idx, N, mode, npow2, (const T*)nullptr, 0);
  }
}

// ---------------------------------------------------------------------------------------------
// Register windows of the levels whose spacing is below the vector width.  Long filters take their
// taps in chunks of kWinTaps, each with its own aligned sub-window (a whole-filter window of coif5
// at spacing 2 in fp32 would be 64 registers); per output the taps still ascend.
constexpr int kWinTaps = 8;

__host__ __device__ constexpr int floor_div(int a, int b) { return a >= 0 ? a / b : -((-a + b - 1) / b); }

template <int C, int NC, typename F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (C < NC) {
    f(std::integral_constant<int, C>{});
    static_for<C + 1, NC>(f);
  }
}

// Forward: one 16-byte vector of consecutive outputs t0..t0+V-1, both filters from one set of
// LDS reads.  acc_e (+)= x[t0 + e - i*s] * f[i], i ascending (ScalarOps.java:707-719 order).
template <typename T, int L, bool FMA, int S>
__device__ __forceinline__ void fwd_window(const T* buf, int t0, const T* lo, const T* hi,
                                           T (&al)[VT<T>::V], T (&ah)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  static_for<0, (L + kWinTaps - 1) / kWinTaps>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * kWinTaps;
    constexpr int I1 = (I0 + kWinTaps < L) ? I0 + kWinTaps : L;
    constexpr int A = floor_div(-(I1 - 1) * S, V) * V;       // offsets e - i*S, aligned down
    constexpr int E = (floor_div(V - 1 - I0 * S, V) + 1) * V;
    constexpr int NE = E - A;
    T w[NE];
#pragma unroll
    for (int k = 0; k < NE / V; ++k) {
      vec v = *reinterpret_cast<const vec*>(buf + t0 + A + k * V);
#pragma unroll
      for (int e = 0; e < V; ++e) w[k * V + e] = v[e];
    }
    T fl[I1 - I0], fh[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) { fl[i - I0] = lo[i]; fh[i - I0] = hi[i]; }
#pragma unroll
    for (int i = I0; i < I1; ++i) {
      vmadd<FMA, kPkFwd>(al, &w[-i * S - A], fl[i - I0]);
      vmadd<FMA, kPkFwd>(ah, &w[-i * S - A], fh[i - I0]);
    }
  });
}

template <typename T, int L, bool FMA>
__device__ __forceinline__ void fwd_vec(const T* buf, int t0, int S, const T* lo, const T* hi, int taps,
                                        T (&al)[VT<T>::V], T (&ah)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  if constexpr (L > 0) {
    if (S == 1) { fwd_window<T, L, FMA, 1>(buf, t0, lo, hi, al, ah); return; }
    if constexpr (V == 4) {
      if (S == 2) { fwd_window<T, L, FMA, 2>(buf, t0, lo, hi, al, ah); return; }
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {   // S is a multiple of V: aligned 16-byte reads
      const vec v = *reinterpret_cast<const vec*>(buf + t0 - i * S);
      vmadd<FMA, kPkFwd>(al, v, lo[i]);
      vmadd<FMA, kPkFwd>(ah, v, hi[i]);
    }
  } else {
    for (int i = 0; i < taps; ++i) {
      const T fl = lo[i], fh = hi[i];
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const T xv = buf[t0 + e - i * S];
        al[e] = madd<FMA>(al[e], xv, fl);
        ah[e] = madd<FMA>(ah[e], xv, fh);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Inverse, one branch: acc_e (+)= f[i] * buf[t0 + e + dir*i*s + off], i ascending
// (MultiLevelMODWTTransform.java:578-588 periodic, :612-639 symmetric orientations).
template <typename T, int L, bool FMA, int S, int DIR>
__device__ __forceinline__ void inv_window(const T* buf, int base, const T* f, T (&acc)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  static_for<0, (L + kWinTaps - 1) / kWinTaps>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * kWinTaps;
    constexpr int I1 = (I0 + kWinTaps < L) ? I0 + kWinTaps : L;
    // offsets e + DIR*i*S of the chunk's taps, aligned to whole vectors
    constexpr int A = DIR > 0 ? floor_div(I0 * S, V) * V : floor_div(-(I1 - 1) * S, V) * V;
    constexpr int E = DIR > 0 ? (floor_div(V - 1 + (I1 - 1) * S, V) + 1) * V : (floor_div(V - 1 - I0 * S, V) + 1) * V;
    constexpr int NE = E - A;
    T w[NE];
#pragma unroll
    for (int k = 0; k < NE / V; ++k) {
      vec v = *reinterpret_cast<const vec*>(buf + base + A + k * V);
#pragma unroll
      for (int e = 0; e < V; ++e) w[k * V + e] = v[e];
    }
    T fc[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) fc[i - I0] = f[i];
#pragma unroll
    for (int i = I0; i < I1; ++i) vmadd<FMA>(acc, &w[DIR * i * S - A], fc[i - I0]);
  });
}

template <typename T, int L, bool FMA>
__device__ __forceinline__ void inv_branch(const T* buf, int t0, int S, int dir, int off, const T* f, int taps,
                                           T (&acc)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  if constexpr (L > 0) {
    if ((off & (V - 1)) == 0) {
      const int base = t0 + off;
      if (S == 1) {
        if (dir > 0) inv_window<T, L, FMA, 1, 1>(buf, base, f, acc);
        else inv_window<T, L, FMA, 1, -1>(buf, base, f, acc);
        return;
      }
      if constexpr (V == 4) {
        if (S == 2) {
          if (dir > 0) inv_window<T, L, FMA, 2, 1>(buf, base, f, acc);
          else inv_window<T, L, FMA, 2, -1>(buf, base, f, acc);
          return;
        }
      }
      const int step = dir * S;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const vec v = *reinterpret_cast<const vec*>(buf + base + i * step);
        vmadd<FMA>(acc, v, f[i]);
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = madd<FMA>(acc[e], buf[t0 + e + dir * i * S + off], f[i]);
    }
  } else {
    for (int i = 0; i < taps; ++i) {
      const T fi = f[i];
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = madd<FMA>(acc[e], buf[t0 + e + dir * i * S + off], fi);
    }
  }
}

// Pairwise inverse: acc_e += (h[i]*a[idx] + g[i]*d[idx])  (MODWTTransform.java:251-252, :265-266,
// :290-291; MultiLevelMODWTTransform.java:596-597).  idx = t0 + e + dir*i*s.
template <typename T, bool FMA>
__device__ __forceinline__ T pair_term(T h, T a, T g, T d) {
  if constexpr (FMA) return fma_t(h, a, g * d);
  else return h * a + g * d;
}

template <typename T, int L, bool FMA>
__device__ __forceinline__ void inv_pair(const T* A, const T* D, int t0, int S, int dir, const T* h, const T* g,
                                         int taps, T (&acc)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  if constexpr (L > 0) {
    if (S % V == 0) {
      const int step = dir * S;
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const vec va = *reinterpret_cast<const vec*>(A + t0 + i * step);
        const vec vd = *reinterpret_cast<const vec*>(D + t0 + i * step);
#pragma unroll
        for (int e = 0; e < V; ++e) acc[e] = acc[e] + pair_term<T, FMA>(h[i], va[e], g[i], vd[e]);
        if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // <= 8 reads in flight (VGPR budget)
      }
      return;
    }
#pragma unroll
    for (int i = 0; i < L; ++i) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int idx = t0 + e + dir * i * S;
        acc[e] = acc[e] + pair_term<T, FMA>(h[i], A[idx], g[i], D[idx]);
      }
      if ((i & 1) == 1) __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight (VGPR budget)
    }
  } else {
    for (int i = 0; i < taps; ++i) {
#pragma unroll
      for (int e = 0; e < V; ++e) {
        const int idx = t0 + e + dir * i * S;
        acc[e] = acc[e] + pair_term<T, FMA>(h[i], A[idx], g[i], D[idx]);
      }
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Global <-> register <-> LDS row transfers.  A row is held as NV 16-byte vectors per lane, lane
// `tid` owning vectors w = tid + k*NT (coalesced dwordx4 loads / stores, conflict-free b128 LDS).
//
// Scalar-instruction budget: the scalar unit is shared by the CU's four SIMDs, and per-vector
// runtime checks (bounds, modes, spacing, direction) cost several SALU + a branch each.  So the
// fused kernels make every such decision once per level (row functions below, templated on the
// spacing class and direction), and only the last of a thread's NV vectors carries a bounds check:
// the host sizes the workgroup so that slabs 0..NV-2 are full ((NV-1)*NT <= nvec, vw_capi.cpp).
template <int L, int NV, typename F>
__device__ __forceinline__ void for_vecs(int nvec, F&& fn) {
  const int NT = blockDim.x;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    int w = threadIdx.x + k * NT;
    // Launder w: the addresses derived from it are loop-invariant across the level loop, and
    // hoisting all of them (every vector x every buffer x every spacing path) out of it exhausts
    // the 128-VGPR budget and spills.  Recomputing them per level costs a few VALU.
    asm volatile("" : "+v"(w));
    if ((L > 0 && k < NV - 1) || w < nvec) fn(k, w);
    // ... and keep the scheduler from issuing the LDS reads of every vector at once (NV x L
    // b128 reads in flight = all the VGPRs); 4 waves per SIMD hide the per-vector read latency.
    __builtin_amdgcn_sched_barrier(0);
  }
}

// Cache policy of the streaming row stores / loads (buffer-instruction aux field: 1 = sc0,
// 2 = nt, 16 = sc1).  VW_STORE_AUX < 0 selects the compiler's nontemporal store.
#ifndef VW_STORE_AUX
#define VW_STORE_AUX -1
#endif
#ifndef VW_LOAD_AUX
#define VW_LOAD_AUX -1
#endif
// Forward coefficient rows (read next by an inverse): sc1.  Same box, alternating, rotated buffer
// sets (profiles/r04/ab_store_policy_*.log): db4 4096 x 4096 42.8-44.0K (nt) -> 45.1-46.0K Msamples/s,
// 512 rows 41.0-41.6K -> 42.9-44.1K; write-back (aux 0) 45.1-45.6K / 40.6-41.1K; sym8 / db8 / coif5
// unchanged (their forwards store through k_forward_blk's write-back path or the tiled kernels).
#ifndef VW_FWD_STORE_AUX
#define VW_FWD_STORE_AUX 16
#endif
#ifndef VW_BLK_NT_M
#define VW_BLK_NT_M 8  // k_forward_blk: vector strides m below this store write-back (see there)
#endif
#ifndef VW_INV_STORE_AUX
#define VW_INV_STORE_AUX VW_STORE_AUX  // inverse output rows
#endif
typedef int vw_i4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, 0x7fffffff, 0x00020000);
}

// base: a workgroup-uniform row pointer; i: the lane's 16-byte vector index within the row.
template <int AUX, typename V16, typename T>
__device__ __forceinline__ void stream_store(T* base, int i, V16 v) {
  if constexpr (AUX < 0) {
    __builtin_nontemporal_store(v, reinterpret_cast<V16*>(base) + i);
  } else {
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(vw_i4, v), row_rsrc(base), i * 16, 0, AUX);
  }
}

template <typename V16, typename T>
__device__ __forceinline__ V16 stream_load(const T* base, int i) {
  if constexpr (VW_LOAD_AUX < 0) {
    return __builtin_nontemporal_load(reinterpret_cast<const V16*>(base) + i);
  } else {
    return __builtin_bit_cast(V16, __builtin_amdgcn_raw_buffer_load_b128(row_rsrc(base), i * 16, 0, VW_LOAD_AUX));
  }
}

template <int AUX = VW_STORE_AUX, typename T>
__device__ __forceinline__ void store_vec(T* __restrict__ dst, int t0, int N, bool vec_ok, const T (&v)[VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  if (vec_ok && t0 + V <= N) {
    vec o;
#pragma unroll
    for (int e = 0; e < V; ++e) o[e] = v[e];
    stream_store<AUX, vec>(dst, t0 / V, o);
  } else {
#pragma unroll
    for (int e = 0; e < V; ++e)
      if (t0 + e < N) dst[t0 + e] = v[e];
  }
}

template <typename T>
__device__ __forceinline__ void check_out(int validate, unsigned long long* bad, unsigned long long flat0, int t0,
                                          int N, const T (&v)[VT<T>::V]) {
  if (!validate) return;
  constexpr int V = VT<T>::V;
#pragma unroll
  for (int e = 0; e < V; ++e)
    if (t0 + e < N && !finite_t(v[e])) atomicMin(bad, (1ull << 62) | (flat0 + (unsigned long long)(t0 + e)));
}

// MutableMultiLevelMODWTResult.applyThreshold (:97-114): soft = signum(c)*(|c|-T) above T, hard
// keeps c when |c| > T.
template <typename T>
__device__ __forceinline__ T threshold_t(T c, T thr, int soft) {
  const T av = c < T(0) ? -c : c;
  if (soft) {
    // Math.signum(c) * (|c| - T): c != 0 here, and a product with +-1 is a sign flip, i.e. copysign
    // (c == 0 passes only for a negative threshold: signum(+-0) * x = +-0 * x)
    if (av > thr) return c == T(0) ? c * (av - thr) : __builtin_copysign(av - thr, c);
    return T(0);
  }
  return av <= thr ? T(0) : c;
}

// Issue the loads of one row into registers.  Loads only: the values are first touched where they
// are written to LDS (the zero / threshold selection is applied there), so a prefetch is never
// waited for early.  The vector loads are unconditional (lanes past the row re-read its last vector;
// those registers are never used): an exec-masked load in its own basic block makes the waitcnt
// pass lose count and wait vmcnt(0) at the first use, i.e. for every load in flight.  The unrolled
// kernels (L > 0) only run on 16-byte-aligned rows; the scalar form is the runtime-L kernel's.
template <typename T, int NV>
__device__ __forceinline__ void load_row_regs(T (&r)[NV][VT<T>::V], const T* __restrict__ src, int N, int nvec,
                                              bool vec_ok, bool zero) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  const int NT = blockDim.x;
  if (zero) return;  // r stays undefined; the writer substitutes zeros
  if (vec_ok) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int w = (int)threadIdx.x + k * NT;
      asm volatile("" : "+v"(w));  // not hoisted out of the level loop (see for_vecs)
      w = min(w, nvec - 1);
      const vec v = stream_load<vec>(src, w);
#pragma unroll
      for (int e = 0; e < V; ++e) r[k][e] = v[e];
    }
  } else {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      const int w = threadIdx.x + k * NT;
      if (w < nvec) {
        const int t0 = w * V;
#pragma unroll
        for (int e = 0; e < V; ++e) r[k][e] = (t0 + e < N) ? src[t0 + e] : T(0);
      }
    }
  }
}

// ---- Halo by owner writes ---------------------------------------------------------------------
// Whoever writes element t of a level input into LDS also writes the halo positions the
// reference's index map sends to t, so the halo costs no extra pass and no extra barrier.  With
// hl <= N and hr <= N an element has at most one image per side, an affine function of t:
//   periodic  (i mod N):             t - N (left), t + N (right)
//   symmetric (MathUtils mirror):    -t - 1 (left), 2N - 1 - t (right)
//   fftpad    (i + nextPow2(N) < N):  t - npow2 (left); right halo is zero
// (LevelDesc il_*/ir_*; an image is written when it falls inside [-hl, 0) / [N, N+hr)).  Only
// vectors w < vs (in the thread's first slab) or w >= ve (in its last slab) have images.
// Positions with no source (zero padding, fftpad gaps, streaming history) are written by
// halo_fixed.  When these conditions do not hold the host clears LevelDesc::own and the kernels
// fill the halo from LDS after a barrier (fill_halo), as the reference's modulo does for any index.
template <typename T>
__device__ __forceinline__ void halo_images(T* buf, int w, const typename VT<T>::v& o, int N, const LevelDesc& lv) {
  constexpr int V = VT<T>::V;
#pragma unroll
  for (int e = 0; e < V; ++e) {
    const int t = w * V + e;
    if (t < N) {
      const int l = lv.il_a * t + lv.il_b;
      const int r = lv.ir_a * t + lv.ir_b;
      if (l < 0 && l >= -lv.hl) buf[l] = o[e];
      if (r >= N && r < N + lv.hr) buf[r] = o[e];
    }
  }
}

template <typename T>
__device__ __forceinline__ void halo_fixed(T* buf, int N, const LevelDesc& lv, int npow2, const T* hist_b) {
  if (lv.mode == kHaloPeriodic || lv.mode == kHaloSymmetric) return;
  const int total = lv.hl + lv.hr;
  for (int q = threadIdx.x; q < total; q += blockDim.x) {
    const int idx = q < lv.hl ? q - lv.hl : N + (q - lv.hl);
    if (lv.mode == kHaloFftPad && idx < 0 && idx + npow2 < N) continue;  // an element's image
    T v = T(0);
    if (lv.mode == kHaloHistory && idx < 0 && idx >= -lv.hist_len) v = hist_b[lv.hist_len + idx];
    buf[idx] = v;
  }
}

// Write a register-held row into the LDS level buffer `buf` with its halo for level `lv`.
// MODE 0: values as is; 1: zeros (masked-out level, registers never loaded); 2: thresholded.
template <typename T, int L, int NV, int MODE>
__device__ __forceinline__ void regs_to_level_m(T* buf, const T (&r)[NV][VT<T>::V], int nvec, int N,
                                                const LevelDesc& lv, T thr_b, int soft) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  const bool own = lv.own != 0;
  for_vecs<L, NV>(nvec, [&](int k, int w) {
    vec o;
#pragma unroll
    for (int e = 0; e < V; ++e) {
      if constexpr (MODE == 1) {
        T z = T(0);
        asm volatile("" : "+v"(z));  // materialised here, not a loop-invariant vector held in VGPRs
        o[e] = z;
      }
      else if constexpr (MODE == 2) o[e] = threshold_t(r[k][e], thr_b, soft);
      else o[e] = r[k][e];
    }
    if (L > 0 || w * V + V <= N) {
      *reinterpret_cast<vec*>(buf + w * V) = o;
    } else {  // ragged tail: positions >= N belong to the right halo (written by their owners)
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (w * V + e < N) buf[w * V + e] = o[e];
    }
    if (own && ((k == 0 && w < lv.vs) || (k == NV - 1 && w >= lv.ve))) halo_images(buf, w, o, N, lv);
  });
}

// If the level cannot use owner writes this ends with a barrier and the generic halo fill; either
// way the caller's next lds_barrier() publishes data + halo.
template <typename T, int L, int NV>
__device__ __forceinline__ void regs_to_level(T* buf, const T (&r)[NV][VT<T>::V], int nvec, int N, const LevelDesc& lv,
                                              int npow2, const T* hist_b, bool zero = false, const T* thr = nullptr,
                                              T thr_b = T(0), int soft = 0) {
  if (zero) regs_to_level_m<T, L, NV, 1>(buf, r, nvec, N, lv, thr_b, soft);
  else if (thr) regs_to_level_m<T, L, NV, 2>(buf, r, nvec, N, lv, thr_b, soft);
  else regs_to_level_m<T, L, NV, 0>(buf, r, nvec, N, lv, thr_b, soft);
  if (lv.own) {
    halo_fixed(buf, N, lv, npow2, hist_b);
  } else {
    lds_barrier();
    fill_halo(buf, N, lv.hl, lv.hr, lv.mode, npow2, hist_b, lv.hist_len);
  }
}

// ---- Row compute: one level's convolution over the thread's NV vectors -------------------------
// Forward, both filters from one set of LDS reads; emit(k, w, al, ah) consumes each output vector.
// SC: 1 / 2 = register window for spacing 1 / 2 (the latter fp32 only), 0 = strided b128 reads.
template <typename T, int L, bool FMA, int NV, int SC, typename Emit>
__device__ __forceinline__ void fwd_row_t(const T* buf, int nvec, int s, const T* lo, const T* hi, int taps,
                                          Emit&& emit) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  for_vecs<L, NV>(nvec, [&](int k, int w) {
    const int t0 = w * V;
    T al[V], ah[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { al[e] = T(0); ah[e] = T(0); }
    if constexpr (L > 0 && SC > 0) {
      fwd_window<T, L, FMA, SC>(buf, t0, lo, hi, al, ah);
    } else if constexpr (L > 0) {
#pragma unroll
      for (int i = 0; i < L; ++i) {  // s is a multiple of V: aligned 16-byte reads
        const vec v = *reinterpret_cast<const vec*>(buf + t0 - i * s);
        vmadd<FMA, kPkFwd>(al, v, lo[i]);
        vmadd<FMA, kPkFwd>(ah, v, hi[i]);
        if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // <= 4 reads in flight (VGPR budget)
      }
    } else {
      fwd_vec<T, 0, FMA>(buf, t0, s, lo, hi, taps, al, ah);
    }
    emit(k, w, al, ah);
  });
}

template <typename T, int L, bool FMA, int NV, typename Emit>
__device__ __forceinline__ void fwd_row(const T* buf, int nvec, int s, const T* lo, const T* hi, int taps,
                                        Emit&& emit) {
  constexpr int V = VT<T>::V;
  if constexpr (L > 0) {
    if (s == 1) return fwd_row_t<T, L, FMA, NV, 1>(buf, nvec, s, lo, hi, taps, emit);
    if constexpr (V == 4) {
      if (s == 2) return fwd_row_t<T, L, FMA, NV, 2>(buf, nvec, s, lo, hi, taps, emit);
    }
  }
  fwd_row_t<T, L, FMA, NV, 0>(buf, nvec, s, lo, hi, taps, emit);
}

// Inverse, one branch over the row: acc[k]_e (+)= f[i] * buf[t0 + e + dir*i*s + off], i ascending
// (MultiLevelMODWTTransform.java:578-588 periodic, :612-639 symmetric orientations).
// SC as above; SC = -1: generic per-element form (runtime taps, or an offset that is not a
// multiple of V -- the symmetric alignment shifts).
template <typename T, int L, bool FMA, int NV, int SC, int DIR>
__device__ __forceinline__ void inv_row_t(const T* buf, int nvec, int s, int dir, int off, const T* f, int taps,
                                          T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  for_vecs<L, NV>(nvec, [&](int k, int w) {
    const int t0 = w * V;
    if constexpr (L > 0 && SC > 0) {
      inv_window<T, L, FMA, SC, DIR>(buf, t0 + off, f, acc[k]);
    } else if constexpr (L > 0 && SC == 0) {
#pragma unroll
      for (int i = 0; i < L; ++i) {
        const vec v = *reinterpret_cast<const vec*>(buf + t0 + off + DIR * i * s);
        vmadd<FMA>(acc[k], v, f[i]);
        if ((i & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // <= 4 reads in flight (VGPR budget)
      }
    } else {
      inv_branch<T, L, FMA>(buf, t0, s, dir, off, f, taps, acc[k]);
    }
    // Pin the sums here: otherwise the arithmetic is sunk to the next use of acc (the other branch,
    // after a barrier) while the LDS reads stay put, and every read value is live until then.
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(acc[k][e]));
  });
}

template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void inv_row(const T* buf, int nvec, int s, int dir, int off, const T* f, int taps,
                                        T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  if constexpr (L > 0) {
    if ((off & (V - 1)) == 0) {
      if (s == 1) {
        if (dir > 0) return inv_row_t<T, L, FMA, NV, 1, 1>(buf, nvec, s, dir, off, f, taps, acc);
        return inv_row_t<T, L, FMA, NV, 1, -1>(buf, nvec, s, dir, off, f, taps, acc);
      }
      if constexpr (V == 4) {
        if (s == 2) {
          if (dir > 0) return inv_row_t<T, L, FMA, NV, 2, 1>(buf, nvec, s, dir, off, f, taps, acc);
          return inv_row_t<T, L, FMA, NV, 2, -1>(buf, nvec, s, dir, off, f, taps, acc);
        }
      }
      if (dir > 0) return inv_row_t<T, L, FMA, NV, 0, 1>(buf, nvec, s, dir, off, f, taps, acc);
      return inv_row_t<T, L, FMA, NV, 0, -1>(buf, nvec, s, dir, off, f, taps, acc);
    }
  }
  inv_row_t<T, L, FMA, NV, -1, 1>(buf, nvec, s, dir, off, f, taps, acc);
}

template <typename T, int NV>
__device__ __forceinline__ void zero_regs(T (&r)[NV][VT<T>::V]) {
#pragma unroll
  for (int k = 0; k < NV; ++k)
#pragma unroll
    for (int e = 0; e < VT<T>::V; ++e) r[k][e] = T(0);
}

// Launch bounds of the fused kernels.  NV = 4: at most 512 threads and W waves per SIMD -- W = 8
// (64 VGPRs: four 512-thread workgroups per CU, LDS permitting) for the forward, W = 6 (80 VGPRs,
// three workgroups) for the inverse, whose prefetched detail row occupies 16 more VGPRs -- so
// several workgroups share a CU and hide each other's barriers and row loads.  NV = 8 (long
// signals): up to 1024 threads, 128 VGPRs.
// Longer filters need wider register windows (the s = 1 window holds L + V - 1 values): L <= 8 gets
// W waves, longer filters 4 (128 VGPRs; with 512-thread workgroups 5 waves would not add one).
// NV = 2 (small batches: one 1024-thread workgroup per signal, two per CU = 8 waves per SIMD, 64 VGPRs):
// twice the waves per signal where the batch leaves the CUs short of signals.
#ifndef VW_LONG_WAVES
#define VW_LONG_WAVES 4  // waves per SIMD the fused kernels of long filters (L > 8) are compiled for
#endif
#define VW_FUSED_W(L, W) ((L) <= 8 ? (W) : VW_LONG_WAVES)
#define VW_FUSED_BOUNDS(NV, W)                                                        \
  __attribute__((amdgpu_flat_work_group_size(1, ((NV) <= 4 && (NV) != 2) ? 512 : 1024), \
                 amdgpu_waves_per_eu((NV) == 2 ? 8 : (NV) <= 4 ? (W) : 4)))

// ---------------------------------------------------------------------------------------------
// Fused multi-level forward: MultiLevelMODWTTransform.decompose (:243-251) / BatchSIMDMODWT
// .batchMultiLevelMODWTSoA (:362-377) / VectorWaveSwtAdapter.decomposeSWT (:370-390) /
// BatchStreamingMODWT.processMultiLevel (:130-158) for one signal per workgroup.
//
// Level inputs alternate between two LDS buffers (p.region1 != 0): level j reads X while its
// approximation -- the input of level j+1, halo included -- is written into Y, so each level costs
// ONE workgroup barrier.  With one buffer (long signals), a second barrier guards the overwrite.
// Non-finite probe (VW_FLAG_REF_NONFINITE, vw_ref.hip): z = v * 0 + z stays +-0 while every v is finite
// and becomes NaN for good at the first NaN / +-Inf -- one FMA per value, no compare or mask in the loop.
template <typename T>
__device__ __forceinline__ T nf_step(T v, T z) {
  if constexpr (sizeof(T) == 8) return __builtin_fma(v, T(0), z);
  else return __builtin_fmaf(v, T(0), z);
}
template <typename T, int V>
__device__ __forceinline__ void nf_probe(T& z, const T (&v)[V]) {
#pragma unroll
  for (int e = 0; e < V; ++e) z = nf_step<T>(v[e], z);
}
// a row in registers (load_row_regs layout): only the vectors the thread holds (for_vecs)
template <typename T, int L, int NV, int V>
__device__ __forceinline__ void nf_probe_rows(T& z, const T (&v)[NV][V], int nvec) {
  for_vecs<L, NV>(nvec, [&](int k, int) { nf_probe<T, V>(z, v[k]); });
}
// row b flagged when any lane of any wave saw one (a plain vector store: every writer stores the same 1)
template <typename T>
__device__ __forceinline__ void nf_flag_row(int* flag, long long b, T z) {
  if (__any(z != z) && (threadIdx.x & 63) == 0) flag[b] = 1;
}

// NFP: probe the final approximation (nf: the row's accumulator, see nf_probe)
template <typename T, int L, bool FMA, int NV, bool VALIDATE, bool NFP = false>
__device__ __forceinline__ void fwd_level(const FwdArgs<T>& p, const T* X, int nvec, const LevelDesc& lv, T* dout,
                                          T* aout, bool vec_ok, unsigned long long flat0, T (&areg)[NV][VT<T>::V],
                                          T* nf = nullptr) {
  constexpr int V = VT<T>::V;
  const int N = p.N;
  fwd_row<T, L, FMA, NV>(X, nvec, lv.s, p.lo, p.hi, p.taps, [&](int k, int w, const T (&al)[V], const T (&ah)[V]) {
    const int t0 = w * V;
    store_vec<VW_FWD_STORE_AUX>(dout, t0, N, vec_ok, ah);
    if (aout) store_vec<VW_FWD_STORE_AUX>(aout, t0, N, vec_ok, al);
    if constexpr (VALIDATE) {
      check_out<T>(1, p.bad, flat0, t0, N, ah);
      check_out<T>(1, p.bad, flat0, t0, N, al);
    }
    if constexpr (NFP) {
      if (aout) nf_probe<T, V>(*nf, al);  // a_J suffices (k_forward_persist; vw_ref.hip)
    }
#pragma unroll
    for (int e = 0; e < V; ++e) areg[k][e] = al[e];
  });
}

// HIST: streaming history halos (kHaloHistory) possible.  The history is the only global load inside
// the level loop; without it (HIST = false) no load can be pending there, so the waitcnt pass never
// waits vmcnt(0) -- which on gfx950 would also wait for every detail store still in flight.
template <typename T, int L, bool FMA, int NV, bool HIST>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, 8)) k_forward_fused(const FwdArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* X = reinterpret_cast<T*>(smem) + p.hlpad;
  T* Y = p.region1 ? reinterpret_cast<T*>(smem) + p.region1 + p.hlpad : X;
  const bool dbl = p.region1 != 0;
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const int N = p.N;
  const int nvec = (N + V - 1) / V;
  const int NT = blockDim.x;
  const int tid = threadIdx.x;
  const bool vec_ok = (L > 0) || p.vec_io != 0;  // unrolled kernels run with aligned rows only
  const unsigned long long flat0 = (unsigned long long)b * (unsigned long long)N;
  auto hist_of = [&](int j) -> const T* {  // level j's streaming history row (or nullptr)
    if constexpr (!HIST) return nullptr;
    const LevelDesc& d = p.lv[j - 1];
    return d.mode == kHaloHistory ? p.hist[j - 1] + b * d.hist_len : nullptr;
  };

  T areg[NV][V];
  load_row_regs<T, NV>(areg, p.x + b * p.ldx, N, nvec, vec_ok, false);
  wait_vmem();
  if (p.validate) {
    for_vecs<L, NV>(nvec, [&](int k, int w) {
#pragma unroll
      for (int e = 0; e < V; ++e)
        if (w * V + e < N && !finite_t(areg[k][e])) atomicMin(p.bad, flat0 + (unsigned long long)(w * V + e));
    });
  }
  regs_to_level<T, L, NV>(X, areg, nvec, N, p.lv[0], p.npow2, hist_of(1));

  for (int j = 1; j <= p.J; ++j) {
    const LevelDesc lv = p.lv[j - 1];
    lds_barrier();  // X = level input + halo; every read of Y (previous level) done
    T* dout = p.details + ((size_t)(j - 1) * (size_t)p.B + (size_t)b) * (size_t)N;
    T* aout = (j == p.J) ? p.approx + b * (size_t)N : nullptr;
    if (p.validate) fwd_level<T, L, FMA, NV, true>(p, X, nvec, lv, dout, aout, vec_ok, flat0, areg);
    else fwd_level<T, L, FMA, NV, false>(p, X, nvec, lv, dout, aout, vec_ok, flat0, areg);
    // Streaming: new left history = last hist_len samples of this level's input
    // (BatchStreamingMODWT.updateHistoryFromSoA :337-352).
    if (HIST && p.hist_update && lv.hist_len > 0) {
      T* hnew = p.hist[j - 1] + b * lv.hist_len;
      for (int q = tid; q < lv.hist_len; q += NT) hnew[q] = X[q + N - lv.hist_len];
    }
    if (j < p.J) {
      if (!dbl) lds_barrier();  // one buffer: every read of this level's input done first
      regs_to_level<T, L, NV>(Y, areg, nvec, N, p.lv[j], p.npow2, hist_of(j + 1));
      T* t = X; X = Y; Y = t;
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Persistent fused forward: the same cascade as k_forward_fused, but each workgroup walks the
// signals b = blockIdx.x, + gridDim.x, ... and copies the NEXT signal's row into LDS while the
// current one computes its last level.  With two level buffers, level J reads X and writes no next
// level, so the other buffer is free from its first barrier on: the row goes there by LDS-DMA
// (global_load_lds_dwordx4, no VGPRs), overlapping the read of x with level J's arithmetic and
// detail stores instead of starting every signal with an exposed load (one workgroup per signal
// waits for its row before any store can be issued; at 2 workgroups per CU both often wait at once).
//
// The DMA is issued from inline asm so the compiler does not pessimistically wait for it before the
// LDS reads of level J (it cannot prove the buffers disjoint).  Completion is waited for explicitly:
// vmcnt counts a wave's vector-memory operations in issue order, and exactly 2*NV stores (detail +
// approximation rows) follow the DMA, so vmcnt(2*NV) retires the DMA and leaves those stores in
// flight.  Host contract (vw_capi.cpp): two buffers, every slab full (threads*NV == N/V), whole
// waves, N/V a multiple of 64 (one wave instruction = 64 x 16 B), no validation, no history.
// One wave instruction of LDS-DMA: 64 lanes x 16 bytes from per-lane global addresses into 1 KiB of
// LDS at the wave-uniform byte address `lds` (global_load_lds_dwordx4; no VGPR is written).  nt: the
// non-temporal cache policy (a row read once by this launch need not be kept in L2 / Infinity Cache).
// Issued from inline asm so the compiler's waitcnt pass does not wait for it before unrelated LDS
// reads; the caller retires it with an explicit vmcnt wait.
__device__ __forceinline__ void lds_dma16(unsigned lds, const void* g, bool nt) {
  unsigned keep;
  if (nt) {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off nt\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds))
        : "memory");
  } else {
    asm volatile(
        "s_mov_b32 %0, m0\n\t"
        "s_mov_b32 m0, %2\n\t"
        "s_nop 0\n\t"
        "global_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(g), "s"(__builtin_amdgcn_readfirstlane(lds))
        : "memory");
  }
}

template <typename T>
__device__ __forceinline__ void dma_row(T* buf, const T* __restrict__ src, int nvec, bool nt) {
  constexpr int V = VT<T>::V;
  const int lane = threadIdx.x & 63, wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), nw = blockDim.x >> 6;
  for (int c = wv; c * 64 < nvec; c += nw)
    lds_dma16((unsigned)(uintptr_t)(buf + c * 64 * V), src + (size_t)(c * 64 + lane) * V, nt);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() {
  static_assert(N >= 0 && N < 64, "vmcnt range");
  __builtin_amdgcn_s_waitcnt((N & 0xF) | ((N >> 4) << 14) | (0x7 << 4) | (0xF << 8));
}

// vmcnt(n) for a wave-uniform runtime n (0..63; larger waits for 63, i.e. for more)
__device__ __forceinline__ void wait_vmcnt_rt(int n) {
  // the count is wave-uniform; without this the switch compiles to an exec-masked compare tree on a VGPR
  switch (__builtin_amdgcn_readfirstlane(n)) {
    case 0: wait_vmcnt<0>(); break;
    case 1: wait_vmcnt<1>(); break;
    case 2: wait_vmcnt<2>(); break;
    case 3: wait_vmcnt<3>(); break;
    case 4: wait_vmcnt<4>(); break;
    case 5: wait_vmcnt<5>(); break;
    case 6: wait_vmcnt<6>(); break;
    case 7: wait_vmcnt<7>(); break;
    case 8: wait_vmcnt<8>(); break;
    case 9: wait_vmcnt<9>(); break;
    case 10: wait_vmcnt<10>(); break;
    case 11: wait_vmcnt<11>(); break;
    case 12: wait_vmcnt<12>(); break;
    case 13: wait_vmcnt<13>(); break;
    case 14: wait_vmcnt<14>(); break;
    case 15: wait_vmcnt<15>(); break;
    case 16: wait_vmcnt<16>(); break;
    case 17: wait_vmcnt<17>(); break;
    case 18: wait_vmcnt<18>(); break;
    case 19: wait_vmcnt<19>(); break;
    case 20: wait_vmcnt<20>(); break;
    case 21: wait_vmcnt<21>(); break;
    case 22: wait_vmcnt<22>(); break;
    case 23: wait_vmcnt<23>(); break;
    case 24: wait_vmcnt<24>(); break;
    case 25: wait_vmcnt<25>(); break;
    case 26: wait_vmcnt<26>(); break;
    case 27: wait_vmcnt<27>(); break;
    case 28: wait_vmcnt<28>(); break;
    case 29: wait_vmcnt<29>(); break;
    case 30: wait_vmcnt<30>(); break;
    case 31: wait_vmcnt<31>(); break;
    case 32: wait_vmcnt<32>(); break;
    case 33: wait_vmcnt<33>(); break;
    case 34: wait_vmcnt<34>(); break;
    case 35: wait_vmcnt<35>(); break;
    case 36: wait_vmcnt<36>(); break;
    case 37: wait_vmcnt<37>(); break;
    case 38: wait_vmcnt<38>(); break;
    case 39: wait_vmcnt<39>(); break;
    case 40: wait_vmcnt<40>(); break;
    case 41: wait_vmcnt<41>(); break;
    case 42: wait_vmcnt<42>(); break;
    case 43: wait_vmcnt<43>(); break;
    case 44: wait_vmcnt<44>(); break;
    case 45: wait_vmcnt<45>(); break;
    case 46: wait_vmcnt<46>(); break;
    case 47: wait_vmcnt<47>(); break;
    case 48: wait_vmcnt<48>(); break;
    case 49: wait_vmcnt<49>(); break;
    case 50: wait_vmcnt<50>(); break;
    case 51: wait_vmcnt<51>(); break;
    case 52: wait_vmcnt<52>(); break;
    case 53: wait_vmcnt<53>(); break;
    case 54: wait_vmcnt<54>(); break;
    case 55: wait_vmcnt<55>(); break;
    case 56: wait_vmcnt<56>(); break;
    case 57: wait_vmcnt<57>(); break;
    case 58: wait_vmcnt<58>(); break;
    case 59: wait_vmcnt<59>(); break;
    case 60: wait_vmcnt<60>(); break;
    case 61: wait_vmcnt<61>(); break;
    case 62: wait_vmcnt<62>(); break;
    case 63: wait_vmcnt<63>(); break;
    default: wait_vmcnt<63>(); break;
  }
}

template <typename T, int L, bool FMA, int NV>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, NV <= 4 ? 512 : 1024), amdgpu_waves_per_eu(4)))
k_forward_persist(const FwdArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* const B0 = reinterpret_cast<T*>(smem) + p.hlpad;  // (no pointer array: it would lose the LDS address space)
  T* const B1 = reinterpret_cast<T*>(smem) + p.region1 + p.hlpad;
  const int N = p.N;
  const int nvec = N / V;
  const long long G = gridDim.x;
  long long b = blockIdx.x;
  if (b >= p.B) return;
  int cur = 0;
  T nf = T(0);
  dma_row<T>(B0, p.x + b * p.ldx, nvec, p.dma_nt != 0);
  wait_vmem();
  for (;;) {
    T* X = cur ? B1 : B0;
    T* Y = cur ? B0 : B1;
    lds_barrier();  // the row is in X (every wave's share); every read of the previous signal done
    const LevelDesc lv0 = p.lv[0];
    fill_halo(X, N, lv0.hl, lv0.hr, lv0.mode, p.npow2, (const T*)nullptr, 0);
    const long long bn = b + G;
    T areg[NV][V];
    for (int j = 1; j <= p.J; ++j) {
      const LevelDesc lv = p.lv[j - 1];
      lds_barrier();  // X = level input + halo; every read of Y (previous level) done
      if (j == p.J && bn < p.B) {
        dma_row<T>(Y, p.x + bn * p.ldx, nvec, p.dma_nt != 0);  // next signal -> free buffer
      }
      T* dout = p.details + ((size_t)(j - 1) * (size_t)p.B + (size_t)b) * (size_t)N;
      T* aout = (j == p.J) ? p.approx + b * (size_t)N : nullptr;
      if (p.nf_flag) fwd_level<T, L, FMA, NV, false, true>(p, X, nvec, lv, dout, aout, true, 0ull, areg, &nf);
      else fwd_level<T, L, FMA, NV, false>(p, X, nvec, lv, dout, aout, true, 0ull, areg);
      if (j < p.J) {
        regs_to_level<T, L, NV>(Y, areg, nvec, N, p.lv[j], p.npow2, (const T*)nullptr);
        T* t = X; X = Y; Y = t;
      }
    }
    // VW_FLAG_REF_NONFINITE: probing a_J flags every row vw_ref.hip must recompute (see there)
    if (p.nf_flag) {
      nf_flag_row<T>(p.nf_flag, b, nf);
      nf = T(0);
    }
    if (bn >= p.B) break;
    wait_vmcnt<2 * NV>();  // this wave's DMA share landed; level J's stores stay in flight
    cur = (cur + p.J) & 1;  // the buffer that was free during level J
    b = bn;
  }
}

// ---------------------------------------------------------------------------------------------
// Fused multi-level inverse: MultiLevelMODWTTransform.reconstruct (:339-349, :554-645),
// VectorWaveSwtAdapter.reconstructPeriodic (:444-474), MODWTTransform.inverse (J=1, pairwise),
// with the denoise threshold (MutableMultiLevelMODWTResult.java:97-114) fused into the detail load.
//
// Pairwise form (sum += h*a + g*d per tap): a_j and d_j in two LDS regions.
template <typename T, int L, bool FMA, int NV>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, 6)) k_inverse_fused(const InvArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* A = reinterpret_cast<T*>(smem) + p.hlpad_a;
  T* D = reinterpret_cast<T*>(smem) + p.region_d + p.hlpad_d;
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const int N = p.N;
  const int nvec = (N + V - 1) / V;
  const bool vec_ok = (L > 0) || p.vec_io != 0;
  // threshold of level j (denoise): thr[(j-1)*thr_ld + b]; thr_ld = 0 -> one threshold for every level
  auto thr_of = [&](int j) { return p.thr ? load_uniform(p.thr + (size_t)(j - 1) * (size_t)p.thr_ld + (size_t)b) : T(0); };
  const size_t plane = (size_t)p.B * (size_t)N;

  T reg[NV][V];
  T dnext[NV][V];
  // coarsest level: approximation -> A, d_J -> D
  load_row_regs<T, NV>(reg, p.approx + b * (size_t)N, N, nvec, vec_ok, p.approx_zero != 0);
  load_row_regs<T, NV>(dnext, p.details + (size_t)(p.J - 1) * plane + b * (size_t)N, N, nvec, vec_ok,
                       p.lv[p.J - 1].use_d == 0);
  wait_vmem();
  regs_to_level<T, L, NV>(A, reg, nvec, N, p.lv[p.J - 1], 0, (const T*)nullptr, p.approx_zero != 0);
  regs_to_level<T, L, NV>(D, dnext, nvec, N, p.lv[p.J - 1], 0, (const T*)nullptr, p.lv[p.J - 1].use_d == 0, p.thr,
                          thr_of(p.J), p.soft);

  for (int j = p.J; j >= 1; --j) {
    const LevelDesc lv = p.lv[j - 1];
    lds_barrier();  // A (level-j approximation) and D (d_j) complete, halos included
    if (j > 1) {    // prefetch d_{j-1} while this level computes
      load_row_regs<T, NV>(dnext, p.details + (size_t)(j - 2) * plane + b * (size_t)N, N, nvec, vec_ok,
                           p.lv[j - 2].use_d == 0);
    }
    for_vecs<L, NV>(nvec, [&](int k, int w) {
      T acc[V];
#pragma unroll
      for (int e = 0; e < V; ++e) acc[e] = T(0);
      inv_pair<T, L, FMA>(A, D, w * V, lv.s, lv.dir_a, p.lo, p.hi, p.taps, acc);
#pragma unroll
      for (int e = 0; e < V; ++e) {
        asm volatile("" : "+v"(acc[e]));  // pin the sum here (see inv_row_t)
        reg[k][e] = acc[e];
      }
    });
    if (j == 1) {
      for_vecs<L, NV>(nvec, [&](int k, int w) { store_vec<VW_INV_STORE_AUX>(p.y + b * (size_t)N, w * V, N, vec_ok, reg[k]); });
    } else {
      const LevelDesc ln = p.lv[j - 2];
      lds_barrier();  // all reads of A and D done
      regs_to_level<T, L, NV>(A, reg, nvec, N, ln, 0, (const T*)nullptr);
      wait_vmem();  // the d_{j-1} prefetch
      regs_to_level<T, L, NV>(D, dnext, nvec, N, ln, 0, (const T*)nullptr, ln.use_d == 0, p.thr, thr_of(j - 1), p.soft);
    }
  }
}

// Sequential-sum form (PERIODIC K4 / SYMMETRIC K6: all approximation taps, then all detail taps,
// into one accumulator), double-buffered: X holds a_j, Y holds d_j.  Per level:
//   barrier -> stage d_j (prefetched last level) into Y, prefetch d_{j-1} -> approx branch on X
//   -> barrier -> detail branch on Y -> a_{j-1} into X
// i.e. two workgroup barriers per level, and d_{j-1}'s loads have a whole level to land.
template <typename T, int L, bool FMA, int NV>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, 6)) k_inverse_db(const InvArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* const X = reinterpret_cast<T*>(smem) + p.hlpad_a;
  T* const Y = reinterpret_cast<T*>(smem) + p.region_d + p.hlpad_d;
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const int N = p.N;
  const int nvec = (N + V - 1) / V;
  const bool vec_ok = (L > 0) || p.vec_io != 0;
  // threshold of level j (denoise): thr[(j-1)*thr_ld + b]; thr_ld = 0 -> one threshold for every level
  auto thr_of = [&](int j) { return p.thr ? load_uniform(p.thr + (size_t)(j - 1) * (size_t)p.thr_ld + (size_t)b) : T(0); };
  const size_t plane = (size_t)p.B * (size_t)N;

  T acc[NV][V];
  T dreg[NV][V];
  load_row_regs<T, NV>(acc, p.approx + b * (size_t)N, N, nvec, vec_ok, p.approx_zero != 0);
  load_row_regs<T, NV>(dreg, p.details + (size_t)(p.J - 1) * plane + b * (size_t)N, N, nvec, vec_ok,
                       p.lv[p.J - 1].use_d == 0);
  wait_vmem();
  regs_to_level<T, L, NV>(X, acc, nvec, N, p.lv[p.J - 1], 0, (const T*)nullptr, p.approx_zero != 0);

  for (int j = p.J; j >= 1; --j) {
    const LevelDesc lv = p.lv[j - 1];
    lds_barrier();  // X = a_j + halo; every read of Y (previous level) done
    wait_vmem();    // the d_j prefetch (the only global ops in flight)
    regs_to_level<T, L, NV>(Y, dreg, nvec, N, lv, 0, (const T*)nullptr, lv.use_d == 0, p.thr, thr_of(j), p.soft);
    if (j > 1)
      load_row_regs<T, NV>(dreg, p.details + (size_t)(j - 2) * plane + b * (size_t)N, N, nvec, vec_ok,
                           p.lv[j - 2].use_d == 0);
    zero_regs<T, NV>(acc);
    inv_row<T, L, FMA, NV>(X, nvec, lv.s, lv.dir_a, lv.off_a, p.lo, p.taps, acc);
    lds_barrier();  // Y = d_j + halo; every read of X done
    inv_row<T, L, FMA, NV>(Y, nvec, lv.s, lv.dir_d, lv.off_d, p.hi, p.taps, acc);
    if (j > 1) regs_to_level<T, L, NV>(X, acc, nvec, N, p.lv[j - 2], 0, (const T*)nullptr);
  }
  for_vecs<L, NV>(nvec, [&](int k, int w) { store_vec<VW_INV_STORE_AUX>(p.y + b * (size_t)N, w * V, N, vec_ok, acc[k]); });
}

// Single-buffer sequential-sum form for signals too long for two LDS buffers: ONE region is
// time-shared (a_j -> approx branch -> d_j -> detail branch -> a_{j-1}); four barriers per level.
#ifndef VW_INV_LATE_PF
#define VW_INV_LATE_PF 0
#endif
#ifndef VW_INV_W
#define VW_INV_W 6  // waves per SIMD of k_inverse_seq (experiment builds: -DVW_INV_W=8 -> 64 VGPRs)
#endif
template <typename T, int L, bool FMA, int NV>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, VW_INV_W)) k_inverse_seq(const InvArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* R = reinterpret_cast<T*>(smem) + p.hlpad_a;
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const int N = p.N;
  const int nvec = (N + V - 1) / V;
  const bool vec_ok = (L > 0) || p.vec_io != 0;
  // threshold of level j (denoise): thr[(j-1)*thr_ld + b]; thr_ld = 0 -> one threshold for every level
  auto thr_of = [&](int j) { return p.thr ? load_uniform(p.thr + (size_t)(j - 1) * (size_t)p.thr_ld + (size_t)b) : T(0); };
  const size_t plane = (size_t)p.B * (size_t)N;

  T acc[NV][V];
  T dreg[NV][V];
  // VW_FLAG_REF_NONFINITE: probing y flags every row vw_ref.hip must recompute (see there)
  T nf = T(0);
  const bool nfp = p.nf_flag != nullptr;
  load_row_regs<T, NV>(acc, p.approx + b * (size_t)N, N, nvec, vec_ok, p.approx_zero != 0);
  load_row_regs<T, NV>(dreg, p.details + (size_t)(p.J - 1) * plane + b * (size_t)N, N, nvec, vec_ok,
                       p.lv[p.J - 1].use_d == 0);
  wait_vmem();
  regs_to_level<T, L, NV>(R, acc, nvec, N, p.lv[p.J - 1], 0, (const T*)nullptr, p.approx_zero != 0);

  for (int j = p.J; j >= 1; --j) {
    const LevelDesc lv = p.lv[j - 1];
    lds_barrier();  // R = a_j + halo
#if VW_INV_LATE_PF
    // (experiment) d_j issued at the start of level j, live only across the approximation branch
    if (j < p.J)
      load_row_regs<T, NV>(dreg, p.details + (size_t)(j - 1) * plane + b * (size_t)N, N, nvec, vec_ok,
                           lv.use_d == 0);
#endif
    zero_regs<T, NV>(acc);
    inv_row<T, L, FMA, NV>(R, nvec, lv.s, lv.dir_a, lv.off_a, p.lo, p.taps, acc);
    lds_barrier();  // every approximation-branch read done
    wait_vmem();    // the d_j prefetch
    regs_to_level<T, L, NV>(R, dreg, nvec, N, lv, 0, (const T*)nullptr, lv.use_d == 0, p.thr, thr_of(j), p.soft);
#if !VW_INV_LATE_PF
    if (j > 1)
      load_row_regs<T, NV>(dreg, p.details + (size_t)(j - 2) * plane + b * (size_t)N, N, nvec, vec_ok,
                           p.lv[j - 2].use_d == 0);
#endif
    lds_barrier();  // R = d_j + halo
    inv_row<T, L, FMA, NV>(R, nvec, lv.s, lv.dir_d, lv.off_d, p.hi, p.taps, acc);
    if (j > 1) {
      lds_barrier();  // every detail-branch read done
      regs_to_level<T, L, NV>(R, acc, nvec, N, p.lv[j - 2], 0, (const T*)nullptr);
    }
  }
  for_vecs<L, NV>(nvec, [&](int k, int w) { store_vec<VW_INV_STORE_AUX>(p.y + b * (size_t)N, w * V, N, vec_ok, acc[k]); });
  if (nfp) {
    nf_probe_rows<T, L, NV, V>(nf, acc, nvec);
    nf_flag_row<T>(p.nf_flag, b, nf);
  }
}

// ---------------------------------------------------------------------------------------------
// Register-blocked PERIODIC kernels for long filters (L > 8: sym8, coif5, ...).  At a level with
// spacing s >= V (vector stride m = s/V) a thread owns the NV output vectors vb, vb+m, .., vb+(NV-1)m
// of a block of m columns; they read the same input vectors shifted by one tap, so a branch costs
// NV+L-1 LDS reads instead of NV*L (33 vs 120 at L = 30): the per-level LDS read traffic, which bounds
// the one-vector-per-tap kernels for long filters, drops ~3.6x.  The block mapping alone would put
// 4..16 lanes of one ds_read_b128 lane group on the same banks, so every level input is written into
// LDS in a padded layout chosen for that level -- NV = 4: one pad vector per 4 (m <= 4), two per 8
// (m = 8); NV = 8: one per 8 (m <= 8); none for m >= 16 -- under which the reads are conflict-free
// (modelled with the gfx950 lane groups of the microarchitecture guide's LDS table).  Levels with
// s < V run the register-window code in the standard mapping.  Per output the taps run i ascending
// (forward: ScalarOps.java:707-719; inverse: approximation branch then detail branch,
// MultiLevelMODWTTransform.java:576-589): the reference's sums bit for bit in EXACT mode.
struct BlkLayout {
  int sh, pad;  // logical vector u -> u + (u >> sh) * pad
};

// tight (host: the standard layout does not fit LDS, e.g. sym8 at N = 16384): NV = 8 pads one
// vector per 16 -- 6 % of LDS instead of 12.5 %, 1.3-2x the conflict-free cycles, still 3-4x fewer
// than the one-vector-per-tap reads.
__device__ __forceinline__ BlkLayout blk_layout(int m, int nv, int tight = 0) {
  if (m <= 0 || m >= 16) return BlkLayout{30, 0};
  if (nv >= 8) return tight ? BlkLayout{4, 1} : BlkLayout{3, 1};
  if (m == 8) return BlkLayout{3, 2};
  return BlkLayout{2, 1};
}

__device__ __forceinline__ int blk_phys(const BlkLayout& lo, int u) { return u + (u >> lo.sh) * lo.pad; }

template <typename T>
__device__ __forceinline__ void blk_store(T* R, const BlkLayout& lo, int u, const typename VT<T>::v& o) {
  *reinterpret_cast<typename VT<T>::v*>(R + blk_phys(lo, u) * VT<T>::V) = o;
}

// thread tid's block base at vector stride m (NV vectors per column)
template <int NV>
__device__ __forceinline__ int blk_base(int m) {
  const int tid = threadIdx.x;
  return (tid / m) * (m * NV) + tid % m;
}

// Tap chunk of the blocked kernels: 8, or 4 where NV = 8 fp64 accumulators already take 32-64 VGPRs
// (1024-thread workgroups cap a lane at 128 VGPRs; 8-tap chunks spilled there).
template <typename T, int NV>
constexpr int blk_chunk() { return (NV >= 8 && sizeof(T) == 8) ? 4 : kWinTaps; }

// One branch of the inverse (reads t + i*s): acc[r] (+)= f[i] * in[vb + (r+i)m], i ascending per r.
// Taps in chunks of kWinTaps (each re-read at its start): NV+TC-1 reads per chunk, the chunk's taps
// the only ones live.
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_inv_branch(const T* R, const BlkLayout& lo, int vb, int m, const T* f,
                                               T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  constexpr int TC = blk_chunk<T, NV>();
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fc[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) fc[i - I0] = f[i];
#pragma unroll
    for (int q = I0; q < I1 + NV - 1; ++q) {
      const vec x = *reinterpret_cast<const vec*>(R + blk_phys(lo, vb + q * m) * V);
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = q - r;
        if (i >= I0 && i < I1) {
          vmadd<FMA>(acc[r], x, fc[i - I0]);
        }
      }
      if (((q - I0) & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(acc[r][e]));  // pin the sums (see inv_row_t)
}

// Compile-time form of blk_layout at vector stride M (NV outputs per column, TIGHT: blk_tight).  A
// thread's block base vb = (tid/M)*M*NV + tid%M; when M*NV is a multiple of the pad group 2^SH, the
// physical offset of logical vector vb + q*M from vb's is off(q) for every thread, so the branch
// reads at immediate offsets from one base address instead of computing u + (u >> SH)*PAD per read.
template <int M, int NV, int TIGHT>
struct BlkC {
  static constexpr int SH = (M >= 16) ? 30 : (NV >= 8 ? (TIGHT ? 4 : 3) : (M == 8 ? 3 : 2));
  static constexpr int PAD = (M >= 16) ? 0 : (NV >= 8 ? 1 : (M == 8 ? 2 : 1));
  static constexpr bool ok = PAD == 0 || (M * NV) % (1 << SH) == 0;
  static constexpr int off(int q) { return q * M + ((q * M) >> SH) * PAD; }
};

// blk_inv_branch at a compile-time stride: Rb = R + blk_phys(layout, vb) * V
template <typename T, int L, bool FMA, int NV, int M, int TIGHT>
__device__ __forceinline__ void blk_inv_branch_c(const T* Rb, const T* f, T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  using C = BlkC<M, NV, TIGHT>;
  constexpr int TC = blk_chunk<T, NV>();
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fc[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) fc[i - I0] = f[i];
#pragma unroll
    for (int q = I0; q < I1 + NV - 1; ++q) {
      const vec x = *reinterpret_cast<const vec*>(Rb + C::off(q) * V);
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = q - r;
        if (i >= I0 && i < I1) {
          vmadd<FMA>(acc[r], x, fc[i - I0]);
        }
      }
      if (((q - I0) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(acc[r][e]));
}

// blk_inv_branch with wave-uniform offsets: under the same condition as BlkC::ok (the pad groups
// align with a thread's block), the physical offset of logical vector vb + q*m from vb's is
// q*m + ((q*m) >> sh)*pad for every thread -- a scalar value per read, so a read costs one vector
// add (base + scalar offset) instead of the per-lane shift / multiply / add of blk_phys.  One code
// copy for every stride (the compile-time forms, one copy per m, measured slower at NV = 8).
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_inv_branch_s(const T* Rb, int m, int sh, int pad, const T* f,
                                                 T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  constexpr int TC = blk_chunk<T, NV>();
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fc[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) fc[i - I0] = f[i];
#pragma unroll
    for (int q = I0; q < I1 + NV - 1; ++q) {
      const int qm = __builtin_amdgcn_readfirstlane(q * m);
      const int off = __builtin_amdgcn_readfirstlane(qm + (qm >> sh) * pad);
      const vec x = *reinterpret_cast<const vec*>(Rb + off * V);
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = q - r;
        if (i >= I0 && i < I1) {
          vmadd<FMA>(acc[r], x, fc[i - I0]);
        }
      }
      if (((q - I0) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(acc[r][e]));
}

#ifndef VW_BLK_SOFF
#define VW_BLK_SOFF 1  // NV = 8 inverse branch: wave-uniform offsets where the layout allows (0: per-lane blk_phys)
#endif
#ifndef VW_BLK_CK8
#define VW_BLK_CK8 1  // NV = 8 blocked inverse (FMA) at m = 1..64: immediate LDS offsets off one laundered base
                      // (the same for k_forward_blk measured slower: forward 4.92-4.97 vs 4.78-4.85 ms, sym8)
#endif

// blk_inv_branch_c with the base laundered into a 32-bit LDS address (lds_base): every read is one
// ds_read_b128 at an immediate offset -- no per-read scalar offset arithmetic (blk_inv_branch_s: four SALU
// and one VALU per read) and no re-based 64-bit pointers.
template <typename T, int L, bool FMA, int NV, int M, int TIGHT>
__device__ __forceinline__ void blk_inv_branch_cl(const T* Rb, const T* f, T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  using C = BlkC<M, NV, TIGHT>;
  constexpr int TC = blk_chunk<T, NV>();
  const unsigned ab = lds_base(Rb);
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fc[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) fc[i - I0] = f[i];
#pragma unroll
    for (int q = I0; q < I1 + NV - 1; ++q) {
      const vec x = lds_vec_at<vec>(ab + (unsigned)(C::off(q) * V * (int)sizeof(T)));
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = q - r;
        if (i >= I0 && i < I1) {
          vmadd<FMA>(acc[r], x, fc[i - I0]);
        }
      }
      if (((q - I0) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) asm volatile("" : "+v"(acc[r][e]));
}

// One inverse branch at vector stride m >= 1: the compile-time forms for m = 1..64 (immediate LDS
// offsets stay below 64 KiB for L <= 30), the generic one otherwise.  Same reads, same sums.
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_inv_any(const T* R, const BlkLayout& lo, int tight, int vb, int m, const T* f,
                                            T (&acc)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  if constexpr (NV >= 8) {
    // compile-time forms through plain pointers measured slower at NV = 8 (sym8 fp64 inverse 7.18 -> 8.08 ms,
    // profiles/r03/ab_sym8_cinv.log); off a laundered 32-bit base (blk_inv_branch_cl) they win: 6.32-6.38
    // -> 6.17-6.28 ms (profiles/r05/ab_sym8_inverse_ck8.log)
    const int sh = __builtin_amdgcn_readfirstlane(lo.sh), pad = __builtin_amdgcn_readfirstlane(lo.pad);
    if constexpr (VW_BLK_CK8 != 0 && FMA) {
      // m = 1..64 where the pad group (8 vectors, or 16 in the tight layout) divides a thread's 8m-vector
      // block (BlkC::ok) or there is none (m >= 16): the offset of vb + q*m from vb is the same for every
      // lane.  FMA only: the EXACT kernel (mul + add per tap) spills 28 B/lane at its 128-VGPR cap with it.
      const T* Rb = R + blk_phys(lo, vb) * V;
      const int sel = (m == 1 || m == 2 || m == 4 || m == 8) && pad == 1 ? m * 2 + (tight ? 1 : 0)
                      : (m == 16 || m == 32 || m == 64) && pad == 0 ? 4 * m : 0;
      switch (sel) {
        case 2: blk_inv_branch_cl<T, L, FMA, NV, 1, 0>(Rb, f, acc); return;
        // (m = 1 in the tight layout: a thread's 8-vector block is half a 16-vector pad group -- per lane)
        case 4: blk_inv_branch_cl<T, L, FMA, NV, 2, 0>(Rb, f, acc); return;
        case 5: blk_inv_branch_cl<T, L, FMA, NV, 2, 1>(Rb, f, acc); return;
        case 8: blk_inv_branch_cl<T, L, FMA, NV, 4, 0>(Rb, f, acc); return;
        case 9: blk_inv_branch_cl<T, L, FMA, NV, 4, 1>(Rb, f, acc); return;
        case 16: blk_inv_branch_cl<T, L, FMA, NV, 8, 0>(Rb, f, acc); return;
        case 17: blk_inv_branch_cl<T, L, FMA, NV, 8, 1>(Rb, f, acc); return;
        case 64: blk_inv_branch_cl<T, L, FMA, NV, 16, 0>(Rb, f, acc); return;   // m >= 16: natural layout
        case 128: blk_inv_branch_cl<T, L, FMA, NV, 32, 0>(Rb, f, acc); return;
        case 256: blk_inv_branch_cl<T, L, FMA, NV, 64, 0>(Rb, f, acc); return;
        default: break;
      }
    }
    if (VW_BLK_SOFF && (pad == 0 || ((m * NV) & ((1 << sh) - 1)) == 0))
      blk_inv_branch_s<T, L, FMA, NV>(R + blk_phys(lo, vb) * V, m, sh, pad, f, acc);
    else
      blk_inv_branch<T, L, FMA, NV>(R, lo, vb, m, f, acc);
  } else {
    const T* Rb = R + blk_phys(lo, vb) * V;
    auto go = [&](auto mc, auto tc) __attribute__((always_inline)) {
      constexpr int M = decltype(mc)::value, TT = decltype(tc)::value;
      if constexpr (BlkC<M, NV, TT>::ok) blk_inv_branch_c<T, L, FMA, NV, M, TT>(Rb, f, acc);
      else blk_inv_branch<T, L, FMA, NV>(R, lo, vb, m, f, acc);
    };
    auto go_m = [&](auto mc) __attribute__((always_inline)) { go(mc, std::integral_constant<int, 0>{}); };
    (void)tight;  // the tight layout exists only at NV >= 8
    switch (m) {
      case 1: go_m(std::integral_constant<int, 1>{}); break;
      case 2: go_m(std::integral_constant<int, 2>{}); break;
      case 4: go_m(std::integral_constant<int, 4>{}); break;
      case 8: go_m(std::integral_constant<int, 8>{}); break;
      case 16: go_m(std::integral_constant<int, 16>{}); break;
      case 32: go_m(std::integral_constant<int, 32>{}); break;
      case 64: go_m(std::integral_constant<int, 64>{}); break;
      default: blk_inv_branch<T, L, FMA, NV>(R, lo, vb, m, f, acc); break;
    }
  }
}

// The forward (reads t - i*s, both filters from one set of reads): within a tap chunk q runs down so
// that for every output r the tap i = r - q ascends; chunks ascend.  Input vector u sits at logical
// u + HLV.
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_fwd(const T* X, const BlkLayout& lo, int HLV, int vb, int m, const T* flo,
                                        const T* fhi, T (&al)[NV][VT<T>::V], T (&ah)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  constexpr int TC = blk_chunk<T, NV>();
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) { al[r][e] = T(0); ah[r][e] = T(0); }
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fl[I1 - I0], fh[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) { fl[i - I0] = flo[i]; fh[i - I0] = fhi[i]; }
#pragma unroll
    for (int q = NV - 1 - I0; q > -I1; --q) {
      const vec x = *reinterpret_cast<const vec*>(X + blk_phys(lo, vb + q * m + HLV) * V);
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = r - q;
        if (i >= I0 && i < I1) {
          vmadd<FMA, kPkFwd>(al[r], x, fl[i - I0]);
          vmadd<FMA, kPkFwd>(ah[r], x, fh[i - I0]);
        }
      }
      if (((NV - 1 - I0 - q) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      asm volatile("" : "+v"(al[r][e]));
      asm volatile("" : "+v"(ah[r][e]));
    }
}

// blk_fwd with wave-uniform offsets (as blk_inv_branch_s): Xb = X + blk_phys(layout, vb + HLV) * V, and the
// read of logical vector vb + HLV + q*m sits off(q) = q*m + ((q*m) >> sh)*pad from it for every thread
// when the pad groups align with a thread's block and HLV is a multiple of the group (host: vw_capi.cpp
// rounds HLV up to 16 vectors); q*m < 0 shifts arithmetically (floor), as blk_phys does.
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_fwd_s(const T* Xb, int m, int sh, int pad, const T* flo, const T* fhi,
                                          T (&al)[NV][VT<T>::V], T (&ah)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  constexpr int TC = blk_chunk<T, NV>();
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) { al[r][e] = T(0); ah[r][e] = T(0); }
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fl[I1 - I0], fh[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) { fl[i - I0] = flo[i]; fh[i - I0] = fhi[i]; }
#pragma unroll
    for (int q = NV - 1 - I0; q > -I1; --q) {
      const int qm = __builtin_amdgcn_readfirstlane(q * m);
      const int off = __builtin_amdgcn_readfirstlane(qm + (qm >> sh) * pad);
      const vec x = *reinterpret_cast<const vec*>(Xb + off * V);
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = r - q;
        if (i >= I0 && i < I1) {
          vmadd<FMA, kPkFwd>(al[r], x, fl[i - I0]);
          vmadd<FMA, kPkFwd>(ah[r], x, fh[i - I0]);
        }
      }
      if (((NV - 1 - I0 - q) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      asm volatile("" : "+v"(al[r][e]));
      asm volatile("" : "+v"(ah[r][e]));
    }
}

#ifndef VW_INV_KTAPS
#define VW_INV_KTAPS -1  // k_inverse_blk: taps from the kernel arguments (SGPRs) instead of LDS; -1: at NV >= 8
#endif

#ifndef VW_FWD_KTAPS
#define VW_FWD_KTAPS -1  // k_forward_blk: taps from the kernel arguments (SGPRs) instead of LDS; -1: at NV >= 8 (coif5 NV = 4: neutral)
#endif

#ifndef VW_BLK_FWD_C
#define VW_BLK_FWD_C 1  // NV < 8 forward: compile-time stride forms (0: per-lane blk_phys per read)
#endif

// blk_fwd at a compile-time stride M (NV < 8, as blk_inv_branch_c): with the halo HLV a multiple of 16
// vectors (host) the physical offset of logical vector vb + HLV + q*M from vb + HLV's is BlkC::off(q)
// for every thread.  The reads run q = -(L-1) .. NV-1; they are addressed from the lowest one, laundered
// into a 32-bit LDS base (lds_base: through a plain pointer the compiler re-based most of them, 3 of 63 reads
// per coif5 fp32 block kept an immediate), so every offset is a non-negative immediate of the ds_read.
template <typename T, int L, bool FMA, int NV, int M>
__device__ __forceinline__ void blk_fwd_c(const T* Xb, const T* flo, const T* fhi, T (&al)[NV][VT<T>::V],
                                          T (&ah)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  using C = BlkC<M, NV, 0>;
  constexpr int TC = blk_chunk<T, NV>();
  constexpr int QMIN = -(L - 1);
  const unsigned aq = lds_base(Xb + C::off(QMIN) * V);  // laundered: every read at an immediate offset
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) { al[r][e] = T(0); ah[r][e] = T(0); }
  static_for<0, (L + TC - 1) / TC>([&](auto c) __attribute__((always_inline)) {
    constexpr int I0 = decltype(c)::value * TC;
    constexpr int I1 = (I0 + TC < L) ? I0 + TC : L;
    T fl[I1 - I0], fh[I1 - I0];
#pragma unroll
    for (int i = I0; i < I1; ++i) { fl[i - I0] = flo[i]; fh[i - I0] = fhi[i]; }
#pragma unroll
    for (int q = NV - 1 - I0; q > -I1; --q) {
      const vec x = lds_vec_at<vec>(aq + (unsigned)((C::off(q) - C::off(QMIN)) * V * (int)sizeof(T)));
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        const int i = r - q;
        if (i >= I0 && i < I1) {
          vmadd<FMA, kPkFwd>(al[r], x, fl[i - I0]);
          vmadd<FMA, kPkFwd>(ah[r], x, fh[i - I0]);
        }
      }
      if (((NV - 1 - I0 - q) & 3) == 3) __builtin_amdgcn_sched_barrier(0);
    }
  });
#pragma unroll
  for (int r = 0; r < NV; ++r)
#pragma unroll
    for (int e = 0; e < V; ++e) {
      asm volatile("" : "+v"(al[r][e]));
      asm volatile("" : "+v"(ah[r][e]));
    }
}

// One forward level at vector stride m >= 1, NV < 8: the compile-time forms for m = 1..64, the generic one
// otherwise.  Same reads, same sums (bit-identical to blk_fwd).
template <typename T, int L, bool FMA, int NV>
__device__ __forceinline__ void blk_fwd_any(const T* X, const BlkLayout& lo, int HLV, int vb, int m, const T* flo,
                                            const T* fhi, T (&al)[NV][VT<T>::V], T (&ah)[NV][VT<T>::V]) {
  constexpr int V = VT<T>::V;
  const T* Xb = X + blk_phys(lo, vb + HLV) * V;
  auto go = [&](auto mc) __attribute__((always_inline)) {
    constexpr int M = decltype(mc)::value;
    if constexpr (BlkC<M, NV, 0>::ok) blk_fwd_c<T, L, FMA, NV, M>(Xb, flo, fhi, al, ah);
    else blk_fwd<T, L, FMA, NV>(X, lo, HLV, vb, m, flo, fhi, al, ah);
  };
  switch (m) {
    case 1: go(std::integral_constant<int, 1>{}); break;
    case 2: go(std::integral_constant<int, 2>{}); break;
    case 4: go(std::integral_constant<int, 4>{}); break;
    case 8: go(std::integral_constant<int, 8>{}); break;
    case 16: go(std::integral_constant<int, 16>{}); break;
    case 32: go(std::integral_constant<int, 32>{}); break;
    case 64: go(std::integral_constant<int, 64>{}); break;
    default: blk_fwd<T, L, FMA, NV>(X, lo, HLV, vb, m, flo, fhi, al, ah); break;
  }
}

// Forward, PERIODIC, one signal per workgroup: MultiLevelMODWTTransform.decompose (:243-251) /
// BatchSIMDMODWT.batchMultiLevelMODWTSoA (:362-377) / VectorWaveSwtAdapter forward.  Level inputs in
// one LDS buffer (p.region1 == 0: two barriers per level) or two (one barrier).  Left wrap images:
// element t is also the value at t - N.  Host contract: unrolled (L > 0), aligned rows, nvec =
// threads * NV, nvec a multiple of NV * m_J, no validation / history, p.hlpad = HLV * V.
template <typename T, int L, bool FMA, int NV>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, 8)) k_forward_blk(const FwdArgs<T> p) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* X = reinterpret_cast<T*>(smem);
  T* Y = p.region1 ? X + p.region1 : X;
  const bool dbl = p.region1 != 0;
  const long long b = blockIdx.x;
  // the taps live in LDS (p.tap_lds): read per level and chunk, never hoisted out of the level loop --
  // all 2L taps of a long filter held in registers across it spill (60 for coif5)
  T* const taps = reinterpret_cast<T*>(smem) + p.tap_lds;
  for (int i = threadIdx.x; i < 2 * L; i += blockDim.x) taps[i] = i < L ? p.lo[i] : p.hi[i - L];
  // kernel-argument taps (scalar loads, SGPR operands) at NV = 8 as in k_inverse_blk: fp64 L = 16 128 VGPRs
  // + 12 B/lane of scratch -> 99, none
  constexpr bool ktaps = VW_FWD_KTAPS < 0 ? NV >= 8 : VW_FWD_KTAPS != 0;
  const T* const flo = ktaps ? p.lo : taps;
  const T* const fhi = ktaps ? p.hi : taps + L;
  const int N = p.N;
  const int nvec = N / V;
  const int NT = blockDim.x;
  const int tid = threadIdx.x;
  const int HLV = p.hlpad / V;
  auto m_of = [&](int j) { return p.lv[j - 1].s / V; };
  auto hlv_of = [&](int j) { return ((L - 1) * p.lv[j - 1].s + V - 1) / V; };
  // vector w of level j's input (+ its left wrap image)
  auto put = [&](T* buf, int j, int w, const vec& o) {
    const BlkLayout lo = blk_layout(m_of(j), NV, p.blk_tight);
    blk_store<T>(buf, lo, w + HLV, o);
    if (w >= nvec - hlv_of(j)) blk_store<T>(buf, lo, w - nvec + HLV, o);
  };
  {
    T r0[NV][V];
    load_row_regs<T, NV>(r0, p.x + b * p.ldx, N, nvec, true, false);
    wait_vmem();
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int w = tid + k * NT;
      asm volatile("" : "+v"(w));
      vec o;
#pragma unroll
      for (int e = 0; e < V; ++e) o[e] = r0[k][e];
      put(X, 1, w, o);
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  T nf = T(0);  // VW_FLAG_REF_NONFINITE: a_J's probe (as k_forward_persist)
  for (int j = 1; j <= p.J; ++j) {
    const int m = m_of(j);
    lds_barrier();  // X = level input + images; every read of Y (previous level) done
    T* dout = p.details + ((size_t)(j - 1) * (size_t)p.B + (size_t)b) * (size_t)N;
    T* aout = p.approx + b * (size_t)N;
    const bool last = j == p.J;
    T al[NV][V], ah[NV][V];
    int vb = 0;
    if (m) {
      vb = blk_base<NV>(m);
      const BlkLayout lo = blk_layout(m, NV, p.blk_tight);
      const int sh = __builtin_amdgcn_readfirstlane(lo.sh), pad = __builtin_amdgcn_readfirstlane(lo.pad);
      bool fc = false;
      if constexpr (NV < 8) {
        if (VW_BLK_FWD_C && (HLV & 15) == 0) {
          blk_fwd_any<T, L, FMA, NV>(X, lo, HLV, vb, m, flo, fhi, al, ah);
          fc = true;
        }
      }
      if (fc) {
      } else if (VW_BLK_SOFF && NV >= 8 && (pad == 0 || (((m * NV) & ((1 << sh) - 1)) == 0 && (HLV & ((1 << sh) - 1)) == 0)))
        blk_fwd_s<T, L, FMA, NV>(X + blk_phys(lo, vb + HLV) * V, m, sh, pad, flo, fhi, al, ah);
      else
        blk_fwd<T, L, FMA, NV>(X, lo, HLV, vb, m, flo, fhi, al, ah);
      if (m < VW_BLK_NT_M) {
        // a lane's outputs are m*16-byte pieces NV*m*16 bytes apart: write-back stores, so that L2
        // merges a line's pieces before it goes to HBM (nontemporal stores of 16-byte pieces wrote
        // 1.5x the algorithmic bytes on coif5 fp32, profiles/hbm_traffic_coif5-f32.json)
#pragma unroll
        for (int r = 0; r < NV; ++r) {
          store_vec<0>(dout, (vb + r * m) * V, N, true, ah[r]);
          if (last) store_vec<0>(aout, (vb + r * m) * V, N, true, al[r]);
        }
      } else {
#pragma unroll
        for (int r = 0; r < NV; ++r) {
          store_vec<VW_FWD_STORE_AUX>(dout, (vb + r * m) * V, N, true, ah[r]);
          if (last) store_vec<VW_FWD_STORE_AUX>(aout, (vb + r * m) * V, N, true, al[r]);
        }
      }
    } else {
      // s < V (m == 0): only the register-window forms.  (fwd_row's strided form, unreachable here,
      // kept all 2L taps of its loop live and spilled coif5 fp32: 193 VGPRs of scratch, 1.5x the
      // kernel's HBM write bytes -- profiles/r02/hbm_traffic_coif5-f32.json.)
      auto em = [&](int k, int w, const T (&l)[V], const T (&h)[V]) {
        store_vec<VW_FWD_STORE_AUX>(dout, w * V, N, true, h);
        if (last) store_vec<VW_FWD_STORE_AUX>(aout, w * V, N, true, l);
#pragma unroll
        for (int e = 0; e < V; ++e) { al[k][e] = l[e]; ah[k][e] = h[e]; }
      };
      if constexpr (V == 4) {
        if (p.lv[j - 1].s == 2) fwd_row_t<T, L, FMA, NV, 2>(X + HLV * V, nvec, 2, flo, fhi, p.taps, em);
        else fwd_row_t<T, L, FMA, NV, 1>(X + HLV * V, nvec, 1, flo, fhi, p.taps, em);
      } else {
        fwd_row_t<T, L, FMA, NV, 1>(X + HLV * V, nvec, 1, flo, fhi, p.taps, em);
      }
    }
    if (p.nf_flag && last) {
#pragma unroll
      for (int r = 0; r < NV; ++r) nf_probe<T, V>(nf, al[r]);
    }
    if (!last) {
      if (!dbl) lds_barrier();  // one buffer: every read of this level's input done first
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        int w = m ? vb + r * m : tid + r * NT;
        asm volatile("" : "+v"(w));
        vec o;
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = al[r][e];
        put(Y, j + 1, w, o);
        __builtin_amdgcn_sched_barrier(0);
      }
      T* t = X; X = Y; Y = t;
    }
  }
  if (p.nf_flag) nf_flag_row<T>(p.nf_flag, b, nf);
}

// Inverse, PERIODIC, sequential sums (K4), one region time-shared as k_inverse_seq.  Right wrap
// images: element t is also the value at t + N.  Host contract as k_forward_blk (hlpad = 0).
template <typename T, int L, bool FMA, int NV>
__global__ void VW_FUSED_BOUNDS(NV, VW_FUSED_W(L, 6)) k_inverse_blk(const InvArgs<T> p) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* R = reinterpret_cast<T*>(smem);
  const long long b = p.rev ? p.B - 1 - (long long)blockIdx.x : (long long)blockIdx.x;
  const int N = p.N;
  const int nvec = N / V;
  const int NT = blockDim.x;
  const int tid = threadIdx.x;
  T* const taps = reinterpret_cast<T*>(smem) + p.tap_lds;  // as k_forward_blk
  for (int i = tid; i < 2 * L; i += NT) taps[i] = i < L ? p.lo[i] : p.hi[i - L];
  // NV = 8 (sym8 fp64 at N = 16384): the taps from the kernel arguments -- scalar loads, SGPR operands of the
  // FMAs -- free the VGPRs that held them (128 + 12-40 B/lane of scratch -> 123-125, none) and the LDS tap
  // reads: inverse 6.72-6.77 -> 6.27-6.32 ms.  NV = 4 (coif5 fp32) keeps them in LDS: there the freed VGPRs
  // admit a third workgroup per CU and the inverse slows, 6.73-6.80 -> 6.94-6.96 ms
  // (profiles/r04/ab_ktaps_coif5_sym8.log)
  constexpr bool ktaps = VW_INV_KTAPS < 0 ? NV >= 8 : VW_INV_KTAPS != 0;
  const T* const flo = ktaps ? p.lo : taps;
  const T* const fhi = ktaps ? p.hi : taps + L;
  auto thr_of = [&](int j) { return p.thr ? load_uniform(p.thr + (size_t)(j - 1) * (size_t)p.thr_ld + (size_t)b) : T(0); };
  const size_t plane = (size_t)p.B * (size_t)N;
  auto m_of = [&](int j) { return p.lv[j - 1].s / V; };
  auto hrv_of = [&](int j) { return ((L - 1) * p.lv[j - 1].s + V - 1) / V; };
  auto put = [&](int j, int w, const vec& o) {
    const BlkLayout lo = blk_layout(m_of(j), NV, p.blk_tight);
    blk_store<T>(R, lo, w, o);
    if (w < hrv_of(j)) blk_store<T>(R, lo, w + nvec, o);
  };
  // a row held in the standard mapping (w = tid + k*NT) into level j's layout; MODE as regs_to_level_m
  auto stage_std = [&](const T (&r)[NV][V], int j, int mode, T thr_b) {
#pragma unroll
    for (int k = 0; k < NV; ++k) {
      int w = tid + k * NT;
      asm volatile("" : "+v"(w));
      vec o;
#pragma unroll
      for (int e = 0; e < V; ++e) {
        if (mode == 1) o[e] = T(0);
        else if (mode == 2) o[e] = threshold_t(r[k][e], thr_b, p.soft);
        else o[e] = r[k][e];
      }
      put(j, w, o);
      __builtin_amdgcn_sched_barrier(0);
    }
  };

  T acc[NV][V];
  T dreg[NV][V];
  load_row_regs<T, NV>(acc, p.approx + b * (size_t)N, N, nvec, true, p.approx_zero != 0);
  load_row_regs<T, NV>(dreg, p.details + (size_t)(p.J - 1) * plane + b * (size_t)N, N, nvec, true,
                       p.lv[p.J - 1].use_d == 0);
  wait_vmem();
  stage_std(acc, p.J, p.approx_zero ? 1 : 0, T(0));

  for (int j = p.J; j >= 1; --j) {
    const LevelDesc lv = p.lv[j - 1];
    const int m = m_of(j);
    const BlkLayout lo = blk_layout(m, NV, p.blk_tight);
    const int vb = m ? blk_base<NV>(m) : 0;
    lds_barrier();  // R = a_j + wrap images
    zero_regs<T, NV>(acc);
    if (m) blk_inv_any<T, L, FMA, NV>(R, lo, p.blk_tight, vb, m, flo, acc);
    else inv_row<T, L, FMA, NV>(R, nvec, lv.s, 1, 0, flo, p.taps, acc);
    lds_barrier();  // every approximation-branch read done
    wait_vmem();    // the d_j prefetch
    stage_std(dreg, j, lv.use_d == 0 ? 1 : (p.thr ? 2 : 0), thr_of(j));
    if (j > 1)
      load_row_regs<T, NV>(dreg, p.details + (size_t)(j - 2) * plane + b * (size_t)N, N, nvec, true,
                           p.lv[j - 2].use_d == 0);
    lds_barrier();  // R = d_j + wrap images
    if (m) blk_inv_any<T, L, FMA, NV>(R, lo, p.blk_tight, vb, m, fhi, acc);
    else inv_row<T, L, FMA, NV>(R, nvec, lv.s, 1, 0, fhi, p.taps, acc);
    if (j > 1) {
      lds_barrier();  // every detail-branch read done
#pragma unroll
      for (int r = 0; r < NV; ++r) {
        int w = m ? vb + r * m : tid + r * NT;
        asm volatile("" : "+v"(w));
        vec o;
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = acc[r][e];
        put(j - 1, w, o);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  }
  // level 1 (s = 1 < V) ran in the standard mapping: coalesced stores
#pragma unroll
  for (int k = 0; k < NV; ++k) store_vec<VW_INV_STORE_AUX>(p.y + b * (size_t)N, (tid + k * NT) * V, N, true, acc[k]);
  if (p.nf_flag) {  // VW_FLAG_REF_NONFINITE: y's probe (as k_inverse_seq)
    T nf = T(0);
#pragma unroll
    for (int k = 0; k < NV; ++k) nf_probe<T, V>(nf, acc[k]);
    nf_flag_row<T>(p.nf_flag, b, nf);
  }
}

// ---------------------------------------------------------------------------------------------
// Per-level tiled kernels (signals longer than the fused kernels hold in LDS).  One workgroup per
// (tile, signal); the tile and its halo are gathered from HBM through the reference's index map.
template <typename T>
__device__ __forceinline__ T halo_value_global(const T* __restrict__ src, int idx, int N, int mode, int npow2,
                                               const T* hist_b, int hist_len) {
  if (idx >= 0 && idx < N) return src[idx];
  switch (mode) {
    case kHaloPeriodic: { int r = idx % N; if (r < 0) r += N; return src[r]; }
    case kHaloSymmetric: return src[sym_index(idx, N)];
    case kHaloFftPad: { int r = idx < 0 ? idx + npow2 : idx; return (r >= 0 && r < N) ? src[r] : T(0); }
    case kHaloHistory: return (idx < 0 && idx >= -hist_len) ? hist_b[hist_len + idx] : T(0);
    default: return T(0);
  }
}

template <typename T>
__device__ __forceinline__ void tile_to_lds(T* buf, const T* __restrict__ src, int N, int ts, int lo_q, int hi_q,
                                            int mode, int npow2, const T* hist_b, int hist_len, const T* thr,
                                            T thr_b, int soft, bool zero, bool vec_ok = false) {
  // buf[q] = value at signal index ts + q, q in [lo_q, hi_q).  The in-range middle moves as 16-byte
  // vectors (ts and the vector bounds are multiples of V; rows 16-B aligned when vec_ok); the
  // ends go through the index map element by element.
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  int qa = lo_q, qb = lo_q;  // vector range [qa, qb)
  if (vec_ok && !zero) {
    qa = max(lo_q, -ts);
    qa = (qa + V - 1) / V * V;
    qb = min(hi_q, N - ts);
    qb = qb >= qa ? qa + (qb - qa) / V * V : qa;
  }
  for (int q = qa + (int)threadIdx.x * V; q < qb; q += blockDim.x * V) {
    vec v = __builtin_nontemporal_load(reinterpret_cast<const vec*>(src + ts + q));
    if (thr) {
#pragma unroll
      for (int e = 0; e < V; ++e) v[e] = threshold_t(v[e], thr_b, soft);
    }
    *reinterpret_cast<vec*>(buf + q) = v;
  }
  const int tail = (hi_q - lo_q) - (qb - qa);
  for (int r = (int)threadIdx.x; r < tail; r += blockDim.x) {
    const int q = (lo_q + r < qa) ? lo_q + r : qb + (r - (qa - lo_q));
    T v = zero ? T(0) : halo_value_global(src, ts + q, N, mode, npow2, hist_b, hist_len);
    if (thr) v = threshold_t(v, thr_b, soft);
    buf[q] = v;
  }
}

template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(256) k_forward_level(const LevelArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* buf = reinterpret_cast<T*>(smem) + p.hlpad;
  const long long b = blockIdx.y;
  const int N = p.N;
  const int ts = blockIdx.x * p.tile;
  const int cnt = min(p.tile, N - ts);
  const int nv = (cnt + V - 1) / V;
  const LevelDesc lv = p.lv;
  const T* src = p.src_a + b * p.lda;
  const T* hist_b = (lv.mode == kHaloHistory) ? p.hist + b * lv.hist_len : nullptr;
  tile_to_lds(buf, src, N, ts, -lv.hl, nv * V, lv.mode, p.npow2, hist_b, lv.hist_len, (const T*)nullptr, T(0), 0,
              false, p.vec_io != 0 && (p.lda % V) == 0);
  if (p.validate) {
    for (int q = threadIdx.x; q < cnt; q += blockDim.x)
      if (!finite_t(buf[q])) atomicMin(p.bad, (unsigned long long)b * N + ts + q);
  }
  __syncthreads();
  const bool vec_ok = p.vec_io != 0;  // rows 16-B aligned (tile starts are multiples of V)
  for (int w = threadIdx.x; w < nv; w += blockDim.x) {
    const int t0 = w * V;
    T al[V], ah[V];
#pragma unroll
    for (int e = 0; e < V; ++e) { al[e] = T(0); ah[e] = T(0); }
    fwd_vec<T, L, FMA>(buf, t0, lv.s, p.lo, p.hi, p.taps, al, ah);
    store_vec(p.out_a + b * (size_t)N + ts, t0, cnt, vec_ok, al);
    store_vec(p.out_d + b * (size_t)N + ts, t0, cnt, vec_ok, ah);
    check_out<T>(p.validate, p.bad, (unsigned long long)b * N + ts, t0, cnt, al);
    check_out<T>(p.validate, p.bad, (unsigned long long)b * N + ts, t0, cnt, ah);
  }
}

template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(256) k_inverse_level(const LevelArgs<T> p) {
  constexpr int V = VT<T>::V;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* A = reinterpret_cast<T*>(smem) + p.hlpad;
  T* D = reinterpret_cast<T*>(smem) + p.region_d + p.hlpad_d;
  const long long b = blockIdx.y;
  const int N = p.N;
  const int ts = blockIdx.x * p.tile;
  const int cnt = min(p.tile, N - ts);
  const int nv = (cnt + V - 1) / V;
  const LevelDesc lv = p.lv;
  const T thr_b = p.thr ? p.thr[b] : T(0);  // this launch is one level: the host offsets thr
  const int span = nv * V;
  tile_to_lds(A, p.src_a + b * (size_t)N, N, ts, -lv.hl, span + lv.hr, lv.mode, 0, (const T*)nullptr, 0,
              (const T*)nullptr, T(0), 0, p.src_a == nullptr, p.vec_io != 0);
  tile_to_lds(D, p.src_d + b * (size_t)N, N, ts, -lv.hl, span + lv.hr, lv.mode, 0, (const T*)nullptr, 0, p.thr,
              thr_b, p.soft, p.use_d == 0 || p.src_d == nullptr, p.vec_io != 0);
  __syncthreads();
  const bool vec_ok = p.vec_io != 0;
  for (int w = threadIdx.x; w < nv; w += blockDim.x) {
    const int t0 = w * V;
    T acc[V];
#pragma unroll
    for (int e = 0; e < V; ++e) acc[e] = T(0);
    if (p.pair) {
      inv_pair<T, L, FMA>(A, D, t0, lv.s, lv.dir_a, p.lo, p.hi, p.taps, acc);
    } else {
      inv_branch<T, L, FMA>(A, t0, lv.s, lv.dir_a, lv.off_a, p.lo, p.taps, acc);
      inv_branch<T, L, FMA>(D, t0, lv.s, lv.dir_d, lv.off_d, p.hi, p.taps, acc);
    }
    store_vec(p.out_a + b * (size_t)N + ts, t0, cnt, vec_ok, acc);
  }
}

// ---------------------------------------------------------------------------------------------
// Column-sweep kernels for deep levels of long signals (spacing s >= kSweepMinS).  At spacing s
// the level's convolution never mixes residues mod s: view the row as a matrix [N/s][s] and every
// column r is an independent dense L-tap filter over q (t = r + q*s).  One thread owns one column
// and a chunk of QC consecutive q, keeping the L most recent inputs in a register window: each
// input is read from HBM once (+ L-1 warm-up reads per chunk), lanes read consecutive residues
// (>= 128 contiguous bytes per lane group), and there is no LDS halo -- which at level 10 of db8
// (15 x 512 = 7,680 samples) tripled the tiled kernel's reads.  Elements outside [0, N) (warm-up,
// wrap, tail) go through the reference's index map (halo_value_global), so every boundary mode and
// any N (wraps that change residue when s does not divide N) is exact; summation order per output
// is the reference's (taps ascending; approximation branch, then detail branch).
// kSweepMinS (vw_internal.h) = 16: 16 x 8 B = 128 B contiguous per lane group (fp64).

struct SweepPos {
  long long b;
  int r, q0, q1;  // column r, q in [q0, q1)
  bool ok;
};

__device__ __forceinline__ SweepPos sweep_pos(long long B, int N, int s, int qc) {
  // thread -> (signal, chunk, residue), residue fastest: consecutive lanes = consecutive addresses
  const int qn = (N + s - 1) / s;  // q extent of column 0
  const int chunks = (qn + qc - 1) / qc;
  const long long g = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long per = (long long)chunks * s;
  SweepPos p;
  p.b = g / per;
  const long long rem = g - p.b * per;
  const int c = (int)(rem / s);
  p.r = (int)(rem - (long long)c * s);
  const int qr = p.r < N ? (N - 1 - p.r) / s + 1 : 0;  // column r length
  p.q0 = c * qc;
  p.q1 = min(p.q0 + qc, qr);
  p.ok = p.b < B && p.q0 < p.q1;
  return p;
}

template <typename T>
__device__ __forceinline__ T sweep_fetch(const T* __restrict__ src, long long u, int N, int mode, int npow2,
                                         const T* hist_b, int hist_len) {
  if (u >= 0 && u < N) return src[u];
  return halo_value_global(src, (int)u, N, mode, npow2, hist_b, hist_len);
}

// Register window of one branch over a block of K outputs t_k = t_b + k*s (k < K):
//   DIR = -1 (reads t - i*s + off):  w[j] = value at t_b + off + (j - (L-1))*s, tap i of output k = w[k - i + L - 1]
//   DIR = +1 (reads t + i*s + off):  w[j] = value at t_b + off + j*s,           tap i of output k = w[k + i]
// j in [0, K + L - 1).  Between blocks the last L - 1 values move to the front and K new values are
// loaded -- all K loads of a block in flight at once (one load per output step would expose the
// full memory latency per output).
template <typename T, int L, int K, int DIR>
struct SweepWin {
  T w[K + L - 1];
  __device__ __forceinline__ long long first(long long tb, int s, int off) const {
    return tb + off + (DIR < 0 ? -(long long)(L - 1) * s : 0);
  }
  template <typename Fetch>
  __device__ __forceinline__ void fill_head(long long tb, int s, int off, Fetch&& fetch) {  // j < L - 1
    const long long u0 = first(tb, s, off);
#pragma unroll
    for (int j = 0; j < L - 1; ++j) w[j] = fetch(u0 + (long long)j * s);
  }
  template <typename Fetch>
  __device__ __forceinline__ void load_block(long long tb, int s, int off, Fetch&& fetch) {  // j >= L - 1
    const long long u0 = first(tb, s, off);
#pragma unroll
    for (int j = L - 1; j < K + L - 1; ++j) w[j] = fetch(u0 + (long long)j * s);
  }
  __device__ __forceinline__ void shift() {
#pragma unroll
    for (int j = 0; j < L - 1; ++j) w[j] = w[j + K];
  }
  __device__ __forceinline__ T tap(int k, int i) const { return DIR < 0 ? w[k - i + L - 1] : w[k + i]; }
};

// outputs per register block (loads in flight per branch); long filters keep their windows in budget
template <int L> struct SweepK { static constexpr int K = L <= 16 ? 16 : 8; };

// Forward, one level: a[t] = sum_i lo[i] x[g(t - i s)], d[t] likewise (ScalarOps.java:700-835 order).
template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(256) k_forward_sweep(const LevelArgs<T> p) {
  constexpr int K = SweepK<L>::K;
  const LevelDesc lv = p.lv;
  const int s = lv.s, N = p.N;
  const SweepPos sp = sweep_pos(p.B, N, s, p.tile);
  if (!sp.ok) return;
  const T* src = p.src_a + sp.b * p.lda;
  const T* hist_b = (lv.mode == kHaloHistory) ? p.hist + sp.b * lv.hist_len : nullptr;
  T* oa = p.out_a + sp.b * (size_t)N;
  T* od = p.out_d + sp.b * (size_t)N;
  const unsigned long long flat0 = (unsigned long long)sp.b * N;
  // inputs at or beyond the column end are never used by a stored output: read them as zero
  const long long tend = (long long)sp.r + (long long)sp.q1 * s;
  auto fetch = [&](long long u) -> T {
    if (u >= tend) return T(0);
    return sweep_fetch(src, u, N, lv.mode, p.npow2, hist_b, lv.hist_len);
  };
  SweepWin<T, L, K, -1> X;
  long long tb = (long long)sp.r + (long long)sp.q0 * s;
  X.fill_head(tb, s, 0, fetch);
  for (int q = sp.q0; q < sp.q1; q += K, tb += (long long)K * s) {
    X.load_block(tb, s, 0, fetch);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (q + k < sp.q1) {
        T al = T(0), ah = T(0);
#pragma unroll
        for (int i = 0; i < L; ++i) {
          al = madd<FMA>(al, X.tap(k, i), p.lo[i]);
          ah = madd<FMA>(ah, X.tap(k, i), p.hi[i]);
        }
        const long long t = tb + (long long)k * s;
        oa[t] = al;
        od[t] = ah;
        if (p.validate) {
          if (!finite_t(X.tap(k, 0))) atomicMin(p.bad, flat0 + t);
          if (!finite_t(al) || !finite_t(ah)) atomicMin(p.bad, (1ull << 62) | (flat0 + t));
        }
      }
    }
    X.shift();
  }
}

// Inverse, one level: approximation branch (lo, dir_a, off_a) and detail branch (hi, dir_d, off_d),
// each its own register window; sums in the reference's order (K4/K6 sequential, K5 pairwise).
template <typename T, int L, bool FMA, int DA, int DD>
__global__ void __launch_bounds__(256) k_inverse_sweep(const LevelArgs<T> p) {
  constexpr int K = SweepK<L>::K;
  const LevelDesc lv = p.lv;
  const int s = lv.s, N = p.N;
  const SweepPos sp = sweep_pos(p.B, N, s, p.tile);
  if (!sp.ok) return;
  const T thr_b = p.thr ? p.thr[sp.b] : T(0);
  const T* sa = p.src_a ? p.src_a + sp.b * (size_t)N : nullptr;
  const T* sd = p.src_d ? p.src_d + sp.b * (size_t)N : nullptr;
  const bool za = sa == nullptr, zd = sd == nullptr || p.use_d == 0;
  T* y = p.out_a + sp.b * (size_t)N;
  auto fa = [&](long long u) -> T { return za ? T(0) : sweep_fetch(sa, u, N, lv.mode, 0, (const T*)nullptr, 0); };
  auto fd = [&](long long u) -> T {
    if (zd) return T(0);
    const T v = sweep_fetch(sd, u, N, lv.mode, 0, (const T*)nullptr, 0);
    return p.thr ? threshold_t(v, thr_b, p.soft) : v;
  };
  SweepWin<T, L, K, DA> A;
  SweepWin<T, L, K, DD> D;
  long long tb = (long long)sp.r + (long long)sp.q0 * s;
  A.fill_head(tb, s, lv.off_a, fa);
  D.fill_head(tb, s, lv.off_d, fd);
  for (int q = sp.q0; q < sp.q1; q += K, tb += (long long)K * s) {
    A.load_block(tb, s, lv.off_a, fa);
    D.load_block(tb, s, lv.off_d, fd);
#pragma unroll
    for (int k = 0; k < K; ++k) {
      if (q + k < sp.q1) {
        T acc = T(0);
        if (p.pair) {  // MODWTTransform.inverse / K5: sum += h*a + g*d per tap
#pragma unroll
          for (int i = 0; i < L; ++i) acc = acc + pair_term<T, FMA>(p.lo[i], A.tap(k, i), p.hi[i], D.tap(k, i));
        } else {       // K4 / K6: all approximation taps, then all detail taps
#pragma unroll
          for (int i = 0; i < L; ++i) acc = madd<FMA>(acc, A.tap(k, i), p.lo[i]);
#pragma unroll
          for (int i = 0; i < L; ++i) acc = madd<FMA>(acc, D.tap(k, i), p.hi[i]);
        }
        y[tb + (long long)k * s] = acc;
      }
    }
    A.shift();
    D.shift();
  }
}

// ---------------------------------------------------------------------------------------------
// Two or three inverse levels per launch: levels j, j-1 (, j-2) with spacings G*h .. h (G = 2 or 4),
// PERIODIC, sequential sums (K4: MultiLevelMODWTTransform.java:576-589), as column sweeps chained
// through LDS rings, so the intermediate approximations never go to HBM (4 rows per pair of levels
// instead of 6, 5 per triple instead of 9).
//
// In the residue class r mod h, position u is the sample t = r + u*h (u < nu = N/h); the bottom level
// reads u + i, the one above u + 2i, the top u + G*i -- so the top level is a plain sweep over each of
// the G classes u = G*v + e (r + e*h mod G*h).  A workgroup owns R consecutive residues (R = 64: one
// fp64 per lane, 512 contiguous bytes per wave access; R = 32 where h = 32: two residue groups per
// wave, 256 B each) of one signal and a chunk [u0, u1) of u, in groups of R threads:
//   top groups (G of them): group e sweeps class e of the top level with register windows (as
//     k_inverse_sweep) and writes its KA outputs of block n (KB = G*KA positions) into ring 1 at step n;
//   middle groups (triple, 4): at step n, level j-1 over block n-2 -- parity e2, half of the parity's
//     2*KA outputs -- reading a_{j-1}[u + 2i] from ring 1 (it reaches into block n-1, complete) and
//     d_{j-1} from HBM, writing a_{j-2} into ring 2;
//   bottom groups (4 of a triple, 2 of a pair): at step 2 (pair) / 4 (triple) behind the top, KA
//     outputs of the bottom level each, ring -> y in HBM.
// One barrier per step; every ring holds three blocks.  The upper stages run past the chunk by their
// reach (L-1 positions at each level below, <= KB) and wrap mod N: every value equals the reference's
// (t+l)%N read, products summed in the same order -> bit-exact in EXACT mode.
// Host contract (vw_capi.cpp): h % R == 0, N % (G*h) == 0, every level PERIODIC / dir +1 / offset 0,
// (2*KB + 2*L) * G*h <= N (one wrap at most), KB >= 2*(L-1), p.tile (u per chunk) a multiple of KB.

// KA outputs of one level at u = ub + st*k (k < KA, st = the level's spacing in u): a from an LDS ring
// (slot of ub: sl0, slot stride st), d from HBM at t = tb + x*ts (ts = st*h); the approximation branch,
// then the detail branch, each i ascending.
template <typename T, int L, bool FMA, int KA, int R, int RING>
__device__ __forceinline__ void sweep_ring_stage(const T* ring, int lane, int sl0, int st, const T* sd, bool thr_on,
                                                 T thr_b, int soft, long long tb, long long ts, int N, const T* lo,
                                                 const T* hi, T (&acc)[KA]) {
  T wd[KA + L - 1];
#pragma unroll
  for (int x = 0; x < KA + L - 1; ++x) {  // issued first: in flight during the approximation branch
    if (sd) {
      long long t = tb + (long long)x * ts;
      t = t >= N ? t - N : t;
      const T v = sd[t];
      wd[x] = thr_on ? threshold_t(v, thr_b, soft) : v;
    } else {
      wd[x] = T(0);
    }
  }
  T w[KA + L - 1];
#pragma unroll
  for (int x = 0; x < KA + L - 1; ++x) {
    const int sl = sl0 + x * st;
    w[x] = ring[(sl >= RING ? sl - RING : sl) * R + lane];
  }
#pragma unroll
  for (int k = 0; k < KA; ++k) {
    acc[k] = T(0);
#pragma unroll
    for (int i = 0; i < L; ++i) acc[k] = madd<FMA>(acc[k], w[k + i], lo[i]);
  }
#pragma unroll
  for (int k = 0; k < KA; ++k)
#pragma unroll
    for (int i = 0; i < L; ++i) acc[k] = madd<FMA>(acc[k], wd[k + i], hi[i]);
}

// Workgroup -> (signal, R-residue block, u-chunk)
struct SweepGPos {
  long long b;
  int r0, u0, u1;
};
__device__ __forceinline__ bool sweepg_pos(long long B, int N, int h, int R, int uc, SweepGPos* w) {
  const int nu = N / h, nrb = h / R, nch = (nu + uc - 1) / uc;
  long long id = blockIdx.x;
  const int ch = (int)(id % nch);
  id /= nch;
  w->r0 = (int)(id % nrb) * R;
  w->b = id / nrb;
  w->u0 = ch * uc;
  w->u1 = min(w->u0 + uc, nu);
  return w->b < B;
}

// Top stage, class e of G: level-j sweep over t = r + e*h + v*G*h; one step writes KA outputs.
template <typename T, int L, bool FMA, int KA>
struct SweepTop {
  SweepWin<T, L, KA, 1> A, D;
  long long tb;
  int S, N;
  const T *sa, *sd;
  bool thr_on;
  T thr_b;
  int soft;
  __device__ __forceinline__ T fa(long long t) const { return sa ? sa[t >= N ? t - N : t] : T(0); }
  __device__ __forceinline__ T fd(long long t) const {
    if (!sd) return T(0);
    const T v = sd[t >= N ? t - N : t];
    return thr_on ? threshold_t(v, thr_b, soft) : v;
  }
  __device__ __forceinline__ void start() {
    A.fill_head(tb, S, 0, [&](long long t) { return fa(t); });
    D.fill_head(tb, S, 0, [&](long long t) { return fd(t); });
  }
  template <typename Out>
  __device__ __forceinline__ void step(const T* lo, const T* hi, Out&& out) {
    A.load_block(tb, S, 0, [&](long long t) { return fa(t); });
    D.load_block(tb, S, 0, [&](long long t) { return fd(t); });
#pragma unroll
    for (int k = 0; k < KA; ++k) {
      T acc = T(0);
#pragma unroll
      for (int i = 0; i < L; ++i) acc = madd<FMA>(acc, A.tap(k, i), lo[i]);
#pragma unroll
      for (int i = 0; i < L; ++i) acc = madd<FMA>(acc, D.tap(k, i), hi[i]);
      out(k, acc);
    }
    A.shift();
    D.shift();
    tb += (long long)KA * S;
  }
};

// Pair (G = 2): groups 0, 1 top (parity), 2, 3 bottom (half of a block).
template <typename T, int L, bool FMA, int KA, int R>
__global__ void __launch_bounds__(4 * R) k_inverse_sweep2(const LevelArgs<T> p) {
  constexpr int KB = 2 * KA;
  constexpr int RING = 3 * KB;
  static_assert(KB >= L - 1, "the bottom level reads at most one block ahead");
  __shared__ T ring[RING * R];
  const int S = p.lv.s, h = S >> 1, N = p.N;
  SweepGPos w;
  if (!sweepg_pos(p.B, N, h, R, p.tile, &w)) return;  // workgroup-uniform
  const int g = threadIdx.x / R, lane = threadIdx.x % R;
  const int r = w.r0 + lane;
  const int nblk = (w.u1 - w.u0 + KB - 1) / KB;
  const size_t row = (size_t)w.b * (size_t)N;
  if (g < 2) {
    SweepTop<T, L, FMA, KA> top;
    top.S = S; top.N = N; top.soft = p.soft;
    top.sa = p.src_a ? p.src_a + row : nullptr;
    top.sd = (p.src_d && p.use_d) ? p.src_d + row : nullptr;
    top.thr_on = p.thr != nullptr;
    top.thr_b = p.thr ? p.thr[w.b] : T(0);
    top.tb = (long long)r + (long long)g * h + (long long)(w.u0 >> 1) * S;
    top.start();
    for (int n = 0; n <= nblk + 1; ++n) {
      if (n <= nblk) {
        T* rn = ring + ((n % 3) * KB + g) * R + lane;
        top.step(p.lo, p.hi, [&](int k, T v) { rn[2 * k * R] = v; });  // u = u0 + n*KB + 2k + g
      }
      __syncthreads();
    }
  } else {
    const int hh = g - 2;
    const T* sd = (p.src_d2 && p.use_d2) ? p.src_d2 + row : nullptr;
    const T thr_b = p.thr2 ? p.thr2[w.b] : T(0);
    T* y = p.out_a + row;
    for (int n = 0; n <= nblk + 1; ++n) {
      if (n >= 2) {
        const int m = n - 2;
        const int ub = w.u0 + m * KB + hh * KA;
        T acc[KA];
        sweep_ring_stage<T, L, FMA, KA, R, RING>(ring, lane, (m % 3) * KB + hh * KA, 1, sd, p.thr2 != nullptr, thr_b,
                                                 p.soft, (long long)r + (long long)ub * h, h, N, p.lo, p.hi, acc);
#pragma unroll
        for (int k = 0; k < KA; ++k)
          if (ub + k < w.u1) y[(size_t)r + (size_t)(ub + k) * (size_t)h] = acc[k];
      }
      __syncthreads();
    }
  }
}

// Triple (G = 4): groups 0..3 top (class u mod 4), 4..7 middle (parity, half), 8..11 bottom (quarter).
template <typename T, int L, bool FMA, int KA, int R>
__global__ void __launch_bounds__(12 * R) k_inverse_sweep3(const LevelArgs<T> p) {
  constexpr int KB = 4 * KA;
  constexpr int RING = 3 * KB;
  static_assert(KB >= 2 * (L - 1), "the middle level reads at most one block ahead");
  __shared__ T ring1[RING * R];
  __shared__ T ring2[RING * R];
  const int S = p.lv.s, h = S >> 2, N = p.N;
  SweepGPos w;
  if (!sweepg_pos(p.B, N, h, R, p.tile, &w)) return;  // workgroup-uniform
  const int g = threadIdx.x / R, lane = threadIdx.x % R;
  const int r = w.r0 + lane;
  const int nblk = (w.u1 - w.u0 + KB - 1) / KB;
  const size_t row = (size_t)w.b * (size_t)N;
  // top: blocks 0 .. nblk+1 at steps n; middle: blocks 0 .. nblk at n-2; bottom: blocks 0 .. nblk-1 at n-4
  if (g < 4) {
    SweepTop<T, L, FMA, KA> top;
    top.S = S; top.N = N; top.soft = p.soft;
    top.sa = p.src_a ? p.src_a + row : nullptr;
    top.sd = (p.src_d && p.use_d) ? p.src_d + row : nullptr;
    top.thr_on = p.thr != nullptr;
    top.thr_b = p.thr ? p.thr[w.b] : T(0);
    top.tb = (long long)r + (long long)g * h + (long long)(w.u0 >> 2) * S;
    top.start();
    for (int n = 0; n <= nblk + 3; ++n) {
      if (n <= nblk + 1) {
        T* rn = ring1 + ((n % 3) * KB + g) * R + lane;
        top.step(p.lo, p.hi, [&](int k, T v) { rn[4 * k * R] = v; });  // u = u0 + n*KB + 4k + g
      }
      __syncthreads();
    }
  } else if (g < 8) {
    const int e2 = (g - 4) & 1, half = (g - 4) >> 1;
    const T* sd = (p.src_d2 && p.use_d2) ? p.src_d2 + row : nullptr;
    const T thr_b = p.thr2 ? p.thr2[w.b] : T(0);
    for (int n = 0; n <= nblk + 3; ++n) {
      if (n >= 2 && n <= nblk + 2) {
        const int m = n - 2;
        const int o = e2 + 2 * half * KA;  // u offset of this group's first output in the block
        const int ub = w.u0 + m * KB + o;
        T acc[KA];
        sweep_ring_stage<T, L, FMA, KA, R, RING>(ring1, lane, (m % 3) * KB + o, 2, sd, p.thr2 != nullptr, thr_b, p.soft,
                                                 (long long)r + (long long)ub * h, 2LL * h, N, p.lo, p.hi, acc);
        T* rn = ring2 + ((m % 3) * KB + o) * R + lane;
#pragma unroll
        for (int k = 0; k < KA; ++k) rn[2 * k * R] = acc[k];
      }
      __syncthreads();
    }
  } else {
    const int q = g - 8;
    const T* sd = (p.src_d3 && p.use_d3) ? p.src_d3 + row : nullptr;
    const T thr_b = p.thr3 ? p.thr3[w.b] : T(0);
    T* y = p.out_a + row;
    for (int n = 0; n <= nblk + 3; ++n) {
      if (n >= 4) {
        const int m = n - 4;
        const int ub = w.u0 + m * KB + q * KA;
        T acc[KA];
        sweep_ring_stage<T, L, FMA, KA, R, RING>(ring2, lane, (m % 3) * KB + q * KA, 1, sd, p.thr3 != nullptr, thr_b,
                                                 p.soft, (long long)r + (long long)ub * h, h, N, p.lo, p.hi, acc);
#pragma unroll
        for (int k = 0; k < KA; ++k)
          if (ub + k < w.u1) y[(size_t)r + (size_t)(ub + k) * (size_t)h] = acc[k];
      }
      __syncthreads();
    }
  }
}

// ---------------------------------------------------------------------------------------------
// Multi-level tiles for long PERIODIC signals (host: vw_capi.cpp level_groups).  One workgroup runs
// a group of consecutive levels over one tile of one signal; the intermediate approximations stay
// in LDS.  Periodic convolution commutes with shifts, so a level evaluated at a position v outside
// [0, N) (the tile's halo) equals the reference's value at v mod N bit for bit -- the same products
// summed in the same order -- and only the group's inputs go through the index map.  Each level is
// evaluated over the tile plus the reach of the levels after it: to the left in the forward
// (ScalarOps.java:700-723 reads t - l*s), to the right in the inverse (MultiLevelMODWTTransform
// .java:576-589 reads t + l*s).  The redundant ext/tile of the arithmetic buys one HBM round trip
// per group instead of one per level.
template <typename T, int L, bool FMA>
__global__ void __launch_bounds__(256) k_forward_multi(const MultiArgs<T> p) {
  constexpr int V = VT<T>::V;
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* X = reinterpret_cast<T*>(smem) + p.ext[0];  // level input, positions [-ext[k], span)
  T* Y = X + p.region;
  const long long b = blockIdx.y;
  const int N = p.N;
  const int ts = blockIdx.x * p.tile;
  const int cnt = min(p.tile, N - ts);
  const int span = (cnt + V - 1) / V * V;
  tile_to_lds(X, p.src_a + b * p.lda, N, ts, -p.ext[0], span, kHaloPeriodic, 0, (const T*)nullptr, 0,
              (const T*)nullptr, T(0), 0, false, p.vec_io != 0);
  const bool vec_ok = p.vec_io != 0;
  for (int k = 0; k < p.nlev; ++k) {
    lds_barrier();  // X complete; every read of Y (the previous level's input) done
    const int s = p.s0 << k;
    const int q_lo = -p.ext[k + 1];  // outputs [q_lo, span): the tile + what the next levels read
    const int nv = (span - q_lo) / V;
    const bool last = k == p.nlev - 1;
    T* od = p.out_d[k] + b * (size_t)N + ts;
    T* oa = p.out_a + b * (size_t)N + ts;
    for (int w = threadIdx.x; w < nv; w += blockDim.x) {
      const int q0 = q_lo + w * V;
      T al[V], ah[V];
#pragma unroll
      for (int e = 0; e < V; ++e) { al[e] = T(0); ah[e] = T(0); }
      fwd_vec<T, L, FMA>(X, q0, s, p.lo, p.hi, p.taps, al, ah);
      if (q0 >= 0) {  // the tile's own outputs (vectors never straddle 0: q_lo is a multiple of V)
        store_vec(od, q0, cnt, vec_ok, ah);
        if (last) store_vec(oa, q0, cnt, vec_ok, al);
      }
      if (!last) {
        vec o;
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = al[e];
        *reinterpret_cast<vec*>(Y + q0) = o;
      }
    }
    T* t = X; X = Y; Y = t;
  }
}

// Inverse: A = a_j, D = d_j (thresholded on load for denoise); a_{j-1} is computed into registers
// (NI vectors per thread) and written over A after a barrier -- two LDS regions, so three 256-thread
// workgroups fit a CU (a third region for a_{j-1} measured 1.2x slower: two per CU).  NI = 4 (fp64, host
// policy) on a tile whose register-blocked levels give all four waves work: at NI = 8 a 2048-sample db8
// tile had 129-144 threads of work per level, one SIMD idle and one mostly idle.
#ifndef VW_MULTI_CK
#define VW_MULTI_CK 1  // k_inverse_multi register-blocked levels: compile-time strides, immediate LDS offsets
#endif
template <typename T, int L, bool FMA, int NI = kMultiInvNI>
__global__ void __launch_bounds__(256) k_inverse_multi(const MultiArgs<T> p) {
  constexpr int V = VT<T>::V;
  static_assert(NI == 8 || NI == 4, "outputs per thread");  // host contract: every level's blocks fit 256 threads
  using vec = typename VT<T>::v;
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  T* const A = reinterpret_cast<T*>(smem);  // positions [0, span + ext[k])
  T* const D = A + p.region;
  const long long b = blockIdx.y;
  const int N = p.N;
  const int ts = blockIdx.x * p.tile;
  const int cnt = min(p.tile, N - ts);
  const int span = (cnt + V - 1) / V * V;
  const bool vec_ok = p.vec_io != 0;
  const int top = p.nlev - 1;
  T nf = T(0);  // VW_FLAG_REF_NONFINITE (p.nf_flag: the group ends at level 1): y's probe
  // Detail prefetch (p.pf, host contract: whole vectors, (span + ext[top]) / V <= kMultiPF * 256): the
  // tile of d_{k-1} is loaded into registers right after level k's first barrier and written to D
  // after its second, so the HBM latency of the next level's input overlaps this level's arithmetic.
  // The loads are unconditional (clamped vector index): an exec-masked load block makes the waitcnt
  // pass wait for it at the first LDS read.
  const bool pf = p.pf != 0;
  // Padded LDS layout (p.pad, host contract: pf and rblk on): the register-blocked levels (vector
  // stride m = s/V in 1..8) read lanes NI*m vectors apart -- an 8-way bank conflict at m = 1 in the
  // natural layout (62 % of LDS cycles in conflicts on db8 levels 1-5, profiles/r03/pmc_db8_stream.txt).
  // Level k's A and D then hold logical vector u at u + u/8 at NI = 8 (layout 1), at NI = 4 at u + u/4
  // (m <= 4, layout 2) or u + 2*(u/8) (m = 8, layout 3) -- blk_layout's NV = 8 / NV = 4 layouts, conflict-free
  // ds_read_b128 at every m <= 8 under the gfx950 lane groups; levels with m = 0 or m >= 16 keep the natural
  // layout (0).
  // (a layout is (shift, pad): u -> u + (u >> shift) * pad -- one formula, no per-layout copies of the
  // hoisted store addresses)
  auto layout = [&](int k) {
    const int sk = p.s0 << k, m = sk / V;
    int2 lay = make_int2(30, 0);
    if (p.pad != 0 && sk >= V && sk % V == 0) {
      if constexpr (NI >= 8) {
        if (m < 16) lay = make_int2(3, 1);
      } else {
        if (m <= 4) lay = make_int2(2, 1);
        else if (m == 8) lay = make_int2(3, 2);
      }
    }
    return lay;
  };
  auto padded = [](int2 lay) { return lay.y != 0; };
  auto phys = [](int u, int2 lay) { return u + (u >> lay.x) * lay.y; };
  vec dreg[kMultiPF];
  auto d_load = [&](int k) {
    const T* sd = p.src_d[k];
    const int nvd = (span + p.ext[k]) / V;
#pragma unroll
    for (int i = 0; i < kMultiPF; ++i) {
      const int w = min((int)threadIdx.x + i * 256, nvd - 1);
      int pos = ts + w * V;
      if (pos >= N) pos %= N;  // periodic wrap of the right reach
      if (sd)
        dreg[i] = __builtin_nontemporal_load(reinterpret_cast<const vec*>(sd + b * (size_t)N + pos));
      else
#pragma unroll
        for (int e = 0; e < V; ++e) dreg[i][e] = T(0);
    }
  };
  auto d_store = [&](int k) {
    const int2 pd = layout(k);
    const T* th = p.thr[k];
    const T thb = th ? th[b] : T(0);
    const int nvd = (span + p.ext[k]) / V;
#pragma unroll
    for (int i = 0; i < kMultiPF; ++i) {
      const int w = (int)threadIdx.x + i * 256;
      if (w < nvd) {
        vec v = dreg[i];
        if (th)
#pragma unroll
          for (int e = 0; e < V; ++e) v[e] = threshold_t(v[e], thb, p.soft);
        *reinterpret_cast<vec*>(D + phys(w, pd) * V) = v;
      }
    }
  };
  if (p.pad) {
    // a_top through registers into level top's layout (the d_load path, no threshold)
    const int2 pd = layout(top);
    const int nva = (span + p.ext[top]) / V;
#pragma unroll
    for (int i = 0; i < kMultiPF; ++i) {
      const int w = min((int)threadIdx.x + i * 256, nva - 1);
      int pos = ts + w * V;
      if (pos >= N) pos %= N;
      if (p.src_a)
        dreg[i] = __builtin_nontemporal_load(reinterpret_cast<const vec*>(p.src_a + b * (size_t)N + pos));
      else
#pragma unroll
        for (int e = 0; e < V; ++e) dreg[i][e] = T(0);
    }
#pragma unroll
    for (int i = 0; i < kMultiPF; ++i) {
      const int w = (int)threadIdx.x + i * 256;
      if (w < nva) *reinterpret_cast<vec*>(A + phys(w, pd) * V) = dreg[i];
    }
  } else {
    tile_to_lds(A, p.src_a ? p.src_a + b * (size_t)N : p.src_a, N, ts, 0, span + p.ext[top], kHaloPeriodic, 0,
                (const T*)nullptr, 0, (const T*)nullptr, T(0), 0, p.src_a == nullptr, vec_ok);
  }
  if (pf) {
    d_load(top);
    d_store(top);
  }
  for (int k = top; k >= 0; --k) {
    if (!pf) {
      const T* sd = p.src_d[k];
      const T* th = p.thr[k];
      tile_to_lds(D, sd ? sd + b * (size_t)N : sd, N, ts, 0, span + p.ext[k], kHaloPeriodic, 0, (const T*)nullptr, 0,
                  th, th ? th[b] : T(0), p.soft, sd == nullptr, vec_ok);
    }
    lds_barrier();  // A and D complete
    if (pf && k > 0) d_load(k - 1);
    const int s = p.s0 << k;
    const int nv = (span + (k > 0 ? p.ext[k - 1] : 0)) / V;  // the tile + what the next levels read
    T acc[NI][V];
    if constexpr (L > 0) {
      // Register-blocked taps (S a multiple of V): one thread owns the NI outputs v, v+m, .., v+(NI-1)m
      // (m = S/V vectors), which read the same LDS vectors shifted by one tap: NI+L-1 reads per branch
      // instead of NI*L.  Per output the taps still run i ascending, A then D: bit-identical sums.
      const int m = s / V;
      const int pairs = (nv + m * NI - 1) / (m * NI) * m;  // (block, column) pairs, uniform
      if (p.rblk && s >= V && s % V == 0 && pairs <= 256) {
        const int pr = threadIdx.x;
        const int vb = (pr / m) * m * NI + pr % m;
        const int lim = (span + p.ext[k]) / V - 1;  // last vector of the A/D regions
        const int2 pdk = layout(k), pdn = k > 0 ? layout(k - 1) : make_int2(30, 0);
#pragma unroll
        for (int r = 0; r < NI; ++r)
#pragma unroll
          for (int e = 0; e < V; ++e) acc[r][e] = T(0);
        if (pr < pairs) {
          // compile-time stride M and layout LC: the reads of a lane sit at fixed offsets off(j) from
          // phys(vb) -- with G = 8 (layouts 1, 3) or 4 (layout 2) vectors per pad group, (vb % G) + (M*j % G) < G
          // for every M <= 8 here (vb % G = pr % M < M, or M*j % G = 0), so (vb + M*j) / G = vb / G + M*j / G --
          // and each is one ds_read at an immediate offset.
          // Reads past the region end (at most 15*M vectors, only for outputs that are never stored) stay
          // inside the allocation: the host adds p.slack >= 16*8 + 16 vectors after D (M <= 8 here).
          const T* const tlo = p.lo;
          const T* const thi = p.hi;
          auto blk_c = [&](auto mc, auto lc) __attribute__((always_inline)) {
            constexpr int M = decltype(mc)::value;
            constexpr int PD = decltype(lc)::value;
            constexpr auto off = [](int j) {
              return PD == 1 ? M * j + ((M * j) >> 3) : PD == 2 ? M * j + ((M * j) >> 2) : M * j + (((M * j) >> 3) << 1);
            };
#pragma unroll
            for (int br = 0; br < 2; ++br) {
              const unsigned ab = lds_base((br == 0 ? A : D) + phys(vb, PD == 1 ? make_int2(3, 1) : PD == 2 ? make_int2(2, 1)
                                                                                        : make_int2(3, 2)) * V);
#pragma unroll
              for (int j = 0; j < NI + L - 1; ++j) {
                const vec x = lds_vec_at<vec>(ab + (unsigned)(off(j) * V * (int)sizeof(T)));
#pragma unroll
                for (int r = 0; r < NI; ++r) {
                  const int i = j - r;
                  if (i >= 0 && i < L) {
                    // the tap straight from the kernel arguments (a pointer to p.lo / p.hi would copy
                    // the argument block to scratch)
                    const T fi = br == 0 ? tlo[i] : thi[i];
#pragma unroll
                    for (int e = 0; e < V; ++e) acc[r][e] = madd<FMA>(acc[r][e], x[e], fi);
                  }
                }
                if ((j & 3) == 3) __builtin_amdgcn_sched_barrier(0);  // bounded reads in flight (VGPRs)
              }
            }
          };
          using I1 = std::integral_constant<int, 1>;
          using I2 = std::integral_constant<int, 2>;
          using I4 = std::integral_constant<int, 4>;
          using I8 = std::integral_constant<int, 8>;
          using P1 = std::integral_constant<int, NI >= 8 ? 1 : 2>;  // layout of m = 1, 2, 4
          using P8 = std::integral_constant<int, NI >= 8 ? 1 : 3>;  // layout of m = 8
          // padded layouts only (the default, p.pad): more instantiations in this function raised it from 160
          // VGPRs to 238 + 1.3 KiB of scratch (the taps, hoisted across the switch)
          const int sel = VW_MULTI_CK && p.slack && padded(pdk) ? m : -1;
          switch (sel) {
            case 1: blk_c(I1{}, P1{}); break;
            case 2: blk_c(I2{}, P1{}); break;
            case 4: blk_c(I4{}, P1{}); break;
            case 8: blk_c(I8{}, P8{}); break;
            default:
#pragma unroll
              for (int br = 0; br < 2; ++br) {
                const T* buf = br == 0 ? A : D;
                const T* f = br == 0 ? p.lo : p.hi;
#pragma unroll
                for (int j = 0; j < NI + L - 1; ++j) {
                  const vec x = *reinterpret_cast<const vec*>(buf + phys(min(vb + m * j, lim), pdk) * V);
#pragma unroll
                  for (int r = 0; r < NI; ++r) {
                    const int i = j - r;
                    if (i >= 0 && i < L)
#pragma unroll
                      for (int e = 0; e < V; ++e) acc[r][e] = madd<FMA>(acc[r][e], x[e], f[i]);
                  }
                }
              }
              break;
          }
          if (k == 0) {
#pragma unroll
            for (int r = 0; r < NI; ++r)
              if (vb + m * r < nv) {
                store_vec(p.out_a + b * (size_t)N + ts, (vb + m * r) * V, cnt, vec_ok, acc[r]);
                if (p.nf_flag)
#pragma unroll
                  for (int e = 0; e < V; ++e)
                    if ((vb + m * r) * V + e < cnt) nf = nf_step<T>(acc[r][e], nf);
              }
          }
        }
        if (k == 0) break;
        lds_barrier();  // every read of A and D done
        if (pr < pairs) {
#pragma unroll
          for (int r = 0; r < NI; ++r) {
            if (vb + m * r < nv) {
              vec o;
#pragma unroll
              for (int e = 0; e < V; ++e) o[e] = acc[r][e];
              *reinterpret_cast<vec*>(A + phys(vb + m * r, pdn) * V) = o;
            }
          }
        }
        if (pf) d_store(k - 1);
        continue;
      }
    }
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int w = threadIdx.x + i * 256;
#pragma unroll
      for (int e = 0; e < V; ++e) acc[i][e] = T(0);
      if (w < nv) {
        // K4: all approximation taps, then all detail taps, into one accumulator
        inv_branch<T, L, FMA>(A, w * V, s, 1, 0, p.lo, p.taps, acc[i]);
        inv_branch<T, L, FMA>(D, w * V, s, 1, 0, p.hi, p.taps, acc[i]);
        if (k == 0) {
          store_vec(p.out_a + b * (size_t)N + ts, w * V, cnt, vec_ok, acc[i]);
          if (p.nf_flag)
#pragma unroll
            for (int e = 0; e < V; ++e)
              if (w * V + e < cnt) nf = nf_step<T>(acc[i][e], nf);
        }
      }
      __builtin_amdgcn_sched_barrier(0);  // one vector's LDS reads in flight at a time (VGPR budget)
    }
    if (k == 0) break;
    lds_barrier();  // every read of A and D done
    const int2 pdn = layout(k - 1);  // (this level itself is never padded: see layout())
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int w = threadIdx.x + i * 256;
      if (w < nv) {
        vec o;
#pragma unroll
        for (int e = 0; e < V; ++e) o[e] = acc[i][e];
        *reinterpret_cast<vec*>(A + phys(w, pdn) * V) = o;
      }
    }
    if (pf) d_store(k - 1);
  }
  if (p.nf_flag) nf_flag_row<T>(p.nf_flag, b, nf);  // VW_FLAG_REF_NONFINITE: y's probe (vw_ref.hip)
}

template <typename T>
__global__ void k_history_update(const T* __restrict__ in, long long ld_in, const T* __restrict__ old_hist,
                                 T* __restrict__ new_hist, int n, int hist_len) {
  const long long b = blockIdx.y;
  const int p = blockIdx.x * blockDim.x + threadIdx.x;
  if (p >= hist_len) return;
  const int q = p + n - hist_len;
  new_hist[b * hist_len + p] = q >= 0 ? in[b * ld_in + q] : old_hist[b * hist_len + p + n];
}


template <typename T>
__global__ void k_threshold(T* c, long long B, long long N, const T* __restrict__ thr, int soft) {
  const long long total = B * N;
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const long long b = i / N;
    c[i] = threshold_t(c[i], thr[b], soft);
  }
}

__device__ __forceinline__ unsigned long long splitmix64(unsigned long long z) {
  z += 0x9E3779B97F4A7C15ull;
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}

template <typename T>
__global__ void k_fill_uniform(T* x, long long count, unsigned long long seed, long long offset) {
  for (long long i = blockIdx.x * (long long)blockDim.x + threadIdx.x; i < count;
       i += (long long)gridDim.x * blockDim.x) {
    const unsigned long long r = splitmix64(seed ^ (unsigned long long)(offset + i));
    const double u = (double)(r >> 11) * (1.0 / 9007199254740992.0);
    x[i] = (T)(2.0 * u - 1.0);
  }
}

// BatchSIMDMODWT.haarBatchMODWTSoA (:86-140): hard-coded 0.5 / -0.5 taps.
template <typename T>
__global__ void k_single_haar_batch(const T* __restrict__ x, long long ldx, int N, T* approx, T* detail) {
  const long long b = blockIdx.y;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < N; t += gridDim.x * blockDim.x) {
    const int tm1 = (t - 1 + N) % N;
    const T s0 = x[b * ldx + t], s1 = x[b * ldx + tm1];
    approx[b * (size_t)N + t] = s0 * T(0.5) + s1 * T(0.5);
    detail[b * (size_t)N + t] = s0 * T(0.5) + s1 * T(-0.5);
  }
}


}  // namespace vw
