// vw_internal.h -- shared between the HIP kernels (vw_kernels.hip) and the C-ABI host layer
// (vw_capi.cpp).  Not installed; the public boundary is include/vectorwave_amd.h.
#pragma once
#include <hip/hip_runtime.h>
#include <atomic>
#include <cstdint>

namespace vw {

constexpr int kMaxTaps = 64;    // longest base filter accepted (COIF10 = 60 taps)
constexpr int kMaxLevels = 24;  // batch semantics have no level cap; LDS / N bound it in practice
constexpr int kNV = 8;          // max vectors (16 B each) held per thread in the fused kernels (NV = 4 or 8)
constexpr int kMaxThreads = 1024;
constexpr int kLdsBytes = 160 * 1024;
constexpr int kSweepMinS = 16;    // per-level path: spacings >= this run as column sweeps (vw_device.h)
constexpr int kSweepChunk = 128;  // q-chunk per sweep thread (measured: 128 beats 256 and 64)

// Source of the values outside [0, N) of a level's input ("halo"), i.e. the reference's index map.
enum HaloMode : int {
  kHaloPeriodic = 0,   // ((i % N) + N) % N        ScalarOps.java:700-723, (t+l)%N in the inverses
  kHaloZero = 1,       // 0                        ScalarOps.java:790-808, :590-601
  kHaloSymmetric = 2,  // MathUtils.symmetricBoundaryExtension  core/util/MathUtils.java:30-51
  kHaloFftPad = 3,     // i + nextPow2(N) if < N else 0 (FFT branch zero-pads)  ScalarOps.java:650-675
  kHaloHistory = 4     // streaming left history   BatchSIMDMODWT.java:447-507
};

// Per-level description, computed on the host (vw_capi.cpp) from the reference's bookkeeping.
struct LevelDesc {
  int s;        // a-trous spacing 2^(j-1)
  int hl, hr;   // halo extents (elements) the level reads left of 0 / right of N-1
  int mode;     // HaloMode of the level input (forward) / of both inverse inputs
  int dir_a;    // inverse approx branch: +1 reads t + i*s + off_a, -1 reads t - i*s + off_a
  int off_a;
  int dir_d;    // inverse detail branch
  int off_d;
  int use_d;    // inverse: 1 = d_j from memory, 0 = zero details (reconstructFromLevel / Levels)
  int hist_len; // streaming: left history length of this level (L_j - 1)
  int own;      // 1: halo written by the element owners (vw_device.h halo_images), else filled after a barrier
  int il_a, il_b;  // left image of element t: il_a*t + il_b (kept when in [-hl, 0))
  int ir_a, ir_b;  // right image: ir_a*t + ir_b (kept when in [N, N+hr))
  int vs, ve;   // only vectors w < vs or w >= ve have images
};

template <typename T>
struct FwdArgs {
  const T* x;           // [B][ldx]
  long long ldx;
  T* details;           // [J][B][N]
  T* approx;            // [B][N]
  long long B;
  int N;
  int J;
  int npow2;            // nextPow2(N) for kHaloFftPad
  int hlpad;            // LDS offset of element 0 (multiple of the vector width)
  int region1;          // element offset of the second level buffer (0 = single buffer)
  int vec_io;
  int unrolled;         // 1: the tap-unrolled kernel may run (aligned rows, full slabs; vw_capi fused_plan)
  int dma_nt;           // k_forward_persist: non-temporal LDS-DMA of the signal rows
  int validate;         // 1: non-finite check on input and outputs (atomicMin into *bad)
  int rev;              // 1: workgroup g owns signal B-1-g (walk order, see vw_capi.cpp walk_reverse)
  unsigned long long* bad;
  // streaming history (kHaloHistory): hist[j] is [B][hist_len_j], oldest first
  T* hist[kMaxLevels];
  int hist_update;      // 1: write the new history after each level
  int taps;             // L (runtime copy; kernels are also templated on it)
  int tap_lds;          // k_forward_blk: element offset of the LDS tap table
  int blk_tight;        // k_forward_blk: sparse padding (blk_layout)
  int* nf_flag;         // k_forward_persist, VW_FLAG_REF_NONFINITE: nf_flag[b] = 1 when an output of row b is
                        // non-finite (nullptr = off; the rows vw_ref.hip recomputes)
  T lo[kMaxTaps];       // base taps * 1/sqrt(2)  (ScalarOps.java:909-916: same at every level)
  T hi[kMaxTaps];
  LevelDesc lv[kMaxLevels];
};

template <typename T>
struct InvArgs {
  const T* details;     // [J][B][N]
  const T* approx;      // [B][N]
  T* y;                 // [B][N]
  long long B;
  int N;
  int J;
  int hlpad_a, hlpad_d; // LDS offsets of element 0 in the A and D regions
  int region_d;         // element offset of the D region start in LDS
  int vec_io;
  int pair;             // 1: sum += (h*a + g*d) per tap (MODWTTransform.inverse, ZERO multi-level)
  int unrolled;
  int db;               // sequential sum: 1 = two LDS buffers (k_inverse_db), 0 = one (k_inverse_seq)
  int blk;              // 1: register-blocked PERIODIC inverse (k_inverse_blk), padded LDS layouts
  int approx_zero;
  int rev;              // 1: workgroup g owns signal B-1-g
  const T* thr;         // thresholds [J][thr_ld] (nullptr = no thresholding)
  long long thr_ld;     // level stride of thr (0: one threshold per signal for every level)
  int soft;
  int taps;
  int tap_lds;          // k_inverse_blk: element offset of the LDS tap table
  int blk_tight;        // k_inverse_blk: sparse padding (blk_layout)
  int* nf_flag;         // k_inverse_seq, VW_FLAG_REF_NONFINITE: nf_flag[b] = 1 when an input or the output of
                        // row b is non-finite (nullptr = off)
  T lo[kMaxTaps];
  T hi[kMaxTaps];
  LevelDesc lv[kMaxLevels];
};

// Per-level tiled fallback (N too large for the fused kernels): one launch per level.
template <typename T>
struct LevelArgs {
  const T* src_a;       // forward: level input [B][lda]; inverse: approx input [B][N]
  long long lda;
  const T* src_d;       // inverse: details of this level [B][N]
  const T* src_d2;      // k_inverse_sweep2/3: details of level j-1 [B][N]
  const T* thr2;        // k_inverse_sweep2/3: thresholds of level j-1
  int use_d2;
  const T* src_d3;      // k_inverse_sweep3: details / thresholds of level j-2
  const T* thr3;
  int use_d3;
  T* out_a;             // forward: approx out [B][N]; inverse: y out [B][N]
  T* out_d;             // forward: detail out [B][N]
  const T* hist;        // kHaloHistory source [B][hist_len]
  long long B;
  int N;
  int tile;             // outputs per workgroup
  int hlpad;            // LDS offset of tile element 0 (A)
  int region_d, hlpad_d;
  int pair;
  const T* thr;
  int soft;
  int use_d;
  int vec_io;
  int validate;
  unsigned long long* bad;
  int npow2;
  int taps;
  T lo[kMaxTaps];
  T hi[kMaxTaps];
  LevelDesc lv;
};

// Multi-level tiles (PERIODIC, long signals): a group of consecutive levels of one tile in one
// launch, the intermediate approximations kept in LDS (vw_device.h k_forward_multi / k_inverse_multi).
constexpr int kMaxGroup = 8;
constexpr int kMultiInvNI = 8;  // k_inverse_multi: output vectors per thread (256 threads)
constexpr int kMultiPF = 6;     // k_inverse_multi: prefetched detail vectors per thread (256 threads)
template <typename T>
struct MultiArgs {
  const T* src_a;            // forward: input of the group's first level [B][lda]; inverse: a_{j1} [B][N] (nullptr = 0)
  long long lda;
  const T* src_d[kMaxGroup]; // inverse: d_j of group level k (k = 0 is the finest), nullptr = zero
  T* out_d[kMaxGroup];       // forward: d_j of group level k
  T* out_a;                  // forward: approximation of the coarsest level; inverse: a_{j0-1}
  const T* thr[kMaxGroup];   // inverse denoise: thresholds [B] of group level k (nullptr = none)
  long long B;
  int N;
  int tile;                  // stored outputs per workgroup (multiple of V)
  int nlev;                  // levels in the group
  int s0;                    // spacing of the group's finest level
  int ext[kMaxGroup + 1];    // forward: left extent of level k's input (ext[nlev] = 0);
                             // inverse: right extent of level k's input;
                             // multiples of V, each covering the reach of the levels after it
  int region;                // element stride between LDS buffers
  int vec_io;
  int soft;
  int taps;
  int rblk;                  // inverse: register-blocked taps where S is a multiple of V
  int pf;                    // inverse: next level's detail tile prefetched into registers
  int pad;                   // inverse: padded LDS layout at the register-blocked levels (needs pf, rblk)
  int* nf_flag;              // inverse, VW_FLAG_REF_NONFINITE, the group writes y: y's probe (nullptr = off)
  int slack;                 // inverse: LDS vectors allocated past D (compile-time-stride reads, 0 = off)
  int ni;                    // inverse: output vectors per thread, kMultiInvNI or 4 (fp64)
  T lo[kMaxTaps];
  T hi[kMaxTaps];
};

// WaveletDenoiser threshold methods (core/denoising/WaveletDenoiser.java:588-622) and the per-launch
// constants of the threshold kernels (vw_sigma.h).
enum ThrMethod { kThrUniversal = 0, kThrSure = 1, kThrMinimax = 2, kThrBayes = 3, kThrFixed = 4 };
constexpr int kSigmaRegN = 16384;  // k_noise_sigma keeps a row's keys in registers up to this N (1024 x 16)
constexpr int kSureMaxN = 16384;  // SURE on device: the sorted row lives in LDS
struct DenoiseConsts {
  double level_scale[kMaxLevels];  // Math.sqrt(1 << level) (denoiseMultiLevel, :225), 1 for denoise()
  double univ_c;                   // Math.sqrt(2.0 * Math.log(n))
  double log_n;                    // Math.log(n)
  int method;
  int n;
};

// The reference's own arithmetic for rows holding non-finite values (vw_ref.hip, VW_FLAG_REF_NONFINITE).
constexpr int kRefPlanes = 2 * kMaxLevels + 3;  // x, J details, approx, J streaming histories
template <typename T>
struct RefScan {                // flag[b] = 1 when row b of any plane is non-finite somewhere
  const T* p[kRefPlanes];
  long long ld[kRefPlanes];     // row stride of plane k
  int len[kRefPlanes];          // row length of plane k (0: N)
  int np;
  long long B;
  int N;
  int chunks;                   // ref_scan_chunks(N)
  int* flag;                    // [B], kept zero between calls (k_ref_* clear the rows they recompute)
};
template <typename T>
struct RefArgs {
  const T* x;                   // forward: input [B][ldx]; inverse: approximation [B][N] (nullptr = zeros)
  long long ldx;
  const T* det_in;              // inverse: details [J][B][N]
  T* details;                   // forward outputs [J][B][N], [B][N]
  T* approx;
  T* y;                         // inverse output [B][N]
  const T* thr;                 // inverse: thresholds [J][thr_ld] (nullptr = none)
  long long thr_ld;
  int soft;
  long long B;
  int N;
  int J;
  int L;
  int mode;                     // kHaloPeriodic / kHaloZero / kHaloSymmetric
  // forward, BatchStreamingMODWT ZERO / SYMMETRIC blocks: samples left of the block come from the level's
  // history (hist_old, [B][hist_len_j] oldest first; hist_first: the history the first block initialises,
  // zeros / the mirror of the level input); hist_new (nullptr: none, e.g. a flush) receives the updated one
  int hist_mode;
  int hist_first;
  const T* hist_old[kMaxLevels];
  T* hist_new[kMaxLevels];
  int hist_len[kMaxLevels];
  int* flag;                    // rows to recompute (cleared once recomputed)
  T* scratch;                   // [grid][2][N] running approximations
  T lo[kMaxTaps];               // base taps * 1/sqrt(2), as the fast kernels
  T hi[kMaxTaps];
  LevelDesc lv[kMaxLevels];     // inverse: use_d, K6 orientation / offsets
};
template <typename T>
hipError_t launch_flag_nonfinite(const RefScan<T>& a, hipStream_t st);
template <typename T>
hipError_t launch_ref_cascade(const RefArgs<T>& a, int grid, bool inverse, hipStream_t st);
int ref_scan_chunks(int N);

// Matrix-core fp32 kernels (vw_mfma.hip): which (L, N) are instantiated, the halo a level set needs, launchers.
bool mfma_supported(int L, long long N);
int mfma_halo(int L, int J);
int mfma_region(int n);  // LDS floats of the kernels' padded level region for elements [0, n)
hipError_t launch_forward_mfma(const FwdArgs<float>& a, int lds, hipStream_t st);
hipError_t launch_inverse_mfma(const InvArgs<float>& a, int lds, hipStream_t st);

// Raise a kernel's dynamic-LDS limit past the 64 KiB default once per kernel instantiation AND
// device (the attribute belongs to the device's copy of the function; a call per launch costs host
// time).  `once` is a static of the caller, unique per kernel instantiation; several host threads
// (one per context, vw_modwt_*_multi_f64) may race here -- the attribute call is idempotent and the
// flag is atomic.
constexpr int kMaxDevices = 64;
struct LdsOnce {
  std::atomic<int> limit[kMaxDevices];  // zero-initialised as a static: the 64 KiB default applies
};
template <typename Kern>
static hipError_t set_lds(Kern k, int lds_bytes, LdsOnce* once, int want = kLdsBytes) {
  if (lds_bytes <= 64 * 1024) return hipSuccess;
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0) dev = 0;
  std::atomic<int>* f = dev < kMaxDevices ? &once->limit[dev] : nullptr;
  if (f && f->load(std::memory_order_acquire) >= lds_bytes) return hipSuccess;
  if (want < lds_bytes) want = lds_bytes;
  hipError_t e = hipFuncSetAttribute(reinterpret_cast<const void*>(k), hipFuncAttributeMaxDynamicSharedMemorySize, want);
  if (e != hipSuccess) return e;
  if (f) f->store(want, std::memory_order_release);
  return hipSuccess;
}

// Launchers (vw_kernels.hip).  Return hipSuccess or the launch error.
template <typename T>
hipError_t launch_forward_fused(const FwdArgs<T>& a, int threads, int lds_bytes, bool fma, int nv, hipStream_t st);
template <typename T>
hipError_t launch_forward_persist(const FwdArgs<T>& a, int threads, int lds_bytes, bool fma, int nv, hipStream_t st);
template <typename T>
hipError_t launch_forward_blk(const FwdArgs<T>& a, int threads, int lds_bytes, bool fma, int nv, hipStream_t st);
template <typename T>
hipError_t launch_inverse_fused(const InvArgs<T>& a, int threads, int lds_bytes, bool fma, int nv, hipStream_t st);
template <typename T>
hipError_t launch_forward_level(const LevelArgs<T>& a, int lds_bytes, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_inverse_level(const LevelArgs<T>& a, int lds_bytes, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_forward_sweep(const LevelArgs<T>& a, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_inverse_sweep(const LevelArgs<T>& a, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_inverse_sweepg(const LevelArgs<T>& a, int levels, int ka, int R, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_forward_multi(const MultiArgs<T>& a, int lds_bytes, bool fma, hipStream_t st);

template <typename T>
hipError_t launch_inverse_multi(const MultiArgs<T>& a, int lds_bytes, bool fma, hipStream_t st);
template <typename T>
hipError_t launch_history_update(const T* level_in, long long ld_in, const T* old_hist, T* new_hist,
                                 long long B, int n, int hist_len, hipStream_t st);

hipError_t launch_level_threshold(const double* coeffs, long long level_stride, const double* sigma,
                                  const DenoiseConsts& k, long long B, int levels, double* thr, hipStream_t st);
hipError_t launch_noise_sigma(const double* coeffs, long long ld, long long B, int N, double scale_c,
                              double* sigma_out, double* thr_out, hipStream_t st);
// Exact median of |x - center| per row (center nullptr: of |x|); N <= 16384 when center is given.
hipError_t launch_median(const double* x, long long ld, long long B, int N, const double* center, double* median_out,
                         hipStream_t st);
// out[b][i] = |x[b*ld + i] - center[b]| (MathUtils.medianAbsoluteDeviation's deviations), for the
// centered median of rows longer than the register-keyed path holds.
hipError_t launch_abs_center(const double* x, long long ld, long long B, int N, const double* center, double* out,
                             hipStream_t st);
hipError_t launch_seq_std(const double* x, int n, double* out, hipStream_t st);
hipError_t launch_gather_abs(const double* src, const int* idx, int count, double* window, int wsize, int start,
                             hipStream_t st);
template <typename T>
hipError_t launch_transpose(const T* in, long long rows, long long cols, T* out, hipStream_t st);
template <typename T>
hipError_t launch_threshold(T* c, long long B, long long N, const T* thr, int soft, hipStream_t st);
template <typename T>
hipError_t launch_fill_uniform(T* x, long long count, unsigned long long seed, long long offset, hipStream_t st);
template <typename T>
hipError_t launch_single_haar_batch(const T* x, long long ldx, long long B, int N, T* approx, T* detail,
                                    hipStream_t st);

// Register-blocked kernels (k_forward_blk / k_inverse_blk): padded LDS layout of a level with vector
// stride m (must match vw_device.h blk_layout).  Returns (shift, pad): u -> u + (u >> shift) * pad.
inline void blk_layout_host(int m, int nv, int* sh, int* pad, int tight = 0) {
  if (m <= 0 || m >= 16) { *sh = 30; *pad = 0; }
  else if (nv >= 8) { *sh = tight ? 4 : 3; *pad = 1; }
  else if (m == 8) { *sh = 3; *pad = 2; }
  else { *sh = 2; *pad = 1; }
}

// Which compile-time tap counts have unrolled kernels; others use the runtime-L kernel.
bool has_unrolled_taps(int L);
int fused_max_threads();

}  // namespace vw
