// vw_capi.cpp -- C ABI of the MI355X MODWT/SWT engine (include/vectorwave_amd.h).
//
// Host-side bookkeeping restated from the reference (level cap, L_j guard, symmetric alignment
// tables, FFT-switch region, status mapping), then one fused HIP launch per transform
// (vw_kernels.hip), or one tiled launch per level for signals longer than LDS holds.
#include "../../include/vectorwave_amd.h"
#include "vw_internal.h"
#include "vw_deep.h"

#include <algorithm>
#include <cmath>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <map>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

using namespace vw;

// ------------------------------------------------------------------------------------------------
// Errors (thread-local, like the reference's exceptions are per call site)
static thread_local std::string t_err;
static thread_local int64_t t_err_index = -1;
static thread_local int64_t t_signal_base = 0;  // run_sharded: global row of this block's first signal

static vw_status fail(vw_status code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  t_err = buf;
  if (code != VW_ERR_NONFINITE) t_err_index = -1;
  return code;
}

static vw_status ok() {
  t_err.clear();
  t_err_index = -1;
  return VW_OK;
}

#define VW_HIP(call)                                                                         \
  do {                                                                                       \
    hipError_t e_ = (call);                                                                  \
    if (e_ != hipSuccess) return fail(VW_ERR_DEVICE, "%s: %s", #call, hipGetErrorString(e_)); \
  } while (0)

#define VW_TRY(expr)                      \
  do {                                    \
    vw_status s_ = (expr);                \
    if (s_ != VW_OK) return s_;           \
  } while (0)

// ------------------------------------------------------------------------------------------------
struct TimedLaunch {
  std::string family;
  hipEvent_t start, stop;
  bool graph_owned = false;  // recorded inside a captured graph: its events live as long as the graph
};

// Tuning switches (A/B experiments, tools/ab_*.sh), read from the environment ONCE per context at
// vw_ctx_create -- never per call: a transform call does no getenv.  Defaults are the measured best.
struct Tuning {
  int nv = 4;              // VW_NV: vectors per thread of the fused kernels (4 or 8)
  bool fwd_persist = true; // VW_FWD_PERSIST=0: no persistent forward
  int fwd_buf = 0;         // VW_FWD_BUF=1|2: force one / two forward level buffers (0 = policy)
  bool force_tiled = false;// VW_FORCE_TILED: per-level path even when the fused kernels fit
  int fwd_rev = 0, inv_rev = 0;  // VW_FWD_REV / VW_INV_REV: reverse workgroup -> signal walk
  int dma_nt = -1;               // VW_DMA_NT=0|1: LDS-DMA of signal rows non-temporal; -1 = policy (see forward_impl)
  int fwd_tile = 0;        // VW_FWD_TILE: per-level forward tile (0 = default)
  bool multi = true;       // VW_MULTI=0: one launch per level on the long-signal path
  int multi_div = 4;       // VW_MULTI_DIV: reach bound of a level group = tile / div
  int multi_tile = 0;      // VW_MULTI_TILE: multi-level tile (0 = 16 KiB of samples)
  int inv_buf = 0;         // VW_INV_BUF=2: two-buffer sequential inverse (k_inverse_db)
  int inv_tile = 0;        // VW_INV_TILE: per-level inverse tile (0 = 1024)
  int multi_rblk = 1;      // VW_MULTI_RBLK: register-blocked taps in k_inverse_multi
  int multi_pf = 1;        // VW_MULTI_PF: k_inverse_multi prefetches the next detail tile
  int multi_pad = 1;       // VW_MULTI_PAD: k_inverse_multi's padded LDS layout at register-blocked levels
  int multi_inv_tile = 0;  // VW_MULTI_INV_TILE: k_inverse_multi's tile (0 = VW_MULTI_TILE's)
  int multi_ni = 4;        // VW_MULTI_NI: k_inverse_multi's output vectors per thread -- 4 (fp64, on the largest tile
                           // whose levels fit 256 threads) or 8; db8-stream inverse 9.19-9.33 -> 8.75-8.80 ms
                           // (profiles/r05/ab_db8_inverse_multi_ni4.log)
  bool no_sweep = false;   // VW_NO_SWEEP: no column sweeps for deep levels
  int sweep_qc = kSweepChunk;  // VW_SWEEP_QC: q-chunk per sweep thread
  int unroll_max = kMaxTaps;   // VW_UNROLL_MAX: longest filter that runs the tap-unrolled fused kernels
  int blk = 10;                // VW_BLK: shortest filter that runs the register-blocked PERIODIC kernels (0 = off)
                               // (measured on MI355X, db8 J=10 2^20 blocks: no faster than the sweeps yet)
  bool deep = true;             // VW_DEEP=0|1: streaming deep-level forward (vw_deep.hip) off / on
  bool deep_inv = false;       // VW_DEEP_INV=1 (or VW_DEEP=1): the deep inverse too -- measured slower than
                               // the column sweeps on db8-stream (profiles/r03/ab_deep_db8_stream.log)
  int deep_lds = 80;           // VW_DEEP_LDS: LDS budget of one deep group, KiB (80 = two workgroups per CU)
  int deep_waves = 4;          // VW_DEEP_WAVES: target deep workgroups per CU when choosing segments
  int deep_pf_fwd = 1;         // VW_DEEP_PF_FWD / VW_DEEP_PF_INV: tiles of DMA-fed input in flight
  int deep_pf_inv = 1;
  int fwd_nv = 0;              // VW_FWD_NV / VW_INV_NV = 2: 1024-thread fused kernels with 2 vectors per
  int inv_nv = 0;              // thread (L <= 8, unrolled); 0 = policy
  int sweep2 = 3;              // VW_SWEEP2: deep inverse column-sweep levels chained per launch, up to 3 (2 = pairs only,
                               // 0 = one sweep per level)
  int sweep2_ka = 8;           // VW_SWEEP2_KA: stage-A outputs per thread and step (8 or 16)
  int sweep2_uc = 2048;        // VW_SWEEP2_UC: u positions per workgroup chunk (512 / 1024 / 2048: 9.68 / 9.50 / 9.33 ms db8 inverse)
  int sweep2_r = 0;            // VW_SWEEP2_R=32: 32-residue groups even where h allows 64 (0 = widest)
  int sweep2_minb = 64;        // VW_SWEEP2_MINB: blocks a residue class needs for the chained sweeps
  int blk_fwd8 = 1;            // VW_BLK_FWD8=0: fused forward instead of the register-blocked one at NV = 8
  int ref_grid = 0;            // VW_REF_GRID: workgroups of the REF_NONFINITE fix-up launch (0 = 2 per CU)
  int mfma = 0;                // VW_MFMA=1|2|3: fp32 FMA PERIODIC forward (1) / inverse (2) / both (3) on the matrix
                               // cores (vw_mfma.hip)
};

// One switch of the Tuning struct by its environment name; value < 0 = the default.  Returns false
// for an unknown name.
static bool set_tuning(Tuning& t, const char* key, int v) {
  const Tuning d;
  const std::string k(key);
  if (k == "VW_NV") t.nv = v < 0 ? d.nv : v <= 4 ? 4 : 8;
  else if (k == "VW_FWD_PERSIST") t.fwd_persist = v < 0 ? d.fwd_persist : v != 0;
  else if (k == "VW_FWD_BUF") t.fwd_buf = v < 0 ? d.fwd_buf : v;
  else if (k == "VW_FORCE_TILED") t.force_tiled = v > 0;
  else if (k == "VW_FWD_REV") t.fwd_rev = v < 0 ? 0 : v;
  else if (k == "VW_INV_REV") t.inv_rev = v < 0 ? 0 : v;
  else if (k == "VW_DMA_NT") t.dma_nt = v < 0 ? d.dma_nt : v;
  else if (k == "VW_FWD_TILE") t.fwd_tile = v < 0 ? 0 : v;
  else if (k == "VW_MULTI") t.multi = v < 0 ? d.multi : v != 0;
  else if (k == "VW_MULTI_DIV") t.multi_div = v <= 0 ? d.multi_div : v;
  else if (k == "VW_MULTI_TILE") t.multi_tile = v < 0 ? 0 : v;
  else if (k == "VW_INV_BUF") t.inv_buf = v < 0 ? 0 : v;  // 0 = policy
  else if (k == "VW_INV_TILE") t.inv_tile = v < 0 ? 0 : v;
  else if (k == "VW_MULTI_RBLK") t.multi_rblk = v < 0 ? d.multi_rblk : v;
  else if (k == "VW_MULTI_PF") t.multi_pf = v < 0 ? d.multi_pf : v;
  else if (k == "VW_MULTI_PAD") t.multi_pad = v < 0 ? d.multi_pad : v;
  else if (k == "VW_MULTI_INV_TILE") t.multi_inv_tile = v < 0 ? 0 : v;
  else if (k == "VW_MULTI_NI") t.multi_ni = v < 0 ? d.multi_ni : v == 4 ? 4 : 8;
  else if (k == "VW_NO_SWEEP") t.no_sweep = v > 0;
  else if (k == "VW_SWEEP_QC") t.sweep_qc = v >= 16 ? v : d.sweep_qc;
  else if (k == "VW_UNROLL_MAX") t.unroll_max = v < 0 ? d.unroll_max : v;
  else if (k == "VW_BLK") t.blk = v < 0 ? d.blk : v;
  else if (k == "VW_DEEP") { t.deep = v < 0 ? d.deep : v != 0; t.deep_inv = v < 0 ? d.deep_inv : v != 0; }
  else if (k == "VW_DEEP_INV") t.deep_inv = v < 0 ? d.deep_inv : v != 0;
  else if (k == "VW_DEEP_LDS") t.deep_lds = v <= 0 ? d.deep_lds : v;
  else if (k == "VW_DEEP_WAVES") t.deep_waves = v <= 0 ? d.deep_waves : v;
  else if (k == "VW_DEEP_PF_FWD") t.deep_pf_fwd = v <= 0 ? d.deep_pf_fwd : std::min(v, 16);
  else if (k == "VW_DEEP_PF_INV") t.deep_pf_inv = v <= 0 ? d.deep_pf_inv : std::min(v, 16);
  else if (k == "VW_FWD_NV") t.fwd_nv = v < 0 ? d.fwd_nv : v;
  else if (k == "VW_INV_NV") t.inv_nv = v < 0 ? d.inv_nv : v;
  else if (k == "VW_SWEEP2") t.sweep2 = v < 0 ? d.sweep2 : v;
  else if (k == "VW_SWEEP2_KA") t.sweep2_ka = v == 16 ? 16 : v == 8 ? 8 : d.sweep2_ka;
  else if (k == "VW_SWEEP2_UC") t.sweep2_uc = v >= 32 ? v : d.sweep2_uc;
  else if (k == "VW_SWEEP2_R") t.sweep2_r = v == 32 ? 32 : 0;
  else if (k == "VW_SWEEP2_MINB") t.sweep2_minb = v < 0 ? d.sweep2_minb : v;
  else if (k == "VW_BLK_FWD8") t.blk_fwd8 = v < 0 ? d.blk_fwd8 : v;
  else if (k == "VW_MFMA") t.mfma = v < 0 ? d.mfma : v;
  else if (k == "VW_REF_GRID") t.ref_grid = v < 0 ? d.ref_grid : v;
  else return false;
  return true;
}

static const char* const kTuningKeys[] = {
    "VW_NV", "VW_FWD_PERSIST", "VW_FWD_BUF", "VW_FORCE_TILED", "VW_FWD_REV", "VW_INV_REV",
    "VW_FWD_TILE", "VW_MULTI", "VW_MULTI_DIV", "VW_MULTI_TILE", "VW_INV_BUF", "VW_INV_TILE", "VW_MULTI_RBLK", "VW_MULTI_PF", "VW_MULTI_PAD", "VW_MULTI_INV_TILE", "VW_NO_SWEEP", "VW_SWEEP_QC",
    "VW_UNROLL_MAX", "VW_BLK", "VW_FWD_NV",
    "VW_INV_NV", "VW_DEEP", "VW_DEEP_INV", "VW_DEEP_LDS", "VW_DEEP_WAVES", "VW_DEEP_PF_FWD", "VW_DEEP_PF_INV",
    "VW_SWEEP2", "VW_SWEEP2_KA", "VW_SWEEP2_UC", "VW_SWEEP2_R", "VW_SWEEP2_MINB", "VW_BLK_FWD8",
    "VW_DMA_NT", "VW_MULTI_NI", "VW_MFMA", "VW_REF_GRID"};

static Tuning read_tuning() {
  Tuning t;
  for (const char* k : kTuningKeys) {
    const char* e = getenv(k);
    if (!e) continue;
    // presence-style switches (VW_FORCE_TILED, VW_NO_SWEEP) are on when set to anything but "0"
    const int v = (*e == '\0') ? 1 : atoi(e);
    set_tuning(t, k, v);
  }
  return t;
}

struct vw_graph;
struct vw_ctx;
static void kill_pipelines_of(vw_ctx* c);

struct vw_ctx {
  int device = 0;
  hipStream_t stream = nullptr;
  bool own_stream = false;
  bool capturing = false;      // between vw_capture_begin / vw_capture_end
  unsigned ws_gen = 0;         // bumped when ws / ws2 move: graphs recorded before are stale
  Tuning tune;
  int cus = 256;               // compute units of the device (small-batch policies)
  std::recursive_mutex mu;
  void* ws = nullptr;          // tiled-path ping-pong buffers
  size_t ws_bytes = 0;
  void* ws2 = nullptr;         // denoise coefficients / thresholds
  size_t ws2_bytes = 0;
  unsigned long long* bad = nullptr;   // device word for the fused non-finite check
  bool timing = false;
  std::vector<TimedLaunch> pending;
  std::vector<TimedLaunch> captured;   // timed launches recorded during the current capture
  std::vector<hipEvent_t> event_pool;
  std::map<std::string, std::pair<double, int64_t>> totals;
  std::set<vw_graph*> graphs;          // live graphs recorded on this context (invalidated at destroy)
  std::vector<std::pair<void*, size_t>> stage;  // host-memory staging pool (Staging), kept across calls
  void* med = nullptr;         // vw_median_f64 deviations of long rows (not ws: growing ws invalidates graphs)
  size_t med_bytes = 0;
  int* nf = nullptr;           // VW_FLAG_REF_NONFINITE row flags [nf_rows], zero between calls (vw_ref.hip)
  int64_t nf_rows = 0;
};

struct vw_graph {
  vw_ctx* ctx = nullptr;          // nullptr once the context is destroyed (the graph is then dead)
  int device = 0;
  unsigned ws_gen = 0;
  std::vector<TimedLaunch> timed;  // event-record nodes (timing enabled at capture)
  hipGraph_t graph = nullptr;
  hipGraphExec_t exec = nullptr;
};

// Frees the HIP objects of a graph (its context's device must be current).
static void release_graph(vw_graph* gr) {
  for (auto& t : gr->timed) { hipEventDestroy(t.start); hipEventDestroy(t.stop); }
  gr->timed.clear();
  if (gr->exec) hipGraphExecDestroy(gr->exec);
  if (gr->graph) hipGraphDestroy(gr->graph);
  gr->exec = nullptr;
  gr->graph = nullptr;
}

struct vw_stream {
  vw_ctx* ctx = nullptr;
  std::vector<double> lo, hi;
  int L = 0;
  int boundary = 0;
  int levels = 0;
  int64_t last_batch = -1;
  bool hist_init = false;
  std::vector<double*> hist;        // device [B][hist_len_j]
  std::vector<double*> snap;        // VW_FLAG_REF_NONFINITE: the histories a block read (same shapes)
  std::vector<int> hist_len;
};

static hipEvent_t pool_event(vw_ctx* c) {
  if (!c->event_pool.empty()) {
    hipEvent_t e = c->event_pool.back();
    c->event_pool.pop_back();
    return e;
  }
  hipEvent_t e = nullptr;
  if (hipEventCreate(&e) != hipSuccess) return nullptr;
  return e;
}

// An event-record node appended to the graph being captured on `st` (after the current capture
// dependencies, which it then replaces): the graph-API form of recording a timing event inside a
// captured sequence.  Falls back to hipEventRecordWithFlags(..., hipEventRecordExternal).  A failed
// attempt's error is cleared so it does not surface at the next launch's hipGetLastError.
static bool capture_event(hipStream_t st, hipEvent_t ev) {
  hipStreamCaptureStatus status;
  unsigned long long id = 0;
  hipGraph_t g = nullptr;
  const hipGraphNode_t* deps = nullptr;
  size_t ndeps = 0;
  if (hipStreamGetCaptureInfo_v2(st, &status, &id, &g, &deps, &ndeps) == hipSuccess &&
      status == hipStreamCaptureStatusActive && g) {
    hipGraphNode_t node = nullptr;
    if (hipGraphAddEventRecordNode(&node, g, deps, ndeps, ev) == hipSuccess &&
        hipStreamUpdateCaptureDependencies(st, &node, 1, hipStreamSetCaptureDependencies) == hipSuccess)
      return true;
  }
  (void)hipGetLastError();
  if (hipEventRecordWithFlags(ev, st, hipEventRecordExternal) == hipSuccess) return true;
  (void)hipGetLastError();
  return false;
}

// Brackets a kernel launch with HIP events on the context stream when timing is enabled.  While
// capturing, the events become event-record nodes of the graph (hipEventRecordExternal), owned by
// the graph: every replay re-records them, so the launch is timed inside the replayed graph.
struct LaunchTimer {
  vw_ctx* c;
  TimedLaunch tl;
  bool on;
  LaunchTimer(vw_ctx* ctx, const char* family) : c(ctx), on(ctx->timing) {
    if (!on) return;
    tl.family = family;
    if (c->capturing) {
      tl.graph_owned = true;
      tl.start = tl.stop = nullptr;
      if (hipEventCreate(&tl.start) != hipSuccess || hipEventCreate(&tl.stop) != hipSuccess ||
          !capture_event(c->stream, tl.start)) {
        if (tl.start) hipEventDestroy(tl.start);
        if (tl.stop) hipEventDestroy(tl.stop);
        on = false;
      }
      return;
    }
    tl.start = pool_event(c);
    tl.stop = pool_event(c);
    if (!tl.start || !tl.stop) { on = false; return; }
    hipEventRecord(tl.start, c->stream);
  }
  ~LaunchTimer() {
    if (!on) return;
    if (tl.graph_owned) {
      if (capture_event(c->stream, tl.stop)) {
        c->captured.push_back(tl);
      } else {
        hipEventDestroy(tl.start);
        hipEventDestroy(tl.stop);
      }
      return;
    }
    hipEventRecord(tl.stop, c->stream);
    c->pending.push_back(tl);
  }
};

static void collect_timing(vw_ctx* c) {
  for (auto& tl : c->pending) {
    float ms = 0.f;
    if (hipEventSynchronize(tl.stop) == hipSuccess && hipEventElapsedTime(&ms, tl.start, tl.stop) == hipSuccess) {
      auto& t = c->totals[tl.family];
      t.first += ms;
      t.second += 1;
    }
    if (!tl.graph_owned) {
      c->event_pool.push_back(tl.start);
      c->event_pool.push_back(tl.stop);
    }
  }
  c->pending.clear();
}

static vw_status ensure_ws(vw_ctx* c, size_t bytes) {
  if (bytes <= c->ws_bytes) return VW_OK;
  if (c->capturing) return fail(VW_ERR_STATE, "workspace growth during capture: run the call once before capturing it");
  if (c->ws) {
    // the workspace may have been used on streams the context was bound to before: drain the device
    hipDeviceSynchronize();
    ++c->ws_gen;
    hipFree(c->ws);
    c->ws = nullptr;
    c->ws_bytes = 0;
  }
  size_t want = std::max(bytes, (size_t)1 << 20);
  VW_HIP(hipMalloc(&c->ws, want));
  c->ws_bytes = want;
  return VW_OK;
}

// the REF_NONFINITE row flags: zeroed once at allocation, kept zero by the kernels that consume them
static vw_status ensure_nf(vw_ctx* c, int64_t B) {
  if (B <= c->nf_rows) return VW_OK;
  if (c->capturing) return fail(VW_ERR_STATE, "row-flag growth during capture: run the call once before capturing it");
  if (c->nf) {
    hipDeviceSynchronize();
    ++c->ws_gen;
    hipFree(c->nf);
    c->nf = nullptr;
    c->nf_rows = 0;
  }
  const int64_t rows = std::max<int64_t>(B, 4096);
  VW_HIP(hipMalloc(&c->nf, (size_t)rows * sizeof(int)));
  VW_HIP(hipMemset(c->nf, 0, (size_t)rows * sizeof(int)));
  VW_HIP(hipDeviceSynchronize());
  c->nf_rows = rows;
  return VW_OK;
}

static inline size_t align_up(size_t v, size_t a) { return (v + a - 1) / a * a; }
static inline int64_t round_up(int64_t v, int64_t a) { return (v + a - 1) / a * a; }

// ------------------------------------------------------------------------------------------------
// Bookkeeping restated from the reference.

// MultiLevelMODWTTransform.calculateMaxLevels  core/modwt/MultiLevelMODWTTransform.java:455-501
extern "C" int vw_max_levels(int64_t N, int L) {
  if (L <= 0 || N <= L) return 0;
  int max_level = 1;
  const long long lm1 = L - 1;
  while (max_level < 10) {
    const long long scaled = lm1 * (1LL << (max_level - 1)) + 1LL;
    if (scaled > N) break;
    max_level++;
  }
  return max_level - 1;
}

extern "C" int64_t vw_upsampled_length(int L, int level) {
  const int64_t up = (level <= 1) ? 1 : ((int64_t)1 << (level - 1));
  return (int64_t)(L - 1) * up + 1;
}

// SymmetricAlignmentStrategy.decide  core/modwt/SymmetricAlignmentStrategy.java:43-117
static void sym_decide(int wid, int L, int level, int* ap, int* dh, int* dp, int* dg) {
  int detailPlus = 1, deltaG = 0, deltaH = 0;
  const bool isHaar = L <= 2;
  int approxPlus = isHaar ? 1 : 0;
  if (isHaar) {
    deltaG = 0;
    deltaH = (level <= 1) ? 0 : -1;
  } else if (wid == VW_WID_DB6) {
    deltaH = (level <= 1) ? 0 : -1;
    deltaG = (level >= 3) ? 1 : 0;
  } else if (wid == VW_WID_DB8) {
    deltaH = (level <= 1) ? 0 : 1;
    deltaG = (level >= 2) ? 1 : 0;
  } else if (wid == VW_WID_SYM4) {
    approxPlus = 1; detailPlus = 0; deltaH = 0; deltaG = 0;
  } else if (wid == VW_WID_SYM8) {
    if (level <= 1) { deltaH = 0; deltaG = 0; }
    else if (level == 2) { deltaH = 1; deltaG = 0; }
    else { deltaH = 1; deltaG = 1; }
  } else if (wid == VW_WID_COIF2) {
    approxPlus = 1; deltaH = (level <= 1) ? 0 : 1; detailPlus = 0; deltaG = 0;
  } else if (wid == VW_WID_COIF3) {
    detailPlus = 0;
    if (level <= 1) { deltaH = 0; deltaG = 0; } else { deltaH = -1; deltaG = 1; }
  } else if (L >= 12) {
    if (level <= 1) { deltaH = 0; deltaG = 0; }
    else { const bool even = level % 2 == 0; deltaH = even ? 0 : -1; deltaG = even ? 0 : -1; }
  } else {
    if (level <= 1) { deltaH = 0; deltaG = 0; } else { deltaH = -1; deltaG = 0; }
  }
  *ap = approxPlus; *dh = deltaH; *dp = detailPlus; *dg = deltaG;
}

// MultiLevelMODWTTransform.computeTauJ  core/modwt/MultiLevelMODWTTransform.java:795-806
static int compute_tau(int base_len, int level) {
  const int lm1 = base_len - 1;
  if (level <= 1) return std::max(0, lm1 / 2);
  const long long up = 1LL << (level - 1);
  const long long Lj = (long long)lm1 * up + 1LL;
  const long long tau = (Lj - 1LL) / 2LL;
  if (tau < 0) return 0;
  if (tau > 2147483647LL) return 2147483647;
  return (int)tau;
}

static int next_pow2(int64_t n) {
  int64_t p = 1;
  while (p < n) p <<= 1;
  return (int)p;
}

static bool is_pow2(int64_t n) { return n > 0 && (n & (n - 1)) == 0; }

// Level-j input index range read by a branch (dir, off) for outputs t in [0, tmax].
static void branch_extent(int N, int tmax, int L, int s, int dir, int off, int* hl, int* hr) {
  const long long reach = (long long)(L - 1) * s;
  long long mn, mx;
  if (dir > 0) { mn = off; mx = (long long)tmax + reach + off; }
  else { mn = (long long)off - reach; mx = (long long)tmax + off; }
  *hl = (int)std::max<long long>(*hl, -mn);
  *hr = (int)std::max<long long>(*hr, mx - (N - 1));
}

template <typename T> static constexpr int vec_width() { return 16 / (int)sizeof(T); }

static bool aligned16(const void* p) { return ((uintptr_t)p & 15u) == 0; }

// ------------------------------------------------------------------------------------------------
// Context
extern "C" vw_status vw_ctx_create(int device, vw_ctx** out) {
  if (!out) return fail(VW_ERR_NULL, "out is null");
  int n = 0;
  VW_HIP(hipGetDeviceCount(&n));
  if (device < 0 || device >= n) return fail(VW_ERR_ARG, "device %d out of range (%d devices)", device, n);
  VW_HIP(hipSetDevice(device));
  vw_ctx* c = new vw_ctx();
  c->device = device;
  c->tune = read_tuning();
  { int n = 0; if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, device) == hipSuccess && n > 0) c->cus = n; }
  if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return fail(VW_ERR_DEVICE, "hipStreamCreate failed");
  }
  c->own_stream = true;
  if (hipMalloc(&c->bad, sizeof(unsigned long long)) != hipSuccess) {
    hipStreamDestroy(c->stream);
    delete c;
    return fail(VW_ERR_DEVICE, "hipMalloc failed");
  }
  *out = c;
  return ok();
}

extern "C" vw_status vw_ctx_destroy(vw_ctx* c) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  hipSetDevice(c->device);
  if (c->capturing) {  // an unfinished capture: end it and drop what it recorded
    hipGraph_t gph = nullptr;
    if (hipStreamEndCapture(c->stream, &gph) == hipSuccess && gph) hipGraphDestroy(gph);
    (void)hipGetLastError();
    for (auto& t : c->captured) { hipEventDestroy(t.start); hipEventDestroy(t.stop); }
    c->captured.clear();
    c->capturing = false;
  }
  hipStreamSynchronize(c->stream);
  kill_pipelines_of(c);
  hipSetDevice(c->device);
  collect_timing(c);
  // graphs outliving their context: free their HIP objects now; the handles stay valid for
  // vw_graph_destroy, and vw_graph_launch on them fails with VW_ERR_STATE
  for (vw_graph* gr : c->graphs) {
    release_graph(gr);
    gr->ctx = nullptr;
  }
  c->graphs.clear();
  for (auto e : c->event_pool) hipEventDestroy(e);
  if (c->ws) hipFree(c->ws);
  if (c->ws2) hipFree(c->ws2);
  if (c->med) hipFree(c->med);
  if (c->nf) hipFree(c->nf);
  for (auto& b : c->stage) hipFree(b.first);
  if (c->bad) hipFree(c->bad);
  if (c->own_stream) hipStreamDestroy(c->stream);
  delete c;
  return ok();
}

// The device's null (legacy default) stream -- what torch uses when no stream is set: its handle is
// 0, which vw_ctx_set_stream reads as "own stream".
// Rebinding the context: work already enqueued on the old stream (it may still use the shared
// workspaces ws / ws2) is ordered before anything the new stream runs -- an event on the old stream
// that the new one waits for.  An owned stream is drained and destroyed instead.
static vw_status rebind_stream(vw_ctx* c, hipStream_t next, bool own_next) {
  if (c->capturing) return fail(VW_ERR_STATE, "stream change during capture");
  hipStream_t prev = c->stream;
  if (c->own_stream) {
    VW_HIP(hipStreamSynchronize(prev));
    VW_HIP(hipStreamDestroy(prev));
    c->own_stream = false;
  } else if (prev != next) {
    hipEvent_t ev = nullptr;
    VW_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
    hipError_t e = hipEventRecord(ev, prev);
    if (e == hipSuccess && next) e = hipStreamWaitEvent(next, ev, 0);
    if (e == hipSuccess && !next) e = hipEventSynchronize(ev);  // the legacy null stream: drain
    hipEventDestroy(ev);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "stream ordering failed: %s", hipGetErrorString(e));
  }
  c->stream = next;
  c->own_stream = own_next;
  return VW_OK;
}

extern "C" vw_status vw_ctx_use_null_stream(vw_ctx* c) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  VW_TRY(rebind_stream(c, nullptr, false));
  return ok();
}

extern "C" vw_status vw_ctx_set_stream(vw_ctx* c, void* s) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (s) {
    VW_TRY(rebind_stream(c, (hipStream_t)s, false));
  } else {
    hipStream_t ns = nullptr;
    VW_HIP(hipStreamCreateWithFlags(&ns, hipStreamNonBlocking));
    VW_TRY(rebind_stream(c, ns, true));
  }
  return ok();
}

// ------------------------------------------------------------------------------------------------
// Captured steps: the calls made between vw_capture_begin and vw_capture_end are recorded (stream
// capture of the context stream) into one executable HIP graph, replayed by vw_graph_launch with
// one host call -- the host-side planning, argument packing and per-kernel launch cost of the
// transforms are paid once at capture.  Calls that must synchronize (validation, host memory,
// SYNC, workspace growth) are rejected while capturing.

extern "C" vw_status vw_capture_begin(vw_ctx* c) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (c->capturing) return fail(VW_ERR_STATE, "already capturing");
  if (!c->stream) return fail(VW_ERR_STATE, "the null stream cannot be captured; bind a stream first");
  hipSetDevice(c->device);
  VW_HIP(hipStreamBeginCapture(c->stream, hipStreamCaptureModeThreadLocal));
  c->capturing = true;
  c->captured.clear();
  return ok();
}

extern "C" vw_status vw_capture_end(vw_ctx* c, vw_graph** out) {
  if (!c || !out) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (!c->capturing) return fail(VW_ERR_STATE, "not capturing");
  hipSetDevice(c->device);
  c->capturing = false;
  std::vector<TimedLaunch> timed;
  timed.swap(c->captured);
  auto drop = [&] { for (auto& t : timed) { hipEventDestroy(t.start); hipEventDestroy(t.stop); } };
  hipGraph_t graph = nullptr;
  hipError_t ec = hipStreamEndCapture(c->stream, &graph);
  if (ec != hipSuccess) {
    drop();
    return fail(VW_ERR_DEVICE, "hipStreamEndCapture: %s", hipGetErrorString(ec));
  }
  hipGraphExec_t exec = nullptr;
  hipError_t e = hipGraphInstantiate(&exec, graph, nullptr, nullptr, 0);
  if (e != hipSuccess) {
    hipGraphDestroy(graph);
    drop();
    return fail(VW_ERR_DEVICE, "graph instantiate failed: %s", hipGetErrorString(e));
  }
  vw_graph* gr = new vw_graph();
  gr->timed.swap(timed);
  gr->ctx = c;
  gr->device = c->device;
  gr->ws_gen = c->ws_gen;
  gr->graph = graph;
  gr->exec = exec;
  c->graphs.insert(gr);
  *out = gr;
  return ok();
}


extern "C" vw_status vw_graph_launch(vw_graph* gr, int64_t count) {
  if (!gr) return fail(VW_ERR_NULL, "graph is null");
  vw_ctx* c = gr->ctx;
  if (!c) return fail(VW_ERR_STATE, "the context of this graph was destroyed");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (gr->ws_gen != c->ws_gen)
    return fail(VW_ERR_STATE, "the context workspace moved since this graph was recorded; record it again");
  hipSetDevice(c->device);
  for (int64_t i = 0; i < count; ++i) VW_HIP(hipGraphLaunch(gr->exec, c->stream));
  // Timed launches recorded inside the graph: their events hold the LAST replay only, so a graph's
  // entries are pending at most once (a second launch before a collect replaces, not duplicates, them).
  if (c->timing && count > 0 && !gr->timed.empty()) {
    std::set<hipEvent_t> mine;
    for (const auto& t : gr->timed) mine.insert(t.start);
    c->pending.erase(std::remove_if(c->pending.begin(), c->pending.end(),
                                    [&](const TimedLaunch& t) { return t.graph_owned && mine.count(t.start); }),
                     c->pending.end());
    for (const auto& t : gr->timed) c->pending.push_back(t);
  }
  return ok();
}

extern "C" vw_status vw_graph_destroy(vw_graph* gr) {
  if (!gr) return fail(VW_ERR_NULL, "graph is null");
  vw_ctx* c = gr->ctx;
  if (!c) {  // context already destroyed: it released the HIP objects
    delete gr;
    return ok();
  }
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  hipStreamSynchronize(c->stream);
  collect_timing(c);  // pending entries may reference this graph's events
  release_graph(gr);
  c->graphs.erase(gr);
  delete gr;
  return ok();
}

// ------------------------------------------------------------------------------------------------
// Pipelined round trips (include/vectorwave_amd.h "pipelined round trips").  Step i runs the forward
// of buffer set i mod R on the forward context's stream and then, after an event, its inverse on the
// inverse context's stream; step i's forward waits for step i - R's inverse (the set it overwrites).
// So step i + 1's forward runs beside step i's inverse while every step still does its whole forward
// and inverse.  The loop is issued here, in C++, so a small shard (the 8-GPU headline: 512 rows,
// ~50 us of GPU work per step) is not limited by a Python caller's per-call overhead.
struct vw_pipeline {
  vw_ctx* cf = nullptr;
  vw_ctx* ci = nullptr;
  int device = 0;
  int esz = 8;
  int R = 0;
  std::vector<void*> x, det, app, y;
  int64_t B = 0, N = 0;
  std::vector<double> lo, hi;
  int L = 0, wavelet_id = 0, boundary = 0, J = 0;
  unsigned flags = 0;
  std::vector<hipEvent_t> ev_f, ev_i;
  std::vector<char> live;
  hipEvent_t join_ev = nullptr;
  int64_t next = 0;       // index of the next step (selects its buffer set)
  bool dead = false;      // a context was destroyed under it
  std::mutex mu;          // run / join / kill: a kill waits until an in-flight run has issued its steps
};

static std::mutex g_pipe_mu;
static std::set<vw_pipeline*> g_pipes;

static void release_pipeline(vw_pipeline* p) {
  for (auto e : p->ev_f) if (e) hipEventDestroy(e);
  for (auto e : p->ev_i) if (e) hipEventDestroy(e);
  if (p->join_ev) hipEventDestroy(p->join_ev);
  p->ev_f.clear();
  p->ev_i.clear();
  p->join_ev = nullptr;
}

// vw_ctx_destroy: pipelines that use the context die with it (their events are freed, the handles
// stay valid for vw_pipeline_destroy, vw_pipeline_run fails with VW_ERR_STATE)
static void kill_pipelines_of(vw_ctx* c) {
  std::lock_guard<std::mutex> g(g_pipe_mu);
  for (vw_pipeline* p : g_pipes)
    if (!p->dead && (p->cf == c || p->ci == c)) {
      std::lock_guard<std::mutex> pg(p->mu);
      hipSetDevice(p->device);
      hipStreamSynchronize(p->cf->stream);
      hipStreamSynchronize(p->ci->stream);
      release_pipeline(p);
      p->dead = true;
    }
}

extern "C" vw_status vw_pipeline_create(vw_ctx* cf, vw_ctx* ci, int elem_bytes, int sets, void* const* x,
                                        void* const* details, void* const* approx, void* const* y, int64_t B,
                                        int64_t N, const double* lo, const double* hi, int L, int wavelet_id,
                                        int boundary, int J, unsigned flags, vw_pipeline** out) {
  if (!cf || !ci || !x || !details || !approx || !y || !lo || !hi || !out) return fail(VW_ERR_NULL, "null argument");
  if (elem_bytes != 8 && elem_bytes != 4) return fail(VW_ERR_ARG, "elem_bytes must be 8 (f64) or 4 (f32)");
  if (sets < 1 || sets > 1024) return fail(VW_ERR_ARG, "sets must be in [1, 1024]");
  if (B <= 0 || N <= 0) return fail(VW_ERR_EMPTY, "Signals cannot be null or empty");
  if (L <= 0 || L > kMaxTaps) return fail(VW_ERR_ARG, "filter length %d out of range", L);
  if (J < 1) return fail(VW_ERR_ARG, "levels must be >= 1");
  if (cf->device != ci->device) return fail(VW_ERR_ARG, "both contexts must be on one device");
  // calls that synchronize or stage host memory have no place in an asynchronous pipeline
  if (flags & (VW_FLAG_HOST_MEMORY | VW_FLAG_SYNC | VW_FLAG_VALIDATE))
    return fail(VW_ERR_ARG, "pipeline steps take device buffers, no SYNC / VALIDATE / HOST_MEMORY");
  for (int r = 0; r < sets; ++r)
    if (!x[r] || !details[r] || !approx[r] || !y[r]) return fail(VW_ERR_NULL, "buffer set %d has a null pointer", r);
  if (cf->capturing || ci->capturing) return fail(VW_ERR_STATE, "a context is capturing");
  vw_pipeline* p = new vw_pipeline();
  p->cf = cf;
  p->ci = ci;
  p->device = cf->device;
  p->esz = elem_bytes;
  p->R = sets;
  p->x.assign(x, x + sets);
  p->det.assign(details, details + sets);
  p->app.assign(approx, approx + sets);
  p->y.assign(y, y + sets);
  p->B = B;
  p->N = N;
  p->lo.assign(lo, lo + L);
  p->hi.assign(hi, hi + L);
  p->L = L;
  p->wavelet_id = wavelet_id;
  p->boundary = boundary;
  p->J = J;
  p->flags = flags;
  hipSetDevice(p->device);
  p->ev_f.assign(sets, nullptr);
  p->ev_i.assign(sets, nullptr);
  p->live.assign(sets, 0);
  hipError_t e = hipEventCreateWithFlags(&p->join_ev, hipEventDisableTiming);
  for (int r = 0; r < sets && e == hipSuccess; ++r) {
    e = hipEventCreateWithFlags(&p->ev_f[r], hipEventDisableTiming);
    if (e == hipSuccess) e = hipEventCreateWithFlags(&p->ev_i[r], hipEventDisableTiming);
  }
  if (e != hipSuccess) {
    release_pipeline(p);
    delete p;
    return fail(VW_ERR_DEVICE, "event creation failed: %s", hipGetErrorString(e));
  }
  {
    std::lock_guard<std::mutex> g(g_pipe_mu);
    g_pipes.insert(p);
  }
  *out = p;
  return ok();
}

extern "C" vw_status vw_pipeline_run(vw_pipeline* p, int64_t steps) {
  if (!p) return fail(VW_ERR_NULL, "pipeline is null");
  std::lock_guard<std::mutex> pg(p->mu);
  if (p->dead) return fail(VW_ERR_STATE, "a context of this pipeline was destroyed");
  if (steps < 0) return fail(VW_ERR_ARG, "steps must be >= 0");
  // a capture on either context would record one stream's half of each step and wait on events of the
  // other, uncaptured stream: an invalid graph
  if (p->cf->capturing || p->ci->capturing) return fail(VW_ERR_STATE, "a context of this pipeline is capturing");
  hipSetDevice(p->device);
  const bool f32 = p->esz == 4;
  for (int64_t k = 0; k < steps; ++k) {
    const int r = (int)(p->next % p->R);
    hipStream_t sf = p->cf->stream, si = p->ci->stream;
    if (p->live[r]) VW_HIP(hipStreamWaitEvent(sf, p->ev_i[r], 0));
    vw_status st = f32 ? vw_modwt_forward_f32(p->cf, (const float*)p->x[r], p->B, p->N, p->N, p->lo.data(),
                                              p->hi.data(), p->L, p->wavelet_id, p->boundary, p->J, p->flags,
                                              (float*)p->det[r], (float*)p->app[r])
                       : vw_modwt_forward_f64(p->cf, (const double*)p->x[r], p->B, p->N, p->N, p->lo.data(),
                                              p->hi.data(), p->L, p->wavelet_id, p->boundary, p->J, p->flags,
                                              (double*)p->det[r], (double*)p->app[r]);
    if (st != VW_OK) return st;
    VW_HIP(hipEventRecord(p->ev_f[r], sf));
    VW_HIP(hipStreamWaitEvent(si, p->ev_f[r], 0));
    st = f32 ? vw_modwt_inverse_f32(p->ci, (const float*)p->det[r], (const float*)p->app[r], p->B, p->N,
                                    p->lo.data(), p->hi.data(), p->L, p->wavelet_id, p->boundary, p->J, 0xFFFFFFFFu,
                                    0, p->flags, (float*)p->y[r])
             : vw_modwt_inverse_f64(p->ci, (const double*)p->det[r], (const double*)p->app[r], p->B, p->N,
                                    p->lo.data(), p->hi.data(), p->L, p->wavelet_id, p->boundary, p->J, 0xFFFFFFFFu,
                                    0, p->flags, (double*)p->y[r]);
    if (st != VW_OK) return st;
    VW_HIP(hipEventRecord(p->ev_i[r], si));
    p->live[r] = 1;
    ++p->next;
  }
  return ok();
}

extern "C" vw_status vw_pipeline_join(vw_pipeline* p) {
  if (!p) return fail(VW_ERR_NULL, "pipeline is null");
  std::lock_guard<std::mutex> pg(p->mu);
  if (p->dead) return fail(VW_ERR_STATE, "a context of this pipeline was destroyed");
  if (p->cf->capturing || p->ci->capturing) return fail(VW_ERR_STATE, "a context of this pipeline is capturing");
  hipSetDevice(p->device);
  VW_HIP(hipEventRecord(p->join_ev, p->ci->stream));
  VW_HIP(hipStreamWaitEvent(p->cf->stream, p->join_ev, 0));
  std::fill(p->live.begin(), p->live.end(), 0);
  return ok();
}

extern "C" int64_t vw_pipeline_last_set(vw_pipeline* p) {
  if (!p || p->next == 0) return -1;
  return (p->next - 1) % p->R;
}

extern "C" vw_status vw_pipeline_destroy(vw_pipeline* p) {
  if (!p) return fail(VW_ERR_NULL, "pipeline is null");
  {
    std::lock_guard<std::mutex> g(g_pipe_mu);
    g_pipes.erase(p);
  }
  if (!p->dead) {
    hipSetDevice(p->device);
    hipStreamSynchronize(p->cf->stream);
    hipStreamSynchronize(p->ci->stream);
    release_pipeline(p);
  }
  delete p;
  return ok();
}

extern "C" vw_status vw_ctx_set_option(vw_ctx* c, const char* key, int value) {
  if (!c || !key) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (!set_tuning(c->tune, key, value)) return fail(VW_ERR_ARG, "unknown option %s", key);
  return ok();
}

extern "C" void* vw_ctx_get_stream(vw_ctx* c) { return c ? (void*)c->stream : nullptr; }
extern "C" int vw_ctx_device(vw_ctx* c) { return c ? c->device : -1; }

extern "C" vw_status vw_ctx_synchronize(vw_ctx* c) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  hipSetDevice(c->device);
  VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

extern "C" const char* vw_last_error(void) { return t_err.c_str(); }
extern "C" int64_t vw_last_error_index(void) { return t_err_index; }
extern "C" const char* vw_version(void) { return "vectorwave_amd 0.1.0 (gfx950)"; }
extern "C" void vw_set_signal_base(int64_t base) { t_signal_base = base; }

extern "C" vw_status vw_ctx_enable_timing(vw_ctx* c, int enable) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  c->timing = enable != 0;
  return ok();
}

extern "C" vw_status vw_ctx_reset_timing(vw_ctx* c) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  collect_timing(c);
  c->totals.clear();
  return ok();
}

// Start / end of the not-yet-collected timed launches of `family` (the last replay of each graph, or
// the direct launches since the last collect), in ms after `ref_event` (a hipEvent_t recorded before
// them, on any stream of the device) -- for callers that run several contexts concurrently and need
// the wall window of a kernel family across them.  Call before vw_ctx_kernel_time, which consumes the
// launches.  *count receives the number found (at most max are written).
extern "C" vw_status vw_ctx_kernel_spans(vw_ctx* c, const char* family, void* ref_event, int64_t max,
                                         double* start_ms, double* end_ms, int64_t* count) {
  if (!c || !family || !ref_event || !count) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  int64_t n = 0;
  for (const auto& tl : c->pending) {
    if (tl.family != family) continue;
    float a = 0.f, b = 0.f;
    VW_HIP(hipEventSynchronize(tl.stop));
    VW_HIP(hipEventElapsedTime(&a, (hipEvent_t)ref_event, tl.start));
    VW_HIP(hipEventElapsedTime(&b, (hipEvent_t)ref_event, tl.stop));
    if (n < max) {
      if (start_ms) start_ms[n] = a;
      if (end_ms) end_ms[n] = b;
    }
    ++n;
  }
  *count = n;
  return ok();
}

extern "C" vw_status vw_ctx_kernel_time(vw_ctx* c, const char* family, double* total_ms, int64_t* launches) {
  if (!c || !family) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  collect_timing(c);
  auto it = c->totals.find(family);
  if (total_ms) *total_ms = it == c->totals.end() ? 0.0 : it->second.first;
  if (launches) *launches = it == c->totals.end() ? 0 : it->second.second;
  return ok();
}

// ------------------------------------------------------------------------------------------------
// Common argument checks (MultiLevelMODWTTransform.decompose :209-239, BatchMODWT.validateAoS :201-212)
static vw_status check_common(vw_ctx* c, const void* a, const void* b, const double* lo, const double* hi,
                              int64_t B, int64_t N, int L, int boundary) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  if (!a || !b || !lo || !hi) return fail(VW_ERR_NULL, "null array argument");
  if (B <= 0) return fail(VW_ERR_EMPTY, "batch must be non-empty (B=%lld)", (long long)B);
  if (N <= 0) return fail(VW_ERR_EMPTY, "Signal cannot be empty");
  if (N > (1LL << 30)) return fail(VW_ERR_ARG, "signal length %lld too large", (long long)N);
  if (boundary < VW_PERIODIC || boundary > VW_ZERO_PADDING)
    return fail(VW_ERR_BOUNDARY, "MODWT only supports PERIODIC, ZERO_PADDING, and SYMMETRIC boundary modes");
  if (L < 1 || L > kMaxTaps) return fail(VW_ERR_ARG, "filter length %d unsupported (1..%d)", L, kMaxTaps);
  return VW_OK;
}

static vw_status check_levels(int64_t N, int L, int J, unsigned flags) {
  if (flags & VW_FLAG_CORE_LEVELS) {
    const int maxl = vw_max_levels(N, L);
    if (J < 1 || J > maxl)
      return fail(VW_ERR_LEVEL, "Invalid number of decomposition levels: %d (valid 1..%d for N=%lld, L=%d)", J, maxl,
                  (long long)N, L);
  } else {
    if (J < 1) return fail(VW_ERR_LEVEL, "levels must be >= 1");
    if (J > kMaxLevels) return fail(VW_ERR_LEVEL, "levels %d exceeds engine limit %d", J, kMaxLevels);
    if (vw_upsampled_length(L, J) > (int64_t)1 << 30) return fail(VW_ERR_TOO_LARGE, "upsampled filter too long");
  }
  return VW_OK;
}

template <typename T>
static void copy_taps(T* dst, const double* src, int L) {
  // base taps * (1.0 / Math.sqrt(2.0)) in double, then rounded to T  (ScalarOps.java:911-914)
  const double s = 1.0 / std::sqrt(2.0);
  for (int i = 0; i < L; ++i) dst[i] = (T)(src[i] * s);
  for (int i = L; i < kMaxTaps; ++i) dst[i] = T(0);
}

// Calls that synchronize cannot be recorded into a graph (vw_capture_begin).
static vw_status capture_guard(vw_ctx* c, unsigned flags) {
  if (c->capturing && (flags & (VW_FLAG_VALIDATE | VW_FLAG_HOST_MEMORY | VW_FLAG_SYNC)))
    return fail(VW_ERR_STATE, "validation, host memory and SYNC cannot be captured");
  return VW_OK;
}

static vw_status read_bad(vw_ctx* c, unsigned long long* out) {
  VW_HIP(hipMemcpyAsync(out, c->bad, sizeof(unsigned long long), hipMemcpyDeviceToHost, c->stream));
  VW_HIP(hipStreamSynchronize(c->stream));
  return VW_OK;
}

static vw_status report_bad(unsigned long long bad, int64_t N) {
  if (bad == ~0ull) return VW_OK;
  const bool out = (bad >> 62) & 1ull;
  const unsigned long long flat = bad & ((1ull << 62) - 1);
  t_err_index = (int64_t)(flat % (unsigned long long)N);
  return fail(VW_ERR_NONFINITE, "%s contains non-finite value at index %lld (signal %lld)",
              out ? "coefficients" : "signal", (long long)(flat % (unsigned long long)N),
              (long long)(flat / (unsigned long long)N) + (long long)t_signal_base);
}

// Plan of a fused launch: threads, vectors per thread (4 or 8), LDS bytes.  NV = 4 keeps the
// per-thread register arrays small (no spills); NV = 8 reaches N = 1024 * 8 * V.  The workgroup is
// ceil(nvec / NV) threads (not rounded to a wave): thread `tid` owns vectors tid + k*threads, and
// the unrolled kernels rely on slabs 0..NV-2 being full, `fit` = (NV-1)*threads <= nvec (else the
// runtime-L kernel with a bounds check per vector runs).
static bool fused_plan(const Tuning& tu, int64_t N, int V, int elem, int64_t lds_elems_extra, int* threads, int* nv,
                       int* lds, bool* fit, int nv_req = 0) {
  const int64_t nvec = (N + V - 1) / V;
  int want = tu.nv;
  if ((nvec + want - 1) / want > 512) want = 8;  // NV = 4 kernels are bounded to 512 threads (VW_FUSED_BOUNDS)
  // NV = 2: 1024 threads at most, every slab full (the unrolled kernels' contract)
  if (nv_req == 2 && nvec % 2 == 0 && nvec / 2 <= kMaxThreads) want = 2;
  const int64_t th = (nvec + want - 1) / want;
  if (th > kMaxThreads) return false;
  const int64_t bytes = lds_elems_extra * elem;
  if (bytes > kLdsBytes) return false;
  *nv = want;
  *threads = (int)th;
  *lds = (int)bytes;
  *fit = (int64_t)(want - 1) * th <= nvec;
  return true;
}


// Owner-written halo of one level (vw_device.h halo_images): the affine images of an element and
// the vector bands that have them; `own` only when every band lies in the slab that checks it.
static void set_halo_images(LevelDesc& d, int64_t N, int64_t npow2, int V, int threads, int nv) {
  int64_t s_el = 0, e_el = N;
  d.il_a = 0; d.il_b = 1; d.ir_a = 0; d.ir_b = -1;  // no images
  switch (d.mode) {
    case kHaloPeriodic:
      d.il_a = 1; d.il_b = (int)-N; d.ir_a = 1; d.ir_b = (int)N;
      s_el = d.hr; e_el = N - d.hl;
      break;
    case kHaloSymmetric:
      d.il_a = -1; d.il_b = -1; d.ir_a = -1; d.ir_b = (int)(2 * N - 1);
      s_el = d.hl; e_el = N - d.hr;
      break;
    case kHaloFftPad:
      d.il_a = 1; d.il_b = (int)-npow2;
      e_el = npow2 - d.hl;
      break;
    default:
      break;
  }
  e_el = std::min<int64_t>(std::max<int64_t>(e_el, 0), N);
  d.vs = (int)((s_el + V - 1) / V);
  d.ve = (int)(e_el / V);
  d.own = (d.hl <= N && d.hr <= N && d.vs <= threads && (int64_t)d.ve >= (int64_t)(nv - 1) * threads) ? 1 : 0;
}

// Level groups of the per-level path (vw_device.h k_forward_multi / k_inverse_multi): from level 1
// up, consecutive PERIODIC levels run as one multi-level tile launch while their combined reach
// sum((L-1)*s_j) stays within a quarter of the tile (the redundant arithmetic).  groups[j-1] = size
// of the group starting at level j (0 inside a group, 1 = the per-level kernels).  VW_MULTI=0
// disables; VW_MULTI_TILE / VW_MULTI_DIV tune tile and reach bound.
template <typename T>
static int multi_tile(const Tuning& tu) {
  constexpr int V = vec_width<T>();
  const int v = tu.multi_tile ? tu.multi_tile : (int)(16384 / sizeof(T));
  return v >= 64 * V ? v / V * V : 64 * V;
}

static std::vector<int> level_groups(const Tuning& tu, const std::vector<LevelDesc>& lv, int J, int L, int V, int tile,
                                     bool ok) {
  std::vector<int> g(J, 1);
  if (!ok || !tu.multi) return g;
  const int64_t cap = tile / tu.multi_div;
  for (int j = 1; j <= J;) {
    int n = 0;
    int64_t ext = 0;
    while (j + n <= J && n < kMaxGroup && lv[j + n - 1].mode == kHaloPeriodic) {
      const int64_t e2 = ext + round_up((int64_t)(L - 1) * lv[j + n - 1].s, V);
      if (e2 > cap) break;
      ext = e2;
      ++n;
    }
    if (n >= 2) {
      g[j - 1] = n;
      for (int k = 1; k < n; ++k) g[j - 1 + k] = 0;
      j += n;
    } else {
      ++j;
    }
  }
  return g;
}

// Level group of the chained column sweeps (vw_device.h k_inverse_sweep2 / k_inverse_sweep3): inverse levels
// j .. j-levels+1 (spacings G*h .. h, G = 2 / 4), all column-sweep levels outside the multi-level tile
// groups, PERIODIC / dir +1 / offset 0.  Picks KA (outputs per thread and step) and R (residues per
// group, 64 or 32 = h's alignment) under the kernels' rules: a block of G*KA positions covers the
// reach of the levels below the top (L-1 per level, in the bottom level's positions: 1 / 2 steps), the
// LDS rings (1 / 2 of 3 blocks x R) fit, one wrap mod N at most, and residue classes of >= 64 blocks.
template <typename T>
static bool sweepg_plan(const Tuning& tu, const std::vector<LevelDesc>& lv, int j, int levels, int L, int64_t N,
                        const std::vector<char>& in_group, const std::vector<int>& start_of, int* ka_out, int* r_out) {
  if (levels < 2 || levels > 3 || j < levels) return false;
  const int G = levels == 2 ? 2 : 4;
  const int64_t h = lv[j - levels].s;
  if (h < kSweepMinS || h % 32 != 0 || lv[j - 1].s != G * h) return false;
  for (int k = j - levels + 1; k <= j; ++k) {
    const LevelDesc& d = lv[k - 1];
    if (d.mode != kHaloPeriodic || d.dir_a != 1 || d.dir_d != 1 || d.off_a != 0 || d.off_d != 0) return false;
    if (k < j && (in_group[k] || start_of[k] != 0)) return false;
  }
  const int R = (h % 64 == 0 && tu.sweep2_r != 32) ? 64 : 32;
  const int kmin = (levels == 2 ? 1 : 2) * (L - 1);
  for (int ka : {L <= 17 ? tu.sweep2_ka : 16, 16}) {
    for (int r : {R, 32}) {
      const int64_t kb = (int64_t)G * ka;
      const int64_t lds = (levels == 2 ? 1 : 2) * 3 * kb * r * (int64_t)sizeof(T);
      if (kb < kmin || lds > kLdsBytes || h % r != 0) continue;
      if (N % (G * h) != 0 || (2 * kb + 2 * L) * G * h > N) continue;
      // short residue classes: the pipeline's fill (2 / 4 steps per chunk) is not amortised -- on sym8
      // 16384-sample signals through the tiled path a triple ran 21.2 ms vs 12.3 for pairs
      // (profiles/r03/ab_sweepg_short.log); such levels keep one sweep each
      if (N / h < (int64_t)tu.sweep2_minb * kb) continue;
      *ka_out = ka;
      *r_out = r;
      return true;
    }
  }
  return false;
}

// Streaming deep group (vw_deep.hip): PERIODIC levels jlo..jhi of the per-level path in one launch.
// Needs level jlo's spacing P to divide N and hold C = 64 bytes of residues; every ring of the group
// within the LDS budget.  Ring capacities: DMA-fed rings hold their history + two tiles (the next
// tile lands while the current one computes), multiples of 16 positions (one wave's DMA);
// level-fed rings history + one tile.  Returns the LDS bytes, 0 if the group does not qualify.
constexpr int kDeepTile = 128;  // vw_deep.hip kDeepT

template <typename T>
static int deep_plan(const Tuning& tu, const std::vector<LevelDesc>& lv, int jlo, int jhi, int L, int64_t N,
                     bool inverse, DeepArgs<T>* a) {
  constexpr int V = vec_width<T>();
  const int C = 64 / (int)sizeof(T);
  const int g = jhi - jlo + 1;
  if (!(inverse ? tu.deep_inv : tu.deep) || g < 1 || g > kMaxGroup || !has_unrolled_taps(L)) return 0;
  const int P = lv[jlo - 1].s;
  if (P < C || P % C != 0 || N % P != 0 || N / P < 2 * kDeepTile) return 0;
  for (int j = jlo; j <= jhi; ++j)
    if (lv[j - 1].mode != kHaloPeriodic) return 0;
  (void)V;
  int caps[2 * kMaxGroup] = {}, nr = 0;
  int64_t reach = 0;
  const int D = inverse ? tu.deep_pf_inv : tu.deep_pf_fwd;
  for (int k = 0; k < g; ++k) {
    const int64_t H = (int64_t)(L - 1) << k;
    reach += H;
    const bool dma_fed = inverse ? (k == g - 1) : (k == 0);
    caps[k] = dma_fed ? (int)round_up(H + (D + 1) * kDeepTile, 16) : (int)(H + kDeepTile);
    if (inverse) caps[g + k] = (int)round_up(H + (D + 1) * kDeepTile, 16);
  }
  nr = inverse ? 2 * g : g;
  int64_t pos = 0;
  for (int r = 0; r < nr; ++r) pos += caps[r];
  const int64_t bytes = pos * 64;
  if (bytes > (int64_t)tu.deep_lds * 1024 || bytes > kLdsBytes) return 0;
  if (a) {
    a->P = P; a->C = C; a->nq = (int)(N / P); a->nb = P / C; a->g = g; a->N = (int)N;
    a->warm = (int)round_up(reach, kDeepTile);
    a->depth = D;
    int64_t o = 0;
    for (int r = 0; r < nr; ++r) { a->cap[r] = caps[r]; a->off[r] = (int)(o * C); o += caps[r]; }
  }
  return (int)bytes;
}

// Segments per residue block: enough workgroups for `deep_waves` per CU, each segment at least four
// warm-ups long (the warm-up is recomputed per segment).
template <typename T>
static void deep_segments(const Tuning& tu, int cus, int64_t B, DeepArgs<T>* a) {
  const int64_t wg0 = B * a->nb;
  int64_t seg = std::max<int64_t>(1, ((int64_t)tu.deep_waves * cus + wg0 - 1) / wg0);
  seg = std::min<int64_t>(seg, std::max<int64_t>(1, a->nq / (4 * (int64_t)a->warm)));
  a->seg = (int)seg;
  a->seglen = (int)round_up((a->nq + seg - 1) / seg, kDeepTile);
  a->seg = (int)((a->nq + a->seglen - 1) / a->seglen);
}

// ------------------------------------------------------------------------------------------------
// VW_FLAG_REF_NONFINITE (vw_ref.hip): after the fast kernels, flag the rows holding a non-finite value
// in any of `planes` (the call's inputs and outputs: an overflow to Inf inside the cascade shows in an
// output), then recompute those rows with the reference's full-tap loops.  Stream-ordered, capturable
// once the workspace has grown.
template <typename T>
struct ScanPlane {
  const T* p;
  int64_t ld;
  int len;  // 0: the call's N
};

template <typename T>
static vw_status ref_nonfinite(vw_ctx* c, const std::vector<ScanPlane<T>>& planes, RefArgs<T>& r,
                               bool inverse, bool flagged) {
  const int64_t B = r.B, N = r.N;
  if ((int)planes.size() > kRefPlanes) return fail(VW_ERR_ARG, "too many planes for the non-finite scan");
  // rows recomputed at once: one workgroup each, two running-approximation rows of scratch (<= 512 MiB)
  int64_t grid = std::min<int64_t>(B, c->tune.ref_grid > 0 ? c->tune.ref_grid : 2LL * c->cus);
  grid = std::max<int64_t>(1, std::min<int64_t>(grid, ((int64_t)512 << 20) / (2 * N * (int64_t)sizeof(T))));
  VW_TRY(ensure_nf(c, B));
  VW_TRY(ensure_ws(c, (size_t)grid * 2 * (size_t)N * sizeof(T)));
  // timing families: "ref_nonfinite" (the cascade over rows the fast kernel flagged), "ref_nonfinite_scan"
  // (scan + cascade)
  LaunchTimer lt(c, flagged ? "ref_nonfinite" : "ref_nonfinite_scan");
  hipError_t e;
  if (!flagged) {  // the fast kernel did not probe its rows: scan the call's planes
    RefScan<T> s;
    memset(&s, 0, sizeof(s));
    for (const auto& p : planes) {
      s.p[s.np] = p.p;
      s.ld[s.np] = p.ld;
      s.len[s.np] = p.len;
      ++s.np;
    }
    s.B = B; s.N = (int)N; s.chunks = ref_scan_chunks((int)N); s.flag = c->nf;
    e = launch_flag_nonfinite<T>(s, c->stream);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "non-finite scan launch failed: %s", hipGetErrorString(e));
  }
  r.flag = c->nf;
  r.scratch = reinterpret_cast<T*>(c->ws);
  e = launch_ref_cascade<T>(r, (int)grid, inverse, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "reference-arithmetic launch failed: %s", hipGetErrorString(e));
  return VW_OK;
}

// the matrix-core kernels are fp32 only (vw_mfma.hip); the double overloads are never reached
static hipError_t mfma_forward(const FwdArgs<float>& a, int lds, hipStream_t st) { return launch_forward_mfma(a, lds, st); }
static hipError_t mfma_forward(const FwdArgs<double>&, int, hipStream_t) { return hipErrorNotSupported; }
static hipError_t mfma_inverse(const InvArgs<float>& a, int lds, hipStream_t st) { return launch_inverse_mfma(a, lds, st); }
static hipError_t mfma_inverse(const InvArgs<double>&, int, hipStream_t) { return hipErrorNotSupported; }

static int ref_mode(int boundary) {
  return boundary == VW_PERIODIC ? kHaloPeriodic : boundary == VW_ZERO_PADDING ? kHaloZero : kHaloSymmetric;
}

// ------------------------------------------------------------------------------------------------
// Forward (multi-level and single-level share this path).
template <typename T>
static vw_status forward_impl(vw_ctx* c, const T* x, int64_t B, int64_t N, int64_t ldx, const double* lo,
                              const double* hi, int L, int boundary, int J, unsigned flags, T* details, T* approx,
                              bool single_level, int mode_override, T* const* hist, bool hist_update,
                              T* const* hist_snap = nullptr, bool hist_first = false) {
  constexpr int V = vec_width<T>();
  VW_TRY(capture_guard(c, flags));
  const bool fma = flags & VW_FLAG_FMA;
  const bool validate = flags & VW_FLAG_VALIDATE;
  const int64_t nvec = (N + V - 1) / V;

  std::vector<LevelDesc> lv(J);
  int max_hl = 0;
  const int npow2 = next_pow2(N);
  for (int j = 1; j <= J; ++j) {
    LevelDesc& d = lv[j - 1];
    memset(&d, 0, sizeof(d));
    d.s = 1 << (j - 1);
    const int64_t Lj = vw_upsampled_length(L, j);
    d.hl = (int)(Lj - 1);
    d.hr = 0;
    d.hist_len = (int)(Lj - 1);
    if (boundary == VW_PERIODIC) {
      d.mode = kHaloPeriodic;
      // MultiLevelMODWTTransform.applyScaledMODWT :734-742 + FftHeuristics :30-34
      if ((flags & VW_FLAG_FFT_SWITCH) && !single_level && !(N < 64 || Lj > N / 2) && N >= 1024 &&
          (double)Lj > N * (1.0 / 8.0) && !is_pow2(N))
        d.mode = kHaloFftPad;
    } else {
      d.mode = boundary == VW_ZERO_PADDING ? kHaloZero : kHaloSymmetric;
    }
    if (mode_override >= 0) d.mode = mode_override;
    max_hl = std::max(max_hl, d.hl);
  }
  // VW_FLAG_REF_NONFINITE on a streaming block: keep the histories this block reads (the kernels
  // overwrite them) for the rows vw_ref.hip recomputes
  if ((flags & VW_FLAG_REF_NONFINITE) && hist && hist_update && hist_snap && !hist_first && J >= 2)
    for (int j = 0; j < J; ++j)
      if (lv[j].hist_len > 0)
        VW_HIP(hipMemcpyAsync(hist_snap[j], hist[j], (size_t)B * lv[j].hist_len * sizeof(T), hipMemcpyDeviceToDevice,
                              c->stream));

  const int hlpad = (int)round_up(max_hl, V);
  int threads = 0, lds = 0, nv = 4;
  // Level buffers: two (one barrier per level) or one (two barriers per level, but half the LDS:
  // twice the workgroups per CU).  Measured on MI355X (db4 J=6, 4096 x 4096 fp64): two buffers win
  // whenever the persistent forward (which needs them) runs -- FMA and EXACT alike; without it the
  // EXACT kernel is faster with one buffer (more workgroups to overlap its longer arithmetic).
  // VW_FWD_BUF=1|2 overrides.
  //
  // Persistent variant (vw_device.h k_forward_persist): next row by LDS-DMA during the last level.
  // Its contract: two buffers, full slabs of whole waves, rows in 64-vector chunks, no validation
  // or streaming history.  VW_FWD_PERSIST=0 disables it.
  const Tuning& tu = c->tune;
  const bool persist_on = tu.fwd_persist;
  // the unvalidated callers' NaN spread through the zero taps (single level and J = 1 have none); a
  // streaming block that updates its history needs the snapshot of the histories it read (stream_run)
  const bool ref_nf = (flags & VW_FLAG_REF_NONFINITE) && !validate && !single_level && J >= 2 &&
                      !(flags & VW_FLAG_FFT_SWITCH) && (!hist || !hist_update || hist_first || hist_snap);
  bool nf_probed = false;
  const bool io_aligned = (ldx % V == 0) && (N % V == 0) && aligned16(x) && aligned16(details) && aligned16(approx);
  auto persist_ok = [&](int th, int nvv, bool ft) {
    return persist_on && io_aligned && ft && nvv == 4 && !validate && !hist && (int64_t)th * nvv == nvec &&
           th % 64 == 0 && nvec % 64 == 0 && has_unrolled_taps(L) && J >= 1;
  };
  const int64_t region = round_up(hlpad + nvec * V + V, V);
  bool dbl = tu.fwd_buf ? tu.fwd_buf == 2 : true;
  bool fused = false, fit = false;
  // NV = 2 (1024-thread workgroups) only where the unrolled kernel will run (it has no runtime-L form)
  const int fwd_nv2 = (tu.fwd_nv == 2 && io_aligned && L <= 8 && L <= tu.unroll_max && has_unrolled_taps(L) &&
                       !(tu.blk > 0 && L >= tu.blk)) ? 2 : 0;
  if (J <= kMaxLevels && !tu.force_tiled) {
    if (dbl) dbl = fused_plan(tu, N, V, sizeof(T), 2 * region, &threads, &nv, &lds, &fit, fwd_nv2);
    if (dbl && !tu.fwd_buf && !fma && !persist_ok(threads, nv, fit)) dbl = false;  // EXACT without persistence
    fused = dbl || fused_plan(tu, N, V, sizeof(T), region, &threads, &nv, &lds, &fit, fwd_nv2);
  }
  if (fused && nv == 2 && !(fit && (int64_t)threads * 2 == nvec)) return fail(VW_ERR_STATE, "NV=2 plan without full slabs");
  if (fused) {
    for (int j = 0; j < J; ++j) set_halo_images(lv[j], N, npow2, V, threads, nv);
    FwdArgs<T> a;
    memset(&a, 0, sizeof(a));
    a.x = x; a.ldx = ldx; a.details = details; a.approx = approx; a.B = B; a.N = (int)N; a.J = J;
    a.npow2 = npow2; a.hlpad = hlpad; a.region1 = dbl ? (int)region : 0;
    a.vec_io = (ldx % V == 0) && (N % V == 0) && aligned16(x) && aligned16(details) && aligned16(approx);
    a.unrolled = a.vec_io && fit && L <= tu.unroll_max;
    a.validate = validate; a.bad = c->bad;
    a.rev = tu.fwd_rev;
    // non-temporal LDS-DMA of the rows: faster at <= 2 signals per CU (512 rows: forward 0.0268 -> 0.0245 ms),
    // slower on full batches (4096 rows: 0.218-0.225 -> 0.234-0.243 ms; profiles/r04/ab_rotate_default_*.log,
    // ab_overlap_direct_512.log)
    a.dma_nt = tu.dma_nt >= 0 ? tu.dma_nt : (B <= 2LL * c->cus ? 1 : 0);
    for (int j = 0; j < J; ++j) a.hist[j] = hist ? hist[j] : nullptr;
    a.hist_update = hist_update ? 1 : 0;
    a.taps = L;
    copy_taps(a.lo, lo, L);
    copy_taps(a.hi, hi, L);
    for (int j = 0; j < J; ++j) a.lv[j] = lv[j];
    if (validate) VW_HIP(hipMemsetAsync(c->bad, 0xFF, sizeof(unsigned long long), c->stream));
    const bool persist = dbl && a.unrolled && persist_ok(threads, nv, fit);
    // register-blocked PERIODIC forward for long filters (vw_device.h k_forward_blk): padded layouts
    int blk_lds = 0;
    // (NV = 8, 1024-thread workgroups: with its taps from the kernel arguments (round 4, 99 VGPRs, no
    // spills) the blocked forward beats the fused one at sym8 N = 16384: 5.27-5.29 -> 4.76 ms,
    // profiles/r04/ab_blk_fwd8_ktaps_sym8.log; VW_BLK_FWD8=0 restores the fused kernel)
    if (tu.blk > 0 && L >= tu.blk && a.unrolled && !validate && !hist && (int64_t)threads * nv == nvec &&
        (nv == 4 || (nv == 8 && tu.blk_fwd8))) {
      bool okb = true;
      int hlv = 0;
      for (int j = 0; j < J; ++j) {
        if (lv[j].mode != kHaloPeriodic) okb = false;
        hlv = std::max<int>(hlv, (int)(((int64_t)(L - 1) * lv[j].s + V - 1) / V));
      }
      // the kernel reads at wave-uniform (NV = 8) or compile-time (NV = 4) offsets when the halo is whole
      // pad groups (16 vectors)
      if (round_up(hlv, 16) <= nvec) hlv = (int)round_up(hlv, 16);
      const int mJ = std::max(1, lv[J - 1].s / V);
      if (nvec % ((int64_t)nv * mJ) != 0 || hlv > nvec) okb = false;
      auto buf_of = [&](int tight) {
        int64_t bf = 0;
        for (int j = 0; j < J; ++j) {
          int sh, pd;
          blk_layout_host(lv[j].s / V, nv, &sh, &pd, tight);
          const int64_t u = hlv + nvec - 1;
          bf = std::max(bf, u + (u >> sh) * pd + 1);
        }
        return bf;
      };
      int64_t buf = buf_of(0);
      if (buf * 16 + 2 * L * (int64_t)sizeof(T) > kLdsBytes && nv >= 8) {
        a.blk_tight = 1;
        buf = buf_of(1);
      }
      if (okb && buf * 16 <= kLdsBytes) {
        const bool two = 2 * buf * 16 <= 80 * 1024;  // two buffers only where two workgroups still fit a CU
        a.region1 = two ? (int)(buf * V) : 0;
        a.hlpad = hlv * V;
        a.tap_lds = (int)(buf * V * (two ? 2 : 1));
        blk_lds = (int)(buf * 16 * (two ? 2 : 1)) + 2 * L * (int)sizeof(T);
        if (blk_lds > kLdsBytes) blk_lds = 0;
      }
    }
    // fp32 FMA, PERIODIC, long filters: the matrix-core forward (vw_mfma.hip, VW_MFMA bit 0)
    int mfma_lds = 0;
    if constexpr (std::is_same<T, float>::value) {
      bool ok = (tu.mfma & 1) && fma && !single_level && a.vec_io && !validate && !hist && mfma_supported(L, N);
      for (int j = 0; ok && j < J; ++j) ok = lv[j].mode == kHaloPeriodic;
      const int H = ok ? mfma_halo(L, J) : 0;
      const int region = ok ? mfma_region((int)N + H) : 0;  // padded LDS layout (vw_mfma.hip ph)
      const int scratch = 8 * 256 + 4;  // the forward's per-wave transpose scratch (<= 8 waves), aligned
      if (ok && H <= N && (int64_t)(region + 2 * L + scratch) * 4 <= kLdsBytes) {
        a.hlpad = H;
        a.tap_lds = region;
        mfma_lds = (int)((region + 2 * L + scratch) * 4);
      }
    }
    // VW_FLAG_REF_NONFINITE: the persistent and the register-blocked forward probe their a_J (no scan pass
    // afterwards)
    if (ref_nf && !mfma_lds && (blk_lds || persist)) {
      VW_TRY(ensure_nf(c, B));
      a.nf_flag = c->nf;
      nf_probed = true;
    }
    {
      LaunchTimer lt(c, "forward");
      hipError_t e = mfma_lds ? mfma_forward(a, mfma_lds, c->stream)
                   : blk_lds ? launch_forward_blk<T>(a, threads, blk_lds, fma, nv, c->stream)
                   : persist ? launch_forward_persist<T>(a, threads, lds, fma, nv, c->stream)
                             : launch_forward_fused<T>(a, threads, lds, fma, nv, c->stream);
      if (e != hipSuccess) return fail(VW_ERR_DEVICE, "forward launch failed: %s", hipGetErrorString(e));
    }
  } else {
    // Per-level path for long signals: ping-pong the running approximation through the workspace.
    // Deep levels (s >= kSweepMinS) run as column sweeps, shallow ones as LDS tiles with a halo.
    for (int j = 1; hist && j <= J; ++j)
      if (lv[j - 1].hist_len > N) return fail(VW_ERR_UNSUPPORTED, "streaming block shorter than level %d history", j);
    const int tile_max = tu.fwd_tile ? tu.fwd_tile / V * V : 256 * kNV * V;
    const size_t plane = (size_t)B * (size_t)N;
    const vw_status st = ensure_ws(c, 2 * plane * sizeof(T) + 256);
    if (st != VW_OK) return st;
    T* tmp[2] = {reinterpret_cast<T*>(c->ws), reinterpret_cast<T*>(c->ws) + plane};
    if (validate) VW_HIP(hipMemsetAsync(c->bad, 0xFF, sizeof(unsigned long long), c->stream));
    const T* src = x;
    int64_t lda = ldx;
    const int mtile = multi_tile<T>(tu);
    const std::vector<int> groups = level_groups(tu, lv, J, L, V, mtile, !validate && !hist);
    for (int j = 1; j <= J; ++j) {
      T* const nxt = (src == tmp[0]) ? tmp[1] : tmp[0];  // never the level's own input
      // streaming deep group from level j: the longest run j..je within the LDS budget
      if (groups[j - 1] == 1 && !validate && !hist && (lda % V) == 0 && aligned16(src) && aligned16(details) &&
          aligned16(approx) && deep_plan<T>(tu, lv, j, j, L, N, false, nullptr)) {
        int je = j;
        while (je < J && groups[je] == 1 && deep_plan<T>(tu, lv, j, je + 1, L, N, false, nullptr)) ++je;
        DeepArgs<T> d;
        memset(&d, 0, sizeof(d));
        const int lds = deep_plan<T>(tu, lv, j, je, L, N, false, &d);
        deep_segments<T>(tu, c->cus, B, &d);
        d.src = src; d.lda = lda; d.B = B; d.taps = L;
        d.out = (je == J) ? approx : nxt;
        if (ref_nf && je == J) {  // the deep launch writes a_J: it probes it (VW_FLAG_REF_NONFINITE)
          VW_TRY(ensure_nf(c, B));
          d.nf_flag = c->nf;
          nf_probed = true;
        }
        for (int k = 0; k < d.g; ++k) d.out_d[k] = details + (size_t)(j - 1 + k) * plane;
        copy_taps(d.lo, lo, L);
        copy_taps(d.hi, hi, L);
        {
          LaunchTimer lt(c, "forward_level");
          hipError_t e = launch_deep<T>(d, lds, fma, false, c->stream);
          if (e != hipSuccess) return fail(VW_ERR_DEVICE, "forward deep launch failed: %s", hipGetErrorString(e));
        }
        src = d.out;
        lda = N;
        j = je;
        continue;
      }
      if (groups[j - 1] >= 2) {
        const int g = groups[j - 1], je = j + g - 1;
        MultiArgs<T> m;
        memset(&m, 0, sizeof(m));
        m.src_a = src; m.lda = lda;
        m.out_a = (je == J) ? approx : nxt;
        bool al = aligned16(src) && aligned16(m.out_a);
        for (int k = 0; k < g; ++k) {
          m.out_d[k] = details + (size_t)(j - 1 + k) * plane;
          al = al && aligned16(m.out_d[k]);
        }
        m.ext[g] = 0;
        for (int k = g - 1; k >= 0; --k)
          m.ext[k] = m.ext[k + 1] + (int)round_up((int64_t)(L - 1) * lv[j - 1 + k].s, V);
        m.B = B; m.N = (int)N; m.tile = mtile; m.nlev = g; m.s0 = lv[j - 1].s;
        m.region = (int)round_up(m.ext[0] + mtile + V, V);
        m.vec_io = (N % V == 0) && (lda % V == 0) && al;
        m.taps = L;
        copy_taps(m.lo, lo, L);
        copy_taps(m.hi, hi, L);
        {
          LaunchTimer lt(c, "forward_level");
          hipError_t e = launch_forward_multi<T>(m, (int)(2 * m.region * sizeof(T)), fma, c->stream);
          if (e != hipSuccess) return fail(VW_ERR_DEVICE, "forward multi-level launch failed: %s", hipGetErrorString(e));
        }
        src = m.out_a;
        lda = N;
        j = je;
        continue;
      }
      LevelArgs<T> a;
      memset(&a, 0, sizeof(a));
      a.lv = lv[j - 1];
      const int hp = (int)round_up(a.lv.hl, V);
      // deep levels have long halos: shrink the tile so tile + halo fits LDS
      const int64_t fit = ((int64_t)kLdsBytes / (int64_t)sizeof(T) - hp - 2 * V) / V * V;
      const int tile = (int)std::min<int64_t>(tile_max, fit);
      if (tile < 64 * V) return fail(VW_ERR_UNSUPPORTED, "level %d halo (%d samples) exceeds LDS", j, a.lv.hl);
      const int64_t elems = hp + tile + V;
      a.src_a = src; a.lda = lda;
      a.out_a = (j == J) ? approx : nxt;
      a.out_d = details + (size_t)(j - 1) * plane;
      a.hist = hist ? hist[j - 1] : nullptr;
      a.B = B; a.N = (int)N; a.tile = tile; a.hlpad = hp;
      a.vec_io = (N % V == 0) && (lda % V == 0) && aligned16(src) && aligned16(a.out_a) && aligned16(a.out_d);
      a.validate = validate; a.bad = c->bad; a.npow2 = npow2; a.taps = L;
      copy_taps(a.lo, lo, L);
      copy_taps(a.hi, hi, L);
      const bool sweep = a.lv.s >= kSweepMinS && has_unrolled_taps(L) && !tu.no_sweep;
      {
        LaunchTimer lt(c, "forward_level");
        hipError_t e;
        if (sweep) {
          a.tile = tu.sweep_qc;
          e = launch_forward_sweep<T>(a, fma, c->stream);
        } else {
          e = launch_forward_level<T>(a, (int)(elems * sizeof(T)), fma, c->stream);
        }
        if (e != hipSuccess) return fail(VW_ERR_DEVICE, "forward level launch failed: %s", hipGetErrorString(e));
      }
      // streaming: this level's new left history = the last L_j - 1 samples of its input
      // (BatchStreamingMODWT.updateHistoryFromSoA :337-352); read by this level's kernel first
      if (hist && hist_update) {
        hipError_t e = launch_history_update<T>(src, lda, hist[j - 1], hist[j - 1], B, (int)N, a.lv.hist_len,
                                                c->stream);
        if (e != hipSuccess) return fail(VW_ERR_DEVICE, "history update failed: %s", hipGetErrorString(e));
      }
      src = a.out_a;
      lda = N;
    }
  }
  if (ref_nf) {
    // a_J alone: every non-finite level input (x, a_1 .. a_{J-1}, a history) reaches it (vw_ref.hip)
    std::vector<ScanPlane<T>> planes{{approx, N, 0}};
    RefArgs<T> r;
    memset(&r, 0, sizeof(r));
    r.x = x; r.ldx = ldx; r.details = details; r.approx = approx;
    r.B = B; r.N = (int)N; r.J = J; r.L = L; r.mode = ref_mode(boundary);
    if (hist) {  // BatchStreamingMODWT block / flush: the histories the block read, and the ones it leaves
      r.hist_mode = 1;
      r.hist_first = hist_first ? 1 : 0;
      for (int j = 0; j < J; ++j) {
        const int hl = lv[j].hist_len;
        r.hist_len[j] = hl;
        r.hist_old[j] = hist_first ? nullptr : (hist_update ? hist_snap[j] : hist[j]);
        r.hist_new[j] = hist_update ? hist[j] : nullptr;
      }
    }
    copy_taps(r.lo, lo, L);
    copy_taps(r.hi, hi, L);
    VW_TRY(ref_nonfinite<T>(c, planes, r, false, nf_probed));
  }
  if (validate) {
    unsigned long long bad = 0;
    vw_status st = read_bad(c, &bad);
    if (st != VW_OK) return st;
    st = report_bad(bad, N);
    if (st != VW_OK) return st;
  }
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return VW_OK;
}

// ------------------------------------------------------------------------------------------------
// Inverse
template <typename T>
static vw_status inverse_impl(vw_ctx* c, const T* details, const T* approx, int64_t B, int64_t N, const double* lo,
                              const double* hi, int L, int wid, int boundary, int J, unsigned detail_mask,
                              int approx_zero, unsigned flags, T* y, bool single_level, const T* thr, int soft,
                              int64_t thr_ld = 0) {
  constexpr int V = vec_width<T>();
  VW_TRY(capture_guard(c, flags));
  const bool fma = flags & VW_FLAG_FMA;
  const int64_t nvec = (N + V - 1) / V;
  const int tmax = (int)(nvec * V - 1);
  const bool pair = single_level || boundary == VW_ZERO_PADDING;
  // the unvalidated callers' NaN spread through the zero taps (single level and J = 1 have none)
  const bool ref_nf = (flags & VW_FLAG_REF_NONFINITE) && !single_level && J >= 2;
  bool nf_probed = false;

  std::vector<LevelDesc> lv(J);
  int max_hl = 0, max_hr = 0;
  for (int j = 1; j <= J; ++j) {
    LevelDesc& d = lv[j - 1];
    memset(&d, 0, sizeof(d));
    d.s = 1 << (j - 1);
    d.use_d = (detail_mask >> (j - 1)) & 1u;
    d.mode = boundary == VW_PERIODIC ? kHaloPeriodic : boundary == VW_ZERO_PADDING ? kHaloZero : kHaloSymmetric;
    if (boundary == VW_SYMMETRIC && !single_level) {
      int ap, dh, dp, dg;
      sym_decide(wid, L, j, &ap, &dh, &dp, &dg);
      const int tauH = compute_tau(L, j) + dh;
      const int tauG = compute_tau(L, j) + dg;
      d.dir_a = ap ? 1 : -1; d.off_a = ap ? -tauH : tauH;
      d.dir_d = dp ? 1 : -1; d.off_d = dp ? -tauG : tauG;
    } else if (boundary == VW_SYMMETRIC) {
      const int dir = (flags & VW_FLAG_BATCH_SYM_INVERSE) ? 1 : -1;  // inverseBatchOptimized (t+l) vs inverse (t-l)
      d.dir_a = d.dir_d = dir; d.off_a = d.off_d = 0;
    } else {
      d.dir_a = d.dir_d = 1; d.off_a = d.off_d = 0;
    }
    int hl = 0, hr = 0;
    branch_extent((int)N, tmax, L, d.s, d.dir_a, d.off_a, &hl, &hr);
    branch_extent((int)N, tmax, L, d.s, d.dir_d, d.off_d, &hl, &hr);
    d.hl = hl; d.hr = hr;
    max_hl = std::max(max_hl, hl);
    max_hr = std::max(max_hr, hr);
  }
  const int hlpad = (int)round_up(max_hl, V);
  const int64_t region = round_up(hlpad + nvec * V + max_hr + V, V);
  int threads = 0, lds = 0, nv = 4;
  // Pairwise sums need a_j and d_j together (two regions).  Sequential sums time-share one region
  // (k_inverse_seq, four barriers per level) -- measured faster on MI355X than two buffers
  // (k_inverse_db, two barriers per level) because twice the workgroups fit per CU; VW_INV_BUF=2
  // selects the latter.
  const Tuning& tu = c->tune;
  // Two LDS buffers (two barriers per level, two workgroups per CU) vs one (four barriers, three per
  // CU): with at most 2 signals per CU the occupancy of the one-buffer kernel is not reached and the
  // shorter per-level chain wins (measured on MI355X, db4 x 4096, inverse ms one / two buffers:
  // B = 512 0.0335 / 0.0324, B = 768 0.0462 / 0.0504, B = 1024 0.0594 / 0.0606 --
  // profiles/r02/ab_small_batch.log, ab_inv_buf_1024_768.log); VW_INV_BUF=1|2 overrides.
  // Long PERIODIC filters (L >= VW_BLK) keep the register-blocked single-buffer kernel (k_inverse_blk
  // needs !db) at small batches too: its NV+L-1 LDS reads per branch outweigh the shorter barrier chain.
  const bool blk_pref = tu.blk > 0 && L >= tu.blk && boundary == VW_PERIODIC;
  bool db = !pair && (tu.inv_buf ? tu.inv_buf == 2 : (B <= 2LL * c->cus && !blk_pref));
  bool fused = false, fit = false;
  const bool inv_io = (N % V == 0) && aligned16(details) && aligned16(approx) && aligned16(y);
  const int inv_nv2 = (tu.inv_nv == 2 && inv_io && L <= 8 && L <= tu.unroll_max && has_unrolled_taps(L)) ? 2 : 0;
  if (!tu.force_tiled) {
    if (pair || db) fused = fused_plan(tu, N, V, sizeof(T), 2 * region, &threads, &nv, &lds, &fit, inv_nv2);
    if (!fused && !pair) {
      db = false;
      fused = fused_plan(tu, N, V, sizeof(T), region, &threads, &nv, &lds, &fit, inv_nv2);
    }
  }
  if (fused) {
    for (int j = 0; j < J; ++j) set_halo_images(lv[j], N, 0, V, threads, nv);
    InvArgs<T> a;
    memset(&a, 0, sizeof(a));
    a.details = details; a.approx = approx; a.y = y; a.B = B; a.N = (int)N; a.J = J;
    a.db = db ? 1 : 0;
    a.hlpad_a = hlpad; a.hlpad_d = hlpad; a.region_d = (int)region;
    a.vec_io = (N % V == 0) && aligned16(details) && aligned16(approx) && aligned16(y);
    a.unrolled = a.vec_io && fit && L <= tu.unroll_max;
    a.pair = pair; a.approx_zero = approx_zero; a.thr = thr; a.thr_ld = thr_ld; a.soft = soft; a.taps = L;
    a.rev = tu.inv_rev;
    // register-blocked PERIODIC inverse for long filters (vw_device.h k_inverse_blk)
    if (tu.blk > 0 && L >= tu.blk && nv != 2 && !pair && !db && boundary == VW_PERIODIC && a.unrolled &&
        (int64_t)threads * nv == nvec) {
      bool okb = true;
      int64_t buf = 0;
      const int mJ = std::max(1, lv[J - 1].s / V);
      if (nvec % ((int64_t)nv * mJ) != 0) okb = false;
      int64_t buf_t = 0;
      for (int j = 0; j < J && okb; ++j) {
        if (lv[j].dir_a != 1 || lv[j].dir_d != 1 || lv[j].off_a != 0 || lv[j].off_d != 0) okb = false;
        const int64_t hrv = ((int64_t)(L - 1) * lv[j].s + V - 1) / V;
        if (hrv > nvec) okb = false;
        int sh, pd;
        const int64_t u = nvec + hrv - 1;
        blk_layout_host(lv[j].s / V, nv, &sh, &pd);
        buf = std::max(buf, u + (u >> sh) * pd + 1);
        blk_layout_host(lv[j].s / V, nv, &sh, &pd, 1);
        buf_t = std::max(buf_t, u + (u >> sh) * pd + 1);
      }
      const int64_t taps_b = 2 * L * (int64_t)sizeof(T);
      if (okb && buf * 16 + taps_b > kLdsBytes && nv >= 8 && buf_t * 16 + taps_b <= kLdsBytes) {
        a.blk_tight = 1;  // sparse padding so the level fits (sym8 at N = 16384)
        buf = buf_t;
      }
      if (okb && buf * 16 + taps_b <= kLdsBytes) {
        a.blk = 1;
        a.tap_lds = (int)(buf * V);
        lds = (int)(buf * 16) + 2 * L * (int)sizeof(T);
      }
    }
    copy_taps(a.lo, lo, L);
    copy_taps(a.hi, hi, L);
    for (int j = 0; j < J; ++j) a.lv[j] = lv[j];
    // (A persistent form that loads the next signal's approximation during level 1 was measured
    // slower on MI355X: 3 resident workgroups per CU do not divide the batch evenly, and the dynamic
    // dispatch of one-signal workgroups balances better.)
    // fp32 FMA, PERIODIC sequential sums, long filters: the matrix-core inverse (vw_mfma.hip, VW_MFMA bit 1)
    int mfma_lds = 0;
    if constexpr (std::is_same<T, float>::value) {
      bool ok = (tu.mfma & 2) && fma && !pair && boundary == VW_PERIODIC && a.vec_io && mfma_supported(L, N);
      for (int j = 0; ok && j < J; ++j) ok = lv[j].dir_a == 1 && lv[j].dir_d == 1 && lv[j].off_a == 0 && lv[j].off_d == 0;
      const int H = ok ? mfma_halo(L, J) : 0;
      const int region = ok ? mfma_region((int)N + H) : 0;
      if (ok && H <= N && (int64_t)(region + 2 * L) * 4 <= kLdsBytes) {
        a.hlpad_a = H;
        a.tap_lds = region;
        mfma_lds = (int)((region + 2 * L) * 4);
      }
    }
    // VW_FLAG_REF_NONFINITE: the one-buffer sequential kernels (k_inverse_seq / k_inverse_blk, vw_inv.hip's
    // choice) probe their output themselves (no scan pass afterwards)
    if (ref_nf && !mfma_lds && !a.pair && !a.db) {
      VW_TRY(ensure_nf(c, B));
      a.nf_flag = c->nf;
      nf_probed = true;
    }
    LaunchTimer lt(c, "inverse");
    hipError_t e = mfma_lds ? mfma_inverse(a, mfma_lds, c->stream) : launch_inverse_fused<T>(a, threads, lds, fma, nv, c->stream);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "inverse launch failed: %s", hipGetErrorString(e));
  } else {
    // 1024-sample tiles: two LDS regions of ~9 KiB keep many workgroups per CU (measured best on
    // MI355X for db8 2^20-sample blocks; VW_INV_TILE overrides)
    const int tile_max = tu.inv_tile ? tu.inv_tile / V * V : 1024;
    const size_t plane = (size_t)B * (size_t)N;
    const vw_status st = ensure_ws(c, 2 * plane * sizeof(T) + 256);
    if (st != VW_OK) return st;
    T* tmp[2] = {reinterpret_cast<T*>(c->ws), reinterpret_cast<T*>(c->ws) + plane};
    const T* cur = approx_zero ? nullptr : approx;
    // multi-level groups (PERIODIC sequential sums): start level of the group whose top is j
    const int mtile = tu.multi_inv_tile >= 64 * V ? tu.multi_inv_tile / V * V : multi_tile<T>(tu);
    const std::vector<int> groups = level_groups(tu, lv, J, L, V, mtile, !pair && boundary == VW_PERIODIC);
    std::vector<int> start_of(J + 1, 0);
    for (int j = 1; j <= J; ++j) {
      if (groups[j - 1] < 2) continue;
      int64_t ext = 0;  // k_inverse_multi holds (tile + reach) / V vectors in kMultiInvNI per thread
      for (int k = 0; k < groups[j - 1]; ++k) ext += round_up((int64_t)(L - 1) * lv[j - 1 + k].s, V);
      if ((mtile + ext) / V <= (int64_t)kMultiInvNI * 256) start_of[j + groups[j - 1] - 1] = j;
    }
    std::vector<char> in_group(J + 1, 0);  // levels inside a multi-level tile group
    for (int e = 1; e <= J; ++e)
      for (int k = start_of[e]; start_of[e] > 0 && k <= e; ++k) in_group[k] = 1;
    for (int j = J; j >= 1; --j) {
      T* const nxt = (cur == tmp[0]) ? tmp[1] : tmp[0];  // never the level's own input
      // streaming deep group with top level j: the lowest jl whose group jl..j fits the LDS budget
      if (!pair && boundary == VW_PERIODIC && !in_group[j] && aligned16(cur) && aligned16(details) &&
          aligned16(y) && deep_plan<T>(tu, lv, j, j, L, N, true, nullptr)) {
        int jl = j;
        while (jl > 1 && !in_group[jl - 1] && deep_plan<T>(tu, lv, jl - 1, j, L, N, true, nullptr)) --jl;
        DeepArgs<T> d;
        memset(&d, 0, sizeof(d));
        const int lds = deep_plan<T>(tu, lv, jl, j, L, N, true, &d);
        deep_segments<T>(tu, c->cus, B, &d);
        d.src = cur; d.lda = N; d.B = B; d.taps = L; d.soft = soft;
        d.out = (jl == 1) ? y : nxt;
        for (int k = 0; k < d.g; ++k) {
          const LevelDesc& ld = lv[jl - 1 + k];
          d.src_d[k] = ld.use_d ? details + (size_t)(jl - 1 + k) * plane : nullptr;
          d.thr[k] = thr ? thr + (size_t)(jl - 1 + k) * (size_t)thr_ld : nullptr;
        }
        copy_taps(d.lo, lo, L);
        copy_taps(d.hi, hi, L);
        {
          LaunchTimer lt(c, "inverse_level");
          hipError_t e = launch_deep<T>(d, lds, fma, true, c->stream);
          if (e != hipSuccess) return fail(VW_ERR_DEVICE, "inverse deep launch failed: %s", hipGetErrorString(e));
        }
        cur = d.out;
        j = jl;
        continue;
      }
      if (start_of[j] > 0) {
        const int j0 = start_of[j], g = j - j0 + 1;
        MultiArgs<T> m;
        memset(&m, 0, sizeof(m));
        m.src_a = cur;
        m.out_a = (j0 == 1) ? y : nxt;
        if (ref_nf && j0 == 1) {  // the group writes y: it probes it (VW_FLAG_REF_NONFINITE)
          VW_TRY(ensure_nf(c, B));
          m.nf_flag = c->nf;
          nf_probed = true;
        }
        bool al = aligned16(cur) && aligned16(m.out_a);
        for (int k = 0; k < g; ++k) {
          const LevelDesc& d = lv[j0 - 1 + k];
          m.src_d[k] = d.use_d ? details + (size_t)(j0 - 1 + k) * plane : nullptr;
          m.thr[k] = thr ? thr + (size_t)(j0 - 1 + k) * (size_t)thr_ld : nullptr;
          al = al && aligned16(m.src_d[k]);
          m.ext[k] = (k > 0 ? m.ext[k - 1] : 0) + (int)round_up((int64_t)(L - 1) * d.s, V);
        }
        m.B = B; m.N = (int)N; m.tile = mtile; m.nlev = g; m.s0 = lv[j0 - 1].s;
        m.region = (int)round_up(mtile + m.ext[g - 1] + V, V);
        m.vec_io = (N % V == 0) && al;
        m.soft = soft; m.taps = L;
        m.rblk = tu.multi_rblk;
        // register prefetch of d_{j-1} while level j computes: whole vectors, every tile of the group
        m.pf = tu.multi_pf && m.vec_io && (int64_t)(mtile + m.ext[g - 1]) / V <= (int64_t)kMultiPF * 256;
        // padded layout at the register-blocked levels (vw_device.h k_inverse_multi): needs the register
        // paths (prefetch, blocked taps); the regions grow by one vector in eight
        m.pad = tu.multi_pad && m.pf && m.rblk && has_unrolled_taps(L);
        if (m.pad) {
          const int nvmax = (mtile + m.ext[g - 1]) / V + 1;
          m.region = (nvmax + nvmax / 8 + 1) * V;
        }
        // slack past D for the compile-time-stride reads (vw_device.h k_inverse_multi): 15*M <= 120 vectors
        m.slack = 160;
        m.ni = kMultiInvNI;
        // four output vectors per thread (fp64, padded layouts): at NI = 8 a 2048-sample tile gives the
        // register-blocked levels 129-144 threads of work, i.e. 2.0-2.3 of the workgroup's 4 waves (one SIMD idle,
        // one mostly idle); at NI = 4 on the largest tile whose levels fit 256 threads (1792 for db8) all four
        // waves work.  The group itself stays as planned above.
        if (tu.multi_ni == 4 && sizeof(T) == 8 && m.pad) {
          auto fits = [&](int64_t t) {
            if ((t + m.ext[g - 1]) / V > (int64_t)kMultiPF * 256) return false;
            for (int k = 0; k < g; ++k) {
              const int64_t s = lv[j0 - 1 + k].s, M = s % V == 0 ? s / V : 0;
              const int64_t nv = (t + (k > 0 ? m.ext[k - 1] : 0)) / V;
              const bool blk = M == 1 || M == 2 || M == 4 || M == 8;
              if (blk ? (nv + 4 * M - 1) / (4 * M) * M > 256 : nv > 4 * 256) return false;
            }
            return true;
          };
          int64_t t = mtile;
          while (t >= 512 && !fits(t)) t -= 64 * V;
          if (t >= 512) {
            m.ni = 4;
            m.tile = (int)t;
            const int nvmax = (int)((t + m.ext[g - 1]) / V) + 1;
            m.region = (nvmax + nvmax / 4 + 1) * V;  // layouts 2 / 3 add at most u/4
          }
        }
        copy_taps(m.lo, lo, L);
        copy_taps(m.hi, hi, L);
        LaunchTimer lt(c, "inverse_level");
        hipError_t e = launch_inverse_multi<T>(m, (int)((2 * m.region + m.slack * V) * sizeof(T)), fma, c->stream);
        if (e != hipSuccess) return fail(VW_ERR_DEVICE, "inverse multi-level launch failed: %s", hipGetErrorString(e));
        cur = m.out_a;
        j = j0;
        continue;
      }
      // two or three column-sweep levels per launch (k_inverse_sweep2 / 3): the intermediate
      // approximations stay in LDS rings
      if (tu.sweep2 && !tu.deep_inv && !tu.no_sweep && !pair && j >= 2 && has_unrolled_taps(L)) {
        int G = 0, ka = 0, R = 0;
        for (int levels = std::min(tu.sweep2 >= 3 ? 3 : 2, j); levels >= 2 && !G; --levels)
          if (sweepg_plan<T>(tu, lv, j, levels, L, N, in_group, start_of, &ka, &R)) G = levels;
        if (G) {
          const LevelDesc& lj = lv[j - 1];
          LevelArgs<T> a;
          memset(&a, 0, sizeof(a));
          a.lv = lj;
          a.src_a = cur;
          a.src_d = lj.use_d ? details + (size_t)(j - 1) * plane : nullptr;
          a.use_d = lj.use_d;
          a.thr = thr ? thr + (size_t)(j - 1) * (size_t)thr_ld : nullptr;
          a.src_d2 = lv[j - 2].use_d ? details + (size_t)(j - 2) * plane : nullptr;
          a.use_d2 = lv[j - 2].use_d;
          a.thr2 = thr ? thr + (size_t)(j - 2) * (size_t)thr_ld : nullptr;
          if (G == 3) {
            a.src_d3 = lv[j - 3].use_d ? details + (size_t)(j - 3) * plane : nullptr;
            a.use_d3 = lv[j - 3].use_d;
            a.thr3 = thr ? thr + (size_t)(j - 3) * (size_t)thr_ld : nullptr;
          }
          a.soft = soft;
          a.out_a = (j == G) ? y : nxt;
          a.B = B; a.N = (int)N; a.taps = L;
          const int kb = (G == 2 ? 2 : 4) * ka;
          a.tile = (int)round_up(tu.sweep2_uc, kb);
          copy_taps(a.lo, lo, L);
          copy_taps(a.hi, hi, L);
          LaunchTimer lt(c, "inverse_level");
          hipError_t e = launch_inverse_sweepg<T>(a, G == 2 ? 2 : 4, ka, R, fma, c->stream);
          if (e != hipSuccess) return fail(VW_ERR_DEVICE, "inverse level-group launch failed: %s", hipGetErrorString(e));
          cur = a.out_a;
          j -= G - 1;  // levels j-1 (, j-2) done too
          continue;
        }
      }
      LevelArgs<T> a;
      memset(&a, 0, sizeof(a));
      a.lv = lv[j - 1];
      const int hp = (int)round_up(a.lv.hl, V);
      const int64_t fit = ((int64_t)kLdsBytes / (int64_t)sizeof(T) / 2 - hp - a.lv.hr - 2 * V) / V * V;
      const int tile = (int)std::min<int64_t>(tile_max, fit);
      if (tile < 64 * V) return fail(VW_ERR_UNSUPPORTED, "level %d halo exceeds LDS", j);
      const int64_t reg = round_up(hp + tile + a.lv.hr + V, V);
      a.src_a = cur;
      a.src_d = a.lv.use_d ? details + (size_t)(j - 1) * plane : nullptr;
      a.use_d = a.lv.use_d;
      a.out_a = (j == 1) ? y : nxt;
      a.B = B; a.N = (int)N; a.tile = tile; a.hlpad = hp; a.hlpad_d = hp; a.region_d = (int)reg;
      a.pair = pair; a.thr = thr ? thr + (size_t)(j - 1) * (size_t)thr_ld : nullptr; a.soft = soft; a.taps = L;
      a.vec_io = (N % V == 0) && aligned16(a.out_a) && aligned16(a.src_a) && aligned16(a.src_d);
      copy_taps(a.lo, lo, L);
      copy_taps(a.hi, hi, L);
      LaunchTimer lt(c, "inverse_level");
      hipError_t e;
      if (a.lv.s >= kSweepMinS && has_unrolled_taps(L) && !tu.no_sweep) {
        a.tile = tu.sweep_qc;
        e = launch_inverse_sweep<T>(a, fma, c->stream);
      } else {
        e = launch_inverse_level<T>(a, (int)(2 * reg * sizeof(T)), fma, c->stream);
      }
      if (e != hipSuccess) return fail(VW_ERR_DEVICE, "inverse level launch failed: %s", hipGetErrorString(e));
      cur = a.out_a;
    }
  }
  if (ref_nf) {
    // y alone: every non-finite level input (a_J, a kept d_j, an intermediate approximation) reaches it
    std::vector<ScanPlane<T>> planes{{y, N, 0}};
    RefArgs<T> r;
    memset(&r, 0, sizeof(r));
    r.x = approx_zero ? nullptr : approx; r.det_in = details; r.y = y;
    r.thr = thr; r.thr_ld = thr_ld; r.soft = soft;
    r.B = B; r.N = (int)N; r.J = J; r.L = L; r.mode = ref_mode(boundary);
    copy_taps(r.lo, lo, L);
    copy_taps(r.hi, hi, L);
    for (int j = 0; j < J; ++j) r.lv[j] = lv[j];
    VW_TRY(ref_nonfinite<T>(c, planes, r, true, nf_probed));
  }
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return VW_OK;
}

// ------------------------------------------------------------------------------------------------
// Host-memory staging (the JNI / FFM path): copy in, run on device, copy out, synchronize.  Device
// buffers are carved from the context's staging pool (blocks kept across calls, never hipMalloc /
// hipFree per call: a JNI caller's per-batch loop pays only the copies and the kernels).  A call
// carves from offset 0 of the pool; its destructor synchronizes the stream, so the next call may
// reuse the same bytes.  Calls on one context are serialized by its mutex.
struct Staging {
  vw_ctx* c;
  size_t used_block = 0, used_off = 0;
  explicit Staging(vw_ctx* ctx) : c(ctx) {}
  // After the call's copies and kernels: keep only the largest block (the next call of the same
  // shape allocates at most one block >= its whole need, and frees this one here), so the pool holds
  // one block of about the largest call's size instead of every block it ever grew through.
  ~Staging() {
    hipStreamSynchronize(c->stream);
    if (c->stage.size() > 1) {
      auto big = std::max_element(c->stage.begin(), c->stage.end(),
                                  [](const std::pair<void*, size_t>& a, const std::pair<void*, size_t>& b) {
                                    return a.second < b.second;
                                  });
      const auto keep = *big;
      for (auto& blk : c->stage)
        if (blk.first != keep.first) hipFree(blk.first);
      c->stage.assign(1, keep);
    }
  }
  vw_status carve(size_t bytes, void** out) {
    bytes = align_up(std::max<size_t>(bytes, 16), 256);
    for (; used_block < c->stage.size(); ++used_block, used_off = 0) {
      auto& blk = c->stage[used_block];
      if (used_off + bytes <= blk.second) {
        *out = static_cast<char*>(blk.first) + used_off;
        used_off += bytes;
        return VW_OK;
      }
    }
    // a new block covers everything this call has carved so far plus this request, so the pool
    // converges to one block per call shape (see the destructor)
    size_t carved = bytes;
    for (size_t k = 0; k < used_block && k < c->stage.size(); ++k) carved += c->stage[k].second;
    if (used_block < c->stage.size()) carved += used_off;
    const size_t want = std::max({carved, (size_t)4 << 20});
    void* p = nullptr;
    VW_HIP(hipMalloc(&p, want));
    c->stage.push_back({p, want});
    used_block = c->stage.size() - 1;
    used_off = bytes;
    *out = p;
    return VW_OK;
  }
  template <typename T>
  vw_status in(const T* host, size_t count, T** dev) {
    void* p = nullptr;
    VW_TRY(carve(count * sizeof(T), &p));
    if (host && count) VW_HIP(hipMemcpyAsync(p, host, count * sizeof(T), hipMemcpyHostToDevice, c->stream));
    *dev = reinterpret_cast<T*>(p);
    return VW_OK;
  }
  // `planes` blocks of `count` elements, the host blocks `host_stride` elements apart (a row block of a
  // [planes][B][N] host array), packed on the device
  template <typename T>
  vw_status in_planes(const T* host, size_t planes, size_t count, size_t host_stride, T** dev) {
    void* p = nullptr;
    VW_TRY(carve(planes * count * sizeof(T), &p));
    if (host && count && planes)
      VW_HIP(hipMemcpy2DAsync(p, count * sizeof(T), host, host_stride * sizeof(T), count * sizeof(T), planes,
                              hipMemcpyHostToDevice, c->stream));
    *dev = reinterpret_cast<T*>(p);
    return VW_OK;
  }
  template <typename T>
  vw_status out(T* host, const T* dev, size_t count) {
    if (host && count) VW_HIP(hipMemcpyAsync(host, dev, count * sizeof(T), hipMemcpyDeviceToHost, c->stream));
    return VW_OK;
  }
  template <typename T>
  vw_status out_planes(T* host, const T* dev, size_t planes, size_t count, size_t host_stride) {
    if (host && count && planes)
      VW_HIP(hipMemcpy2DAsync(host, host_stride * sizeof(T), dev, count * sizeof(T), count * sizeof(T), planes,
                              hipMemcpyDeviceToHost, c->stream));
    return VW_OK;
  }
};


// Host-memory forward of B rows: x[B][ldx] in, details as J host planes `det_stride` elements apart
// (B * N for a whole batch; the global B * N for a row block of a sharded batch), approx [B][N].
// Caller holds c->mu.  Synchronous.
template <typename T>
static vw_status forward_host(vw_ctx* c, const T* x, int64_t B, int64_t N, int64_t ldx, const double* lo,
                              const double* hi, int L, int boundary, int J, unsigned flags, T* details,
                              int64_t det_stride, T* approx) {
  if (c->capturing) return fail(VW_ERR_STATE, "host-memory calls cannot be captured (they synchronize)");
  Staging s(c);
  T *dx, *dd, *da;
  VW_TRY(s.in(x, (size_t)(B - 1) * ldx + N, &dx));  // (the last row's padding need not exist)
  VW_TRY(s.in<T>(nullptr, (size_t)J * B * N, &dd));
  VW_TRY(s.in<T>(nullptr, (size_t)B * N, &da));
  VW_TRY(forward_impl<T>(c, dx, B, N, ldx, lo, hi, L, boundary, J, flags & ~(VW_FLAG_SYNC | VW_FLAG_HOST_MEMORY), dd,
                         da, false, -1, nullptr, false));
  VW_TRY(s.out_planes(details, dd, (size_t)J, (size_t)(B * N), (size_t)det_stride));
  VW_TRY(s.out(approx, da, (size_t)B * N));
  VW_HIP(hipStreamSynchronize(c->stream));
  return VW_OK;
}

template <typename T>
static vw_status inverse_host(vw_ctx* c, const T* details, int64_t det_stride, const T* approx, int64_t B, int64_t N,
                              const double* lo, const double* hi, int L, int wid, int boundary, int J,
                              unsigned detail_mask, int approx_zero, unsigned flags, T* y) {
  if (c->capturing) return fail(VW_ERR_STATE, "host-memory calls cannot be captured (they synchronize)");
  Staging s(c);
  T *dd = nullptr, *da = nullptr, *dy;
  if (detail_mask) VW_TRY(s.in_planes(details, (size_t)J, (size_t)(B * N), (size_t)det_stride, &dd));
  if (!approx_zero) VW_TRY(s.in(approx, (size_t)B * N, &da));
  VW_TRY(s.in<T>(nullptr, (size_t)B * N, &dy));
  VW_TRY(inverse_impl<T>(c, dd, da, B, N, lo, hi, L, wid, boundary, J, detail_mask, approx_zero,
                         flags & ~(VW_FLAG_SYNC | VW_FLAG_HOST_MEMORY), dy, false, nullptr, 0));
  VW_TRY(s.out(y, dy, (size_t)B * N));
  VW_HIP(hipStreamSynchronize(c->stream));
  return VW_OK;
}

template <typename T>
static vw_status modwt_forward(vw_ctx* c, const T* x, int64_t B, int64_t N, int64_t ldx, const double* lo,
                               const double* hi, int L, int wid, int boundary, int J, unsigned flags, T* details,
                               T* approx) {
  (void)wid;
  VW_TRY(check_common(c, x, details, lo, hi, B, N, L, boundary));
  if (!approx) return fail(VW_ERR_NULL, "approx is null");
  if (ldx < N) return fail(VW_ERR_ARG, "ldx (%lld) < N (%lld)", (long long)ldx, (long long)N);
  VW_TRY(check_levels(N, L, J, flags));
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    VW_TRY(forward_host<T>(c, x, B, N, ldx, lo, hi, L, boundary, J, flags, details, B * N, approx));
    return ok();
  }
  VW_TRY(forward_impl<T>(c, x, B, N, ldx, lo, hi, L, boundary, J, flags, details, approx, false, -1, nullptr, false));
  return ok();
}

template <typename T>
static vw_status modwt_inverse(vw_ctx* c, const T* details, const T* approx, int64_t B, int64_t N, const double* lo,
                               const double* hi, int L, int wid, int boundary, int J, unsigned detail_mask,
                               int approx_zero, unsigned flags, T* y) {
  if (!c) return fail(VW_ERR_NULL, "ctx is null");
  if (!y || !lo || !hi) return fail(VW_ERR_NULL, "null argument");
  if (!details && detail_mask) return fail(VW_ERR_NULL, "details is null");
  if (!approx && !approx_zero) return fail(VW_ERR_NULL, "approx is null");
  VW_TRY(check_common(c, y, y, lo, hi, B, N, L, boundary));
  if (J < 1 || J > kMaxLevels) return fail(VW_ERR_LEVEL, "levels must be in 1..%d", kMaxLevels);
  // applyScaledInverseMODWT guard :561-574 (reconstruct has no level cap, only L_j <= N); the SWT
  // periodic inverse (VectorWaveSwtAdapter.reconstructPeriodic :444-474) wraps instead.
  if ((flags & VW_FLAG_CORE_LEVELS) && vw_upsampled_length(L, J) > N)
    return fail(VW_ERR_TOO_LARGE, "Upsampled reconstruction filter length exceeds signal length");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    VW_TRY(inverse_host<T>(c, details, B * N, approx, B, N, lo, hi, L, wid, boundary, J, detail_mask, approx_zero,
                           flags, y));
    return ok();
  }
  VW_TRY(inverse_impl<T>(c, details, approx, B, N, lo, hi, L, wid, boundary, J, detail_mask, approx_zero, flags, y,
                         false, nullptr, 0));
  return ok();
}

extern "C" vw_status vw_modwt_forward_f64(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx,
                                          const double* lo, const double* hi, int L, int wid, int boundary, int J,
                                          unsigned flags, double* details, double* approx) {
  return modwt_forward<double>(c, x, B, N, ldx, lo, hi, L, wid, boundary, J, flags, details, approx);
}
extern "C" vw_status vw_modwt_forward_f32(vw_ctx* c, const float* x, int64_t B, int64_t N, int64_t ldx,
                                          const double* lo, const double* hi, int L, int wid, int boundary, int J,
                                          unsigned flags, float* details, float* approx) {
  return modwt_forward<float>(c, x, B, N, ldx, lo, hi, L, wid, boundary, J, flags, details, approx);
}
extern "C" vw_status vw_modwt_inverse_f64(vw_ctx* c, const double* details, const double* approx, int64_t B,
                                          int64_t N, const double* lo, const double* hi, int L, int wid, int boundary,
                                          int J, unsigned detail_mask, int approx_zero, unsigned flags, double* y) {
  return modwt_inverse<double>(c, details, approx, B, N, lo, hi, L, wid, boundary, J, detail_mask, approx_zero,
                               flags, y);
}
extern "C" vw_status vw_modwt_inverse_f32(vw_ctx* c, const float* details, const float* approx, int64_t B,
                                          int64_t N, const double* lo, const double* hi, int L, int wid, int boundary,
                                          int J, unsigned detail_mask, int approx_zero, unsigned flags, float* y) {
  return modwt_inverse<float>(c, details, approx, B, N, lo, hi, L, wid, boundary, J, detail_mask, approx_zero, flags,
                              y);
}

// ------------------------------------------------------------------------------------------------
// One batch over several contexts, one host thread per context ("each device has its
// own context, stream, input generator and output buffers; one host thread per device").  The
// reference parallelises one call in-process too (VectorWaveSwtAdapter.java:210-267 executor,
// BatchMODWT.multiLevelAoS :90-111 over a batch); here the batch is split into contiguous row
// blocks (vectorwave_amd/shard.py shard_rows: the first B % n blocks get one extra row) and block k
// runs on ctxs[k] from its own std::thread -- no exchange between devices.  Host memory only (the
// JNI / FFM caller's arrays): each thread stages its block through its context.
static void shard_block(int64_t B, int n, int k, int64_t* start, int64_t* rows) {
  const int64_t base = B / n, extra = B % n;
  *start = k * base + std::min<int64_t>(k, extra);
  *rows = base + (k < extra ? 1 : 0);
}

// fn(k) on context k, one host thread per context (k = 0 on the calling thread); the first failing
// context's status, its message prefixed with `what` k.
template <typename F>
static vw_status run_per_ctx(vw_ctx* const* ctxs, int nctx, const char* what, F&& fn) {
  if (!ctxs) return fail(VW_ERR_NULL, "ctxs is null");
  if (nctx < 1) return fail(VW_ERR_ARG, "need at least one context (got %d)", nctx);
  for (int k = 0; k < nctx; ++k)
    if (!ctxs[k]) return fail(VW_ERR_NULL, "ctxs[%d] is null", k);
  struct Res { vw_status st = VW_OK; std::string msg; int64_t idx = -1; };
  std::vector<Res> res(nctx);
  auto work = [&](int k) {
    const vw_status st = fn(k);
    res[k].st = st;
    if (st != VW_OK) { res[k].msg = t_err; res[k].idx = t_err_index; }
  };
  std::vector<std::thread> th;
  th.reserve(nctx);
  for (int k = 1; k < nctx; ++k) th.emplace_back(work, k);
  work(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < nctx; ++k)
    if (res[k].st != VW_OK) {
      t_err = std::string(what) + " " + std::to_string(k) + ": " + res[k].msg;
      t_err_index = res[k].idx;
      return res[k].st;
    }
  return ok();
}

template <typename F>
static vw_status run_sharded(vw_ctx* const* ctxs, int nctx, int64_t B, F&& fn) {
  if (!ctxs) return fail(VW_ERR_NULL, "ctxs is null");
  if (nctx < 1) return fail(VW_ERR_ARG, "need at least one context (got %d)", nctx);
  for (int k = 0; k < nctx; ++k)
    if (!ctxs[k]) return fail(VW_ERR_NULL, "ctxs[%d] is null", k);
  if (B <= 0) return fail(VW_ERR_EMPTY, "batch must be non-empty (B=%lld)", (long long)B);
  const int used = (int)std::min<int64_t>(nctx, B);
  struct Res { vw_status st = VW_OK; std::string msg; int64_t idx = -1; };
  std::vector<Res> res(used);
  auto work = [&](int k) {
    int64_t start, rows;
    shard_block(B, used, k, &start, &rows);
    t_signal_base = start;  // signal numbers in this thread's error messages count from row 0 of the batch
    const vw_status st = fn(ctxs[k], start, rows);
    t_signal_base = 0;
    res[k].st = st;
    if (st != VW_OK) { res[k].msg = t_err; res[k].idx = t_err_index; }
  };
  std::vector<std::thread> th;
  th.reserve(used);
  for (int k = 1; k < used; ++k) th.emplace_back(work, k);
  work(0);
  for (auto& t : th) t.join();
  for (int k = 0; k < used; ++k)
    if (res[k].st != VW_OK) {
      int64_t start, rows;
      shard_block(B, used, k, &start, &rows);
      t_err = "block " + std::to_string(k) + " (rows " + std::to_string(start) + ".." +
              std::to_string(start + rows - 1) + "): " + res[k].msg;
      t_err_index = res[k].idx;
      return res[k].st;
    }
  return ok();
}

extern "C" vw_status vw_modwt_forward_multi_f64(vw_ctx* const* ctxs, int nctx, const double* x, int64_t B, int64_t N,
                                                int64_t ldx, const double* lo, const double* hi, int L, int wid,
                                                int boundary, int J, unsigned flags, double* details,
                                                double* approx) {
  if (!(flags & VW_FLAG_HOST_MEMORY)) return fail(VW_ERR_ARG, "multi-context calls take host memory (VW_FLAG_HOST_MEMORY)");
  if (!x || !details || !approx || !lo || !hi) return fail(VW_ERR_NULL, "null array argument");
  if (ldx < N) return fail(VW_ERR_ARG, "ldx (%lld) < N (%lld)", (long long)ldx, (long long)N);
  return run_sharded(ctxs, nctx, B, [&](vw_ctx* c, int64_t start, int64_t rows) -> vw_status {
    (void)wid;
    VW_TRY(check_common(c, x, details, lo, hi, rows, N, L, boundary));
    VW_TRY(check_levels(N, L, J, flags));
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipSetDevice(c->device);
    return forward_host<double>(c, x + start * ldx, rows, N, ldx, lo, hi, L, boundary, J, flags,
                                details + start * N, B * N, approx + start * N);
  });
}

extern "C" vw_status vw_modwt_inverse_multi_f64(vw_ctx* const* ctxs, int nctx, const double* details,
                                                const double* approx, int64_t B, int64_t N, const double* lo,
                                                const double* hi, int L, int wid, int boundary, int J,
                                                unsigned detail_mask, int approx_zero, unsigned flags, double* y) {
  if (!(flags & VW_FLAG_HOST_MEMORY)) return fail(VW_ERR_ARG, "multi-context calls take host memory (VW_FLAG_HOST_MEMORY)");
  if (!y || !lo || !hi) return fail(VW_ERR_NULL, "null argument");
  if (!details && detail_mask) return fail(VW_ERR_NULL, "details is null");
  if (!approx && !approx_zero) return fail(VW_ERR_NULL, "approx is null");
  if (J < 1 || J > kMaxLevels) return fail(VW_ERR_LEVEL, "levels must be in 1..%d", kMaxLevels);
  if ((flags & VW_FLAG_CORE_LEVELS) && vw_upsampled_length(L, J) > N)
    return fail(VW_ERR_TOO_LARGE, "Upsampled reconstruction filter length exceeds signal length");
  return run_sharded(ctxs, nctx, B, [&](vw_ctx* c, int64_t start, int64_t rows) -> vw_status {
    VW_TRY(check_common(c, y, y, lo, hi, rows, N, L, boundary));
    std::lock_guard<std::recursive_mutex> g(c->mu);
    hipSetDevice(c->device);
    return inverse_host<double>(c, details ? details + start * N : nullptr, B * N,
                                approx ? approx + start * N : nullptr, rows, N, lo, hi, L, wid, boundary, J,
                                detail_mask, approx_zero, flags, y + start * N);
  });
}

extern "C" vw_status vw_modwt_forward_multi_dev_f64(vw_ctx* const* ctxs, int nctx, const double* const* x,
                                                    const int64_t* rows, int64_t N, int64_t ldx, const double* lo,
                                                    const double* hi, int L, int wid, int boundary, int J,
                                                    unsigned flags, double* const* details,
                                                    double* const* approx) {
  if (flags & VW_FLAG_HOST_MEMORY)
    return fail(VW_ERR_ARG, "device-resident multi-context calls take device memory (no VW_FLAG_HOST_MEMORY)");
  if (!x || !rows || !details || !approx) return fail(VW_ERR_NULL, "null array argument");
  return run_per_ctx(ctxs, nctx, "context", [&](int k) -> vw_status {
    if (rows[k] == 0) return VW_OK;
    return modwt_forward<double>(ctxs[k], x[k], rows[k], N, ldx, lo, hi, L, wid, boundary, J, flags, details[k],
                                 approx[k]);
  });
}

extern "C" vw_status vw_modwt_inverse_multi_dev_f64(vw_ctx* const* ctxs, int nctx, const double* const* details,
                                                    const double* const* approx, const int64_t* rows, int64_t N,
                                                    const double* lo, const double* hi, int L, int wid,
                                                    int boundary, int J, unsigned detail_mask, int approx_zero,
                                                    unsigned flags, double* const* y) {
  if (flags & VW_FLAG_HOST_MEMORY)
    return fail(VW_ERR_ARG, "device-resident multi-context calls take device memory (no VW_FLAG_HOST_MEMORY)");
  if (!rows || !y || (!details && detail_mask) || (!approx && !approx_zero))
    return fail(VW_ERR_NULL, "null array argument");
  return run_per_ctx(ctxs, nctx, "context", [&](int k) -> vw_status {
    if (rows[k] == 0) return VW_OK;
    return modwt_inverse<double>(ctxs[k], details ? details[k] : nullptr, approx ? approx[k] : nullptr, rows[k], N,
                                 lo, hi, L, wid, boundary, J, detail_mask, approx_zero, flags, y[k]);
  });
}

// ------------------------------------------------------------------------------------------------
// Single level (MODWTTransform): any N >= 1 (no L <= N guard), pairwise inverse sums.
extern "C" vw_status vw_modwt1_forward_f64(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx,
                                           const double* lo, const double* hi, int L, int boundary, unsigned flags,
                                           double* approx, double* detail) {
  VW_TRY(check_common(c, x, detail, lo, hi, B, N, L, boundary));
  if (!approx) return fail(VW_ERR_NULL, "approx is null");
  if (ldx < N) return fail(VW_ERR_ARG, "ldx < N");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  const bool haar_quirk = (flags & VW_FLAG_BATCH_HAAR) && L == 2 && boundary == VW_PERIODIC;
  auto run = [&](const double* dx, double* da, double* dd, unsigned fl) -> vw_status {
    if (haar_quirk) {
      LaunchTimer lt(c, "forward1");
      hipError_t e = launch_single_haar_batch<double>(dx, ldx, B, (int)N, da, dd, c->stream);
      if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
      return VW_OK;
    }
    return forward_impl<double>(c, dx, B, N, ldx, lo, hi, L, boundary, 1, fl & ~VW_FLAG_FFT_SWITCH, dd, da, true,
                                -1, nullptr, false);
  };
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *dx, *da, *dd;
    VW_TRY(s.in(x, (size_t)B * ldx, &dx));
    VW_TRY(s.in<double>(nullptr, (size_t)B * N, &da));
    VW_TRY(s.in<double>(nullptr, (size_t)B * N, &dd));
    VW_TRY(run(dx, da, dd, flags & ~VW_FLAG_SYNC));
    VW_TRY(s.out(approx, da, (size_t)B * N));
    VW_TRY(s.out(detail, dd, (size_t)B * N));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  VW_TRY(run(x, approx, detail, flags));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

extern "C" vw_status vw_modwt1_inverse_f64(vw_ctx* c, const double* approx, const double* detail, int64_t B,
                                           int64_t N, const double* lo, const double* hi, int L, int boundary,
                                           unsigned flags, double* y) {
  VW_TRY(check_common(c, approx, detail, lo, hi, B, N, L, boundary));
  if (!y) return fail(VW_ERR_NULL, "y is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *da, *dd, *dy;
    VW_TRY(s.in(approx, (size_t)B * N, &da));
    VW_TRY(s.in(detail, (size_t)B * N, &dd));
    VW_TRY(s.in<double>(nullptr, (size_t)B * N, &dy));
    VW_TRY(inverse_impl<double>(c, dd, da, B, N, lo, hi, L, VW_WID_OTHER, boundary, 1, 1u, 0, flags & ~VW_FLAG_SYNC,
                                dy, true, nullptr, 0));
    VW_TRY(s.out(y, dy, (size_t)B * N));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  VW_TRY(inverse_impl<double>(c, detail, approx, B, N, lo, hi, L, VW_WID_OTHER, boundary, 1, 1u, 0, flags, y, true,
                              nullptr, 0));
  return ok();
}

// ------------------------------------------------------------------------------------------------
// SWT denoise: fused forward -> per-signal exact median of |d_1| -> inverse with fused threshold.
extern "C" vw_status vw_noise_sigma_f64(vw_ctx* c, const double* coeffs, int64_t B, int64_t N, unsigned flags,
                                        double* sigma) {
  if (!c || !coeffs || !sigma) return fail(VW_ERR_NULL, "null argument");
  if (B <= 0 || N <= 0) return fail(VW_ERR_EMPTY, "empty input");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *dc, *ds;
    VW_TRY(s.in(coeffs, (size_t)B * N, &dc));
    VW_TRY(s.in<double>(nullptr, (size_t)B, &ds));
    hipError_t e = launch_noise_sigma(dc, N, B, (int)N, 0.0, ds, nullptr, c->stream);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
    VW_TRY(s.out(sigma, ds, (size_t)B));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  hipError_t e = launch_noise_sigma(coeffs, N, B, (int)N, 0.0, sigma, nullptr, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

extern "C" vw_status vw_threshold_f64(vw_ctx* c, double* coeffs, int64_t B, int64_t N, const double* thr, int soft,
                                      unsigned flags) {
  if (!c || !coeffs || !thr) return fail(VW_ERR_NULL, "null argument");
  if (B <= 0 || N <= 0) return fail(VW_ERR_EMPTY, "empty input");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *dc, *dt;
    VW_TRY(s.in(coeffs, (size_t)B * N, &dc));
    VW_TRY(s.in(thr, (size_t)B, &dt));
    hipError_t e = launch_threshold<double>(dc, B, N, dt, soft, c->stream);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
    VW_TRY(s.out(coeffs, dc, (size_t)B * N));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  hipError_t e = launch_threshold<double>(coeffs, B, N, thr, soft, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

// out[c][r] = in[r][c] (rows x cols).  AoS [B][N] -> SoA [N][B] is (rows=B, cols=N); back is
// (rows=N, cols=B).  BatchSIMDMODWT.convertToSoA / convertFromSoA (BatchSIMDMODWT.java:282-308).
template <typename T>
static vw_status transpose_impl(vw_ctx* c, const T* in, int64_t rows, int64_t cols, unsigned flags, T* out) {
  if (!c || !in || !out) return fail(VW_ERR_NULL, "null argument");
  if (rows <= 0 || cols <= 0) return fail(VW_ERR_EMPTY, "empty input");
  if (in == out) return fail(VW_ERR_ARG, "transpose is out of place");
  if ((rows + 63) / 64 > 65535) return fail(VW_ERR_ARG, "rows %lld too large", (long long)rows);
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  const size_t n = (size_t)rows * (size_t)cols;
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    T *di, *dout;
    VW_TRY(s.in(in, n, &di));
    VW_TRY(s.in<T>(nullptr, n, &dout));
    hipError_t e = launch_transpose<T>(di, rows, cols, dout, c->stream);
    if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
    VW_TRY(s.out(out, dout, n));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  hipError_t e;
  {
    LaunchTimer lt(c, "transpose");
    e = launch_transpose<T>(in, rows, cols, out, c->stream);
  }
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

extern "C" vw_status vw_transpose_f64(vw_ctx* c, const double* in, int64_t rows, int64_t cols, unsigned flags,
                                      double* out) {
  return transpose_impl<double>(c, in, rows, cols, flags, out);
}

extern "C" vw_status vw_transpose_f32(vw_ctx* c, const float* in, int64_t rows, int64_t cols, unsigned flags,
                                      float* out) {
  return transpose_impl<float>(c, in, rows, cols, flags, out);
}

static vw_status denoise_device(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx, const double* lo,
                                const double* hi, int L, int wid, int boundary, int J, double threshold, int soft,
                                unsigned flags, double* y, double* thr_out) {
  const size_t plane = (size_t)B * (size_t)N;
  // workspace: details [J][B][N] | approx [B][N] | thr [B]   (tiled levels use ws beyond, via a 2nd alloc)
  const size_t bytes = align_up(((size_t)J + 1) * plane * sizeof(double), 256) + align_up((size_t)B * 8, 256);
  if (bytes > c->ws2_bytes) {
    if (c->capturing) return fail(VW_ERR_STATE, "workspace growth during capture: run the call once before capturing it");
    if (c->ws2) {
      hipDeviceSynchronize();
      ++c->ws_gen;
      hipFree(c->ws2);
      c->ws2 = nullptr;
      c->ws2_bytes = 0;
    }
    VW_HIP(hipMalloc(&c->ws2, bytes));
    c->ws2_bytes = bytes;
  }
  void* buf = c->ws2;
  double* det = reinterpret_cast<double*>(buf);
  double* app = det + (size_t)J * plane;
  double* thr = reinterpret_cast<double*>(reinterpret_cast<char*>(buf) +
                                          align_up(((size_t)J + 1) * plane * sizeof(double), 256));
  vw_status st = forward_impl<double>(c, x, B, N, ldx, lo, hi, L, boundary, J, flags & ~VW_FLAG_SYNC, det, app, false,
                                      -1, nullptr, false);
  if (st == VW_OK) {
    hipError_t e = hipSuccess;
    if (threshold < 0) {
      // T = sigma * Math.sqrt(2 * Math.log(n))  core/swt/VectorWaveSwtAdapter.java:514
      const double scale_c = std::sqrt(2 * std::log((double)N));
      LaunchTimer lt(c, "sigma");
      e = launch_noise_sigma(det, N, B, (int)N, scale_c, nullptr, thr, c->stream);
    } else if (c->capturing) {
      st = fail(VW_ERR_STATE, "a fixed threshold cannot be captured");
    } else {
      std::vector<double> h((size_t)B, threshold);
      e = hipMemcpyAsync(thr, h.data(), (size_t)B * sizeof(double), hipMemcpyHostToDevice, c->stream);
      if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
    }
    if (e != hipSuccess) st = fail(VW_ERR_DEVICE, "threshold stage failed: %s", hipGetErrorString(e));
  }
  if (st == VW_OK)
    st = inverse_impl<double>(c, det, app, B, N, lo, hi, L, wid, boundary, J, ~0u, 0, flags & ~VW_FLAG_SYNC, y, false,
                              thr, soft);
  if (st == VW_OK && thr_out) {
    hipError_t e = hipMemcpyAsync(thr_out, thr, (size_t)B * sizeof(double), hipMemcpyDeviceToDevice, c->stream);
    if (e != hipSuccess) st = fail(VW_ERR_DEVICE, "copy failed");
  }
  return st;
}

extern "C" vw_status vw_swt_denoise_f64(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx,
                                        const double* lo, const double* hi, int L, int wid, int boundary, int J,
                                        double threshold, int soft, unsigned flags, double* y,
                                        double* thresholds_out) {
  VW_TRY(check_common(c, x, y, lo, hi, B, N, L, boundary));
  if (ldx < N) return fail(VW_ERR_ARG, "ldx < N");
  VW_TRY(check_levels(N, L, J, flags));
  if (vw_upsampled_length(L, J) > N && boundary != VW_PERIODIC)
    return fail(VW_ERR_TOO_LARGE, "Upsampled reconstruction filter length exceeds signal length");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *dx, *dy, *dt = nullptr;
    VW_TRY(s.in(x, (size_t)B * ldx, &dx));
    VW_TRY(s.in<double>(nullptr, (size_t)B * N, &dy));
    if (thresholds_out) VW_TRY(s.in<double>(nullptr, (size_t)B, &dt));
    VW_TRY(denoise_device(c, dx, B, N, ldx, lo, hi, L, wid, boundary, J, threshold, soft, flags, dy, dt));
    VW_TRY(s.out(y, dy, (size_t)B * N));
    if (thresholds_out) VW_TRY(s.out(thresholds_out, dt, (size_t)B));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  VW_TRY(denoise_device(c, x, B, N, ldx, lo, hi, L, wid, boundary, J, threshold, soft, flags, y, thresholds_out));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

// ------------------------------------------------------------------------------------------------
// WaveletDenoiser (core/denoising/WaveletDenoiser.java): forward (single-level MODWTTransform for
// denoise()/denoiseFixed(), MultiLevelMODWTTransform for denoiseMultiLevel()), sigma = MAD of d_1,
// one threshold per (level, signal) by the method (vw_sigma.h), inverse with the per-level threshold
// fused into the detail staging.
static vw_status wavelet_denoise_device(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx,
                                        const double* lo, const double* hi, int L, int wid, int boundary, int levels,
                                        int method, double fixed, int soft, unsigned flags, double* y,
                                        double* thr_out) {
  const int J = levels > 0 ? levels : 1;
  const size_t plane = (size_t)B * (size_t)N;
  const size_t coef_bytes = align_up(((size_t)J + 1) * plane * sizeof(double), 256);
  const size_t bytes = coef_bytes + align_up((size_t)B * 8, 256) + align_up((size_t)J * B * 8, 256);
  if (bytes > c->ws2_bytes) {
    if (c->capturing) return fail(VW_ERR_STATE, "workspace growth during capture: run the call once before capturing it");
    if (c->ws2) {
      hipDeviceSynchronize();
      ++c->ws_gen;
      hipFree(c->ws2);
      c->ws2 = nullptr;
      c->ws2_bytes = 0;
    }
    VW_HIP(hipMalloc(&c->ws2, bytes));
    c->ws2_bytes = bytes;
  }
  double* det = reinterpret_cast<double*>(c->ws2);
  double* app = det + (size_t)J * plane;
  double* sig = reinterpret_cast<double*>(reinterpret_cast<char*>(c->ws2) + coef_bytes);
  double* thr = reinterpret_cast<double*>(reinterpret_cast<char*>(sig) + align_up((size_t)B * 8, 256));
  const unsigned fl = flags & ~VW_FLAG_SYNC;
  vw_status st = levels > 0 ? forward_impl<double>(c, x, B, N, ldx, lo, hi, L, boundary, J, fl, det, app, false, -1,
                                                   nullptr, false)
                            : forward_impl<double>(c, x, B, N, ldx, lo, hi, L, boundary, 1, fl & ~VW_FLAG_FFT_SWITCH,
                                                   det, app, true, -1, nullptr, false);
  if (st != VW_OK) return st;
  hipError_t e = hipSuccess;
  if (method == kThrFixed) {
    if (c->capturing) return fail(VW_ERR_STATE, "a fixed threshold cannot be captured");
    std::vector<double> h((size_t)B, fixed);
    e = hipMemcpyAsync(thr, h.data(), (size_t)B * sizeof(double), hipMemcpyHostToDevice, c->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(c->stream);
  } else {
    DenoiseConsts k;
    memset(&k, 0, sizeof(k));
    for (int j = 1; j <= J; ++j) k.level_scale[j - 1] = levels > 0 ? std::sqrt((double)(1 << j)) : 1.0;
    k.univ_c = std::sqrt(2.0 * std::log((double)N));
    k.log_n = std::log((double)N);
    k.method = method;
    k.n = (int)N;
    {
      LaunchTimer lt(c, "sigma");
      e = launch_noise_sigma(det, N, B, (int)N, 0.0, sig, nullptr, c->stream);
    }
    if (e == hipSuccess) {
      LaunchTimer lt(c, "threshold");
      e = launch_level_threshold(det, (long long)plane, sig, k, B, J, thr, c->stream);
    }
  }
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "threshold stage failed: %s", hipGetErrorString(e));
  if (levels > 0)
    st = inverse_impl<double>(c, det, app, B, N, lo, hi, L, wid, boundary, J, ~0u, 0, fl, y, false, thr, soft, B);
  else
    st = inverse_impl<double>(c, det, app, B, N, lo, hi, L, VW_WID_OTHER, boundary, 1, 1u, 0, fl, y, true, thr, soft);
  if (st == VW_OK && thr_out) {
    e = hipMemcpyAsync(thr_out, thr, (size_t)J * B * sizeof(double), hipMemcpyDeviceToDevice, c->stream);
    if (e != hipSuccess) st = fail(VW_ERR_DEVICE, "copy failed");
  }
  return st;
}

extern "C" vw_status vw_wavelet_denoise_f64(vw_ctx* c, const double* x, int64_t B, int64_t N, int64_t ldx,
                                            const double* lo, const double* hi, int L, int wid, int boundary,
                                            int levels, int method, double fixed_threshold, int soft, unsigned flags,
                                            double* y, double* thresholds_out) {
  VW_TRY(check_common(c, x, y, lo, hi, B, N, L, boundary));
  if (ldx < N) return fail(VW_ERR_ARG, "ldx < N");
  if (method < kThrUniversal || method > kThrFixed) return fail(VW_ERR_ARG, "Unknown threshold selection method");
  if (levels < 0) return fail(VW_ERR_LEVEL, "Invalid number of decomposition levels: %d", levels);
  if (levels > 0) {
    // calculateThreshold (:415-424): FIXED needs an explicit threshold (denoiseFixed is single-level)
    if (method == kThrFixed) return fail(VW_ERR_ARG, "Fixed threshold method requires explicit threshold value");
    VW_TRY(check_levels(N, L, levels, flags));
    if (vw_upsampled_length(L, levels) > N && boundary != VW_PERIODIC)
      return fail(VW_ERR_TOO_LARGE, "Upsampled reconstruction filter length exceeds signal length");
  }
  if (method == kThrSure && N > kSureMaxN)
    return fail(VW_ERR_UNSUPPORTED, "SURE threshold on device supports N <= %d (got %lld)", kSureMaxN, (long long)N);
  const int J = levels > 0 ? levels : 1;
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging s(c);
    double *dx, *dy, *dt = nullptr;
    VW_TRY(s.in(x, (size_t)B * ldx, &dx));
    VW_TRY(s.in<double>(nullptr, (size_t)B * N, &dy));
    if (thresholds_out) VW_TRY(s.in<double>(nullptr, (size_t)J * B, &dt));
    VW_TRY(wavelet_denoise_device(c, dx, B, N, ldx, lo, hi, L, wid, boundary, levels, method, fixed_threshold, soft,
                                  flags & ~VW_FLAG_HOST_MEMORY, dy, dt));
    VW_TRY(s.out(y, dy, (size_t)B * N));
    if (thresholds_out) VW_TRY(s.out(thresholds_out, dt, (size_t)J * B));
    VW_HIP(hipStreamSynchronize(c->stream));
    return ok();
  }
  VW_TRY(wavelet_denoise_device(c, x, B, N, ldx, lo, hi, L, wid, boundary, levels, method, fixed_threshold, soft, flags,
                                y, thresholds_out));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

// ------------------------------------------------------------------------------------------------
// Statistics of MODWTStreamingDenoiser (core/modwt/streaming/MODWTStreamingDenoiser.java:133-272):
// MathUtils.median / medianAbsoluteDeviation / standardDeviation on device rows, and the noise-window
// ring update.  Device pointers only (the window lives on the device between blocks).
extern "C" vw_status vw_median_f64(vw_ctx* c, const double* x, int64_t B, int64_t N, const double* center,
                                   unsigned flags, double* median_out) {
  if (!c || !x || !median_out) return fail(VW_ERR_NULL, "null argument");
  if (B <= 0 || N <= 0) return fail(VW_ERR_EMPTY, "Array cannot be null or empty");
  if (N > (1LL << 30)) return fail(VW_ERR_ARG, "row too long");
  if (flags & VW_FLAG_HOST_MEMORY) return fail(VW_ERR_UNSUPPORTED, "device pointers only");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  hipError_t e;
  if (center && N > kSigmaRegN) {
    // rows beyond the register-keyed centered path: deviations |x - center| into the workspace, then
    // the uncentered selection (any N) on them -- the same keys, the same exact order statistic
    if (B > 65535) return fail(VW_ERR_UNSUPPORTED, "centered median of more than 65535 long rows");
    const size_t need = (size_t)B * (size_t)N * sizeof(double);
    if (need > c->med_bytes) {
      if (c->capturing)
        return fail(VW_ERR_STATE, "median scratch growth during capture: run the call once before capturing it");
      if (c->med) {
        // the scratch may have been used on streams the context was bound to earlier, and graphs that
        // recorded a centred median hold its address: drain the device and make those graphs stale
        // (vw_graph_launch then refuses them with VW_ERR_STATE), as ensure_ws does for the workspace
        hipDeviceSynchronize();
        ++c->ws_gen;
        hipFree(c->med);
        c->med = nullptr;
        c->med_bytes = 0;
      }
      VW_HIP(hipMalloc(&c->med, need));
      c->med_bytes = need;
    }
    double* dev = reinterpret_cast<double*>(c->med);
    e = launch_abs_center(x, N, B, (int)N, center, dev, c->stream);
    if (e == hipSuccess) e = launch_median(dev, N, B, (int)N, nullptr, median_out, c->stream);
  } else {
    e = launch_median(x, N, B, (int)N, center, median_out, c->stream);
  }
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

extern "C" vw_status vw_stddev_f64(vw_ctx* c, const double* x, int64_t N, unsigned flags, double* out) {
  if (!c || !x || !out) return fail(VW_ERR_NULL, "null argument");
  if (N < 2) return fail(VW_ERR_ARG, "Need at least 2 values for standard deviation");
  if (N > (1LL << 30)) return fail(VW_ERR_ARG, "too many values");
  if (flags & VW_FLAG_HOST_MEMORY) return fail(VW_ERR_UNSUPPORTED, "device pointers only");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  hipError_t e = launch_seq_std(x, (int)N, out, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

// window[(start + k) % wsize] = |src[idx[k]]| for k < count; idx is a HOST array (the stratified
// sampling positions are integer bookkeeping, computed by the caller), staged to the device here.
extern "C" vw_status vw_window_gather_abs_f64(vw_ctx* c, const double* src, const int32_t* idx, int64_t count,
                                              double* window, int64_t wsize, int64_t start) {
  if (!c || !src || !window || (count > 0 && !idx)) return fail(VW_ERR_NULL, "null argument");
  if (wsize <= 0 || count < 0 || count > wsize || start < 0 || start >= wsize) return fail(VW_ERR_ARG, "bad window");
  if (count == 0) return ok();
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (c->capturing) return fail(VW_ERR_STATE, "cannot be captured");
  hipSetDevice(c->device);
  Staging s(c);
  int32_t* di = nullptr;
  VW_TRY(s.in(idx, (size_t)count, &di));
  hipError_t e = launch_gather_abs(src, di, (int)count, window, (int)wsize, (int)start, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  return ok();  // Staging's destructor synchronizes before freeing the index copy
}

// ------------------------------------------------------------------------------------------------
// Streaming (BatchStreamingMODWT)
extern "C" vw_status vw_stream_create(vw_ctx* c, const double* lo, const double* hi, int L, int boundary, int levels,
                                      vw_stream** out) {
  if (!c || !lo || !hi || !out) return fail(VW_ERR_NULL, "null argument");
  if (levels < 1) return fail(VW_ERR_ARG, "levels must be >= 1");
  if (levels > kMaxLevels) return fail(VW_ERR_ARG, "levels too large");
  if (L < 1 || L > kMaxTaps) return fail(VW_ERR_ARG, "bad filter length");
  if (boundary < VW_PERIODIC || boundary > VW_ZERO_PADDING) return fail(VW_ERR_BOUNDARY, "bad boundary");
  vw_stream* s = new vw_stream();
  s->ctx = c;
  s->lo.assign(lo, lo + L);
  s->hi.assign(hi, hi + L);
  s->L = L;
  s->boundary = boundary;
  s->levels = levels;
  s->hist.assign(levels, nullptr);
  s->snap.assign(levels, nullptr);
  s->hist_len.resize(levels);
  for (int j = 1; j <= levels; ++j) s->hist_len[j - 1] = (int)(vw_upsampled_length(L, j) - 1);
  *out = s;
  return ok();
}

static void free_hist(vw_stream* s) {
  for (auto* v : {&s->hist, &s->snap})
    for (auto& p : *v) {
      if (p) hipFree(p);
      p = nullptr;
    }
}

extern "C" vw_status vw_stream_destroy(vw_stream* s) {
  if (!s) return fail(VW_ERR_NULL, "stream is null");
  hipSetDevice(s->ctx->device);
  hipStreamSynchronize(s->ctx->stream);
  free_hist(s);
  delete s;
  return ok();
}

extern "C" int64_t vw_stream_batch(vw_stream* s) { return s ? s->last_batch : -1; }

extern "C" int64_t vw_stream_history_length(vw_stream* s, int level) {
  if (!s || level < 1 || level > s->levels) return -1;
  return s->hist_len[level - 1];
}

static vw_status stream_run(vw_stream* s, const double* blk, int64_t B, int64_t n, unsigned flags, double* details,
                            double* approx, bool flush) {
  vw_ctx* c = s->ctx;
  if (s->boundary == VW_PERIODIC) {
    // processMultiLevel PERIODIC -> BatchMODWT.multiLevelAoS (no cap), BatchStreamingMODWT.java:115-116
    return forward_impl<double>(c, blk, B, n, n, s->lo.data(), s->hi.data(), s->L, s->boundary, s->levels,
                                flags & ~VW_FLAG_SYNC, details, approx, false, -1, nullptr, false);
  }
  const bool first = !s->hist_init;
  const int mode = first ? -1 : kHaloHistory;
  return forward_impl<double>(c, blk, B, n, n, s->lo.data(), s->hi.data(), s->L, s->boundary, s->levels,
                              flags & ~VW_FLAG_SYNC, details, approx, false, mode, s->hist.data(), !flush,
                              s->snap[0] ? s->snap.data() : nullptr, first);
}

extern "C" vw_status vw_stream_process_f64(vw_stream* s, const double* block, int64_t B, int64_t n, unsigned flags,
                                           double* details, double* approx) {
  if (!s) return fail(VW_ERR_NULL, "stream is null");
  vw_ctx* c = s->ctx;
  VW_TRY(check_common(c, block, details, s->lo.data(), s->hi.data(), B, n, s->L, s->boundary));
  if (!approx) return fail(VW_ERR_NULL, "approx is null");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  if (s->boundary != VW_PERIODIC) {
    // ensureHistoryCapacity  BatchStreamingMODWT.java:310-324: batch change re-initialises history
    if (s->last_batch != B) {
      free_hist(s);
      for (int j = 0; j < s->levels; ++j)
        VW_HIP(hipMalloc(&s->hist[j], std::max<size_t>((size_t)B * s->hist_len[j] * sizeof(double), 16)));
      s->hist_init = false;
      s->last_batch = B;
    }
    if ((flags & VW_FLAG_REF_NONFINITE) && !s->snap[0])
      for (int j = 0; j < s->levels; ++j)
        VW_HIP(hipMalloc(&s->snap[j], std::max<size_t>((size_t)B * s->hist_len[j] * sizeof(double), 16)));
  }
  vw_status st;
  if (flags & VW_FLAG_HOST_MEMORY) {
    Staging sg(c);
    double *db, *dd, *da;
    VW_TRY(sg.in(block, (size_t)B * n, &db));
    VW_TRY(sg.in<double>(nullptr, (size_t)s->levels * B * n, &dd));
    VW_TRY(sg.in<double>(nullptr, (size_t)B * n, &da));
    st = stream_run(s, db, B, n, flags, dd, da, false);
    if (st != VW_OK) return st;
    VW_TRY(sg.out(details, dd, (size_t)s->levels * B * n));
    VW_TRY(sg.out(approx, da, (size_t)B * n));
    VW_HIP(hipStreamSynchronize(c->stream));
  } else {
    st = stream_run(s, block, B, n, flags, details, approx, false);
    if (st != VW_OK) return st;
    if (flags & VW_FLAG_SYNC) VW_HIP(hipStreamSynchronize(c->stream));
  }
  if (s->boundary != VW_PERIODIC) s->hist_init = true;
  return ok();
}

// flushMultiLevel  BatchStreamingMODWT.java:231-275: tail from level-1 history (ZERO: zeros;
// SYMMETRIC: hist[histLen-1-t]), run through every level's history without updating it.
extern "C" vw_status vw_stream_flush_f64(vw_stream* s, int64_t tail_len, unsigned flags, double* details,
                                         double* approx) {
  if (!s) return fail(VW_ERR_NULL, "stream is null");
  vw_ctx* c = s->ctx;
  if (s->boundary == VW_PERIODIC) return fail(VW_ERR_UNSUPPORTED, "Flush is only applicable to ZERO_PADDING/SYMMETRIC");
  if (tail_len <= 0) return ok();
  if (!s->hist_init || s->last_batch <= 0) return fail(VW_ERR_STATE, "No prior blocks processed; cannot flush");
  int min_hist = s->hist_len[0];
  for (int j = 0; j < s->levels; ++j) min_hist = std::min(min_hist, s->hist_len[j]);
  if (tail_len > min_hist)
    return fail(VW_ERR_ARG, "tailLength (%lld) exceeds maximum allowed across levels (%d)", (long long)tail_len,
                min_hist);
  if (!details || !approx) return fail(VW_ERR_NULL, "null output");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  if (c->capturing) return fail(VW_ERR_STATE, "flush cannot be captured");
  hipSetDevice(c->device);
  const int64_t B = s->last_batch;
  const int h0 = s->hist_len[0];
  std::vector<double> hist((size_t)B * h0), tail((size_t)B * tail_len, 0.0);
  if (s->boundary == VW_SYMMETRIC) {
    VW_HIP(hipMemcpyAsync(hist.data(), s->hist[0], hist.size() * sizeof(double), hipMemcpyDeviceToHost, c->stream));
    VW_HIP(hipStreamSynchronize(c->stream));
    for (int64_t b = 0; b < B; ++b)
      for (int64_t t = 0; t < tail_len; ++t) tail[b * tail_len + t] = hist[b * h0 + (h0 - 1 - t)];
  }
  Staging sg(c);
  double *dt, *dd = nullptr, *da = nullptr;
  VW_TRY(sg.in(tail.data(), tail.size(), &dt));
  const bool host = flags & VW_FLAG_HOST_MEMORY;
  if (host) {
    VW_TRY(sg.in<double>(nullptr, (size_t)s->levels * B * tail_len, &dd));
    VW_TRY(sg.in<double>(nullptr, (size_t)B * tail_len, &da));
  }
  VW_TRY(forward_impl<double>(c, dt, B, tail_len, tail_len, s->lo.data(), s->hi.data(), s->L, s->boundary, s->levels,
                              flags & ~VW_FLAG_SYNC, host ? dd : details, host ? da : approx, false, kHaloHistory,
                              s->hist.data(), false));
  if (host) {
    VW_TRY(sg.out(details, dd, (size_t)s->levels * B * tail_len));
    VW_TRY(sg.out(approx, da, (size_t)B * tail_len));
  }
  VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}

// ------------------------------------------------------------------------------------------------
// Device utilities
extern "C" vw_status vw_fill_uniform_f64(vw_ctx* c, double* x, int64_t count, uint64_t seed, int64_t offset) {
  if (!c || !x) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  hipError_t e = launch_fill_uniform<double>(x, count, seed, offset, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  return ok();
}

extern "C" vw_status vw_fill_uniform_f32(vw_ctx* c, float* x, int64_t count, uint64_t seed, int64_t offset) {
  if (!c || !x) return fail(VW_ERR_NULL, "null argument");
  std::lock_guard<std::recursive_mutex> g(c->mu);
  hipSetDevice(c->device);
  hipError_t e = launch_fill_uniform<float>(x, count, seed, offset, c->stream);
  if (e != hipSuccess) return fail(VW_ERR_DEVICE, "launch failed: %s", hipGetErrorString(e));
  return ok();
}

extern "C" vw_status vw_device_alloc(vw_ctx* c, int64_t bytes, void** out) {
  if (!c || !out) return fail(VW_ERR_NULL, "null argument");
  hipSetDevice(c->device);
  VW_HIP(hipMalloc(out, (size_t)std::max<int64_t>(bytes, 16)));
  return ok();
}

extern "C" vw_status vw_device_free(vw_ctx* c, void* p) {
  if (!c) return fail(VW_ERR_NULL, "null argument");
  hipSetDevice(c->device);
  if (p) VW_HIP(hipFree(p));
  return ok();
}

extern "C" vw_status vw_memcpy(vw_ctx* c, void* dst, const void* src, int64_t bytes, int kind) {
  if (!c || !dst || !src) return fail(VW_ERR_NULL, "null argument");
  hipSetDevice(c->device);
  const hipMemcpyKind k = kind == 0 ? hipMemcpyHostToDevice : kind == 1 ? hipMemcpyDeviceToHost
                                                                        : hipMemcpyDeviceToDevice;
  VW_HIP(hipMemcpyAsync(dst, src, (size_t)bytes, k, c->stream));
  VW_HIP(hipStreamSynchronize(c->stream));
  return ok();
}
