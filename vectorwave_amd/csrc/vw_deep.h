#pragma once
// vw_deep.h -- arguments of the streaming deep-level kernels (vw_deep.hip), kept out of vw_internal.h
// so the kernel unit iterates without rebuilding the others.
#include "vw_internal.h"

namespace vw {

// Streaming deep-level kernels (vw_deep.hip): PERIODIC levels j0..j0+g-1 of long signals in one launch
// each way.  A workgroup streams C residues (64 bytes per decimated position) of one signal segment
// along the decimated coordinate q = t / P (P = 2^(j0-1)); per level an LDS ring of cap[r] positions.
// Rings: forward r = k (input of level j0+k); inverse r = k (approximation input A_k) and g + k (d_k).
template <typename T>
struct DeepArgs {
  const T* src;              // forward: input of level j0 [B][lda]; inverse: a_{j0+g-1} [B][N] (nullptr = zero)
  long long lda;
  T* out_d[kMaxGroup];       // forward: d of level j0+k [B][N]
  const T* src_d[kMaxGroup]; // inverse: d of level j0+k (nullptr = masked / zero)
  const T* thr[kMaxGroup];   // inverse denoise: thresholds [B] of level j0+k (nullptr = none)
  T* out;                    // forward: approximation of level j0+g-1; inverse: a_{j0-1}
  int* nf_flag;              // forward, VW_FLAG_REF_NONFINITE, out = a_J: a_J's probe (nullptr = off)
  long long B;
  int N, P, C, nq, nb;       // nq = N / P decimated positions, nb = P / C residue blocks
  int g;                     // levels in the group
  int warm;                  // warm-up positions before each segment (multiple of the tile)
  int seg, seglen;           // segments per residue block, positions per segment
  int depth;                 // tiles of DMA-fed input in flight ahead of the computing tile
  int cap[2 * kMaxGroup];    // ring capacities (positions)
  int off[2 * kMaxGroup];    // ring offsets (elements)
  int soft, taps;
  T lo[kMaxTaps];
  T hi[kMaxTaps];
};

template <typename T>
hipError_t launch_deep(const DeepArgs<T>& a, int lds_bytes, bool fma, bool inverse, hipStream_t st);

}  // namespace vw
