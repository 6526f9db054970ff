// Ragged batches for the vocoder: every utterance of a padded [B][T][C] batch is computed at its OWN length, as
// the reference's pipeline vocodes it (one utterance per call: main.py:181-198, MOS_audiou_generator.ipynb:265-277,
// where `synthesize` crops the mel to that utterance's y_length). Each conv treats the frames at and past its
// utterance's length as zero padding (exactly what a batch-1 call of that length sees), so its outputs below the
// length are the batch-1 outputs; tiles wholly past the length are not computed at all.
//
// A persistent kernel walks only the live column tiles: wave 0 builds, at kernel start, the inclusive prefix sums
// tc[b] = sum_{b' <= b} ceil(ncols(b') / BN) and the valid input frames lv[b] in LDS (2 * RAG_MAXB ints); a tile
// index r (over column tiles) maps to its utterance by a binary search over tc.
#pragma once
#include "mt_common.h"

namespace mt {

constexpr int RAG_MAXB = 512;                 // utterances per ragged launch
constexpr int RAG_LDS = 2 * RAG_MAXB * 4;     // tc + lv

// valid input frames of utterance b: lens[b] * lmul clamped to [0, Lpad]; column count = that + extra clamped to
// [0, cap]. Called by every thread of the workgroup (wave 0 works), followed by a barrier in the caller.
__device__ __forceinline__ void rag_build(int* tc, int* lv, const int* lens, int lmul, int Lpad, int extra, int cap,
                                          int B, int BN, int tid) {
  if (tid >= 64) return;
  const int per = (B + 63) >> 6, b0 = tid * per;
  int s = 0;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b < B) {
      const int L = min(max(lens[b] * lmul, 0), Lpad);
      const int nc = min(max(L + extra, 0), cap);
      s += (nc + BN - 1) / BN;
    }
  }
  int x = s;  // inclusive scan over the 64 lanes
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int v = __shfl_up(x, o, 64);
    if (tid >= o) x += v;
  }
  int run = x - s;
  for (int i = 0; i < per; ++i) {
    const int b = b0 + i;
    if (b < B) {
      const int L = min(max(lens[b] * lmul, 0), Lpad);
      const int nc = min(max(L + extra, 0), cap);
      run += (nc + BN - 1) / BN;
      tc[b] = run;
      lv[b] = L;
    }
  }
}

// utterance of column tile r (0 <= r < tc[B-1]): the first b with tc[b] > r
__device__ __forceinline__ int rag_find(const int* tc, int B, int r) {
  int lo = 0, hi = B - 1;
  while (lo < hi) {
    const int mid = (lo + hi) >> 1;
    if (tc[mid] > r) hi = mid;
    else lo = mid + 1;
  }
  return lo;
}

// first column tile of utterance b
__device__ __forceinline__ int rag_first(const int* tc, int b) { return b > 0 ? tc[b - 1] : 0; }

// A persistent workgroup's walk over its column tiles r0 < r1 < ... (tiles of one workgroup only increase): the
// utterance of each by advancing from the previous one (one or two LDS reads per tile where a binary search takes
// log2 B dependent ones), then the tile's first frame and the utterance's valid length, read once into scalar
// registers. (A kernel that reads lv[b] where it issues its LDS-DMAs gets it re-read from LDS after every DMA: the
// compiler cannot prove the DMA leaves that word alone.) Tiles past the last (phantom prefetches) stay in range.
struct RagTile {
  int b, n0, lv;
};
struct RagWalk {
  int b = 0;
  __device__ __forceinline__ RagTile at(const int* tc, const int* lv, int B, int BN, int r) {
    while (b < B - 1 && __builtin_amdgcn_readfirstlane(tc[b]) <= r) ++b;
    RagTile t;
    t.b = b;
    t.n0 = __builtin_amdgcn_readfirstlane((r - rag_first(tc, b)) * BN);
    t.lv = __builtin_amdgcn_readfirstlane(lv[b]);
    return t;
  }
};

}  // namespace mt
