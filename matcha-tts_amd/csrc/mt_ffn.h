// Fused decoder FeedForward (mt_ffn.hip): BasicTransformerBlock's ff(norm3(x)) + x as one launch, the 1024-wide
// SnakeBeta intermediate kept on chip (model.py:580-609, 733-741).
#pragma once
#include "mt_common.h"

namespace mt {

struct FfnArgs {
  bf16* x;                // [frames][256] block state: read (LayerNorm input, residual) and overwritten in place
  int frames;             // B * T (1x1 convs: utterance boundaries do not matter)
  const float* ln_stats;  // [frames][4 slabs][2] (mean, M2) partials of x (the producer's VE_ROWSTATS)
  float ln_eps;
  const bf16* w1;         // mt_vconv 1x1 image of ff.net.0.proj with LayerNorm's gamma folded: [4][1024][64]
  const float* b1;        // [1024] (beta folded)
  const float* wsum;      // [1024] row sums of the packed w1 (VE_LN)
  const float* alpha;     // [1024] exp(alpha) (SnakeBeta)
  const float* ibeta;     // [1024] 1 / (exp(beta) + 1e-9)
  const bf16* w2;         // mt_vconv 1x1 image of ff.net.2: [16][256][64]
  const float* b2;        // [256]
  const float* emask;     // [frames] or null: y *= mask (the chain's last block hands out a masked copy)
  // the query-independent attention's output (mt_attn.hip, launch_uniform_attention with apply = false): when set,
  // the tile's rows are first updated x = bf16(x + ovec[utterance]) in LDS and the LayerNorm partials computed there
  // (attn_uni_apply_kernel's arithmetic; ln_stats unused)
  const float* ovec;      // [B][256] or null
  int T;                  // frames per utterance (ovec's utterance of frame f: f / T)
  const bf16* zero;       // >= 128 zero bytes
  bf16* trash;            // >= 1 KiB writable
};

// the fused kernel for the bf16 decoder's shape (C = 256, inner 1024); MT_FFN=0 in the environment or
// mt_ffn_set(0): the two mt_vconv launches instead (same bits)
int launch_ffn(const FfnArgs& a, hipStream_t st);
int ffn_set(int enable);  // -> the previous setting
int ffn_on();
// the fused kernel runs on levels of at least this many frames (B * T; default 16384 = 128 128-frame tiles,
// MT_FFN_MIN in the environment): on fewer tiles its latency-bound K loop loses to the two GEMMs (B = 32: level 0
// fused, 7.89 vs 8.05 ms per solve; level 1 too, 8.19)
int ffn_min_frames();
int ffn_set_min_frames(int frames);  // -> the previous setting

}  // namespace mt
