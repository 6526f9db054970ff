// Fused HiFi-GAN ResBlock1 pair (conv_{k,d} -> lrelu -> conv_{k,1} -> + x) for the 64-channel stage, bf16:
// the intermediate stays in LDS and the input's activation is applied on chip (see mt_vpair.hip).
#pragma once
#include "mt_vconv.h"

namespace mt {

struct VPairArgs {
  const bf16* x;        // [B][L][64] pair input (raw chain state; also the residual)
  int B, L;
  const bf16* w1;       // mt_vconv image [1][taps][64][64] of convs1[q] (dilation dil)
  const float* b1;      // [64]
  const bf16* w2;       // image of convs2[q] (dilation 1)
  const float* b2;      // [64]
  int taps, dil;
  bf16* y;              // [B][L][64] output (must not alias x); VE_ACCUM: also read (xs += ...)
  bf16* y2;             // [B][L][64] lrelu(y) (VE_DUAL: the next upsampler's input)
  float div, slope;     // VE_DIV divisor (nk), lrelu slope (0.1)
  const bf16* zero;     // >= 128 zero bytes
  bf16* trash;          // >= 1 KiB
};

// epilogue flags: 0 | VE_ACCUM | VE_DIV | VE_DUAL combinations (mt_vconv.h values)
bool vpair_supported(int C, int k, int d);
int launch_vpair(int ef, const VPairArgs& a, hipStream_t st);

}  // namespace mt
