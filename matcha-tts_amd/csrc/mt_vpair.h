// Fused HiFi-GAN ResBlock1 pair (conv_{k,d} -> lrelu -> conv_{k,1} -> + x) for the 128-, 64- and 32-channel
// stages, bf16: the intermediate stays in LDS and the input's activation is applied on chip (mt_vpair128.hip,
// mt_vpair.hip, mt_vpair32.hip).
#pragma once
#include "mt_ragged.h"
#include "mt_vconv.h"

namespace mt {

struct VPairArgs {
  const bf16* x;        // [B][L][C] pair input (raw chain state; also the residual)
  int B, L;
  const bf16* w1;       // C = 128 / 64: mt_vconv image [C/64][taps][C][64]; C = 32: generic packing [32][taps][32]
  const float* b1;      // [C]
  const bf16* w2;       // image of convs2[q] (dilation 1)
  const float* b2;      // [C]
  int taps, dil;
  bf16* y;              // [B][L][C] output (must not alias x); VE_ACCUM: also read (xs += ...)
  bf16* y2;             // [B][L][C] lrelu(y) (VE_DUAL: the next upsampler's input)
  float div, slope;     // VE_DIV divisor (nk), lrelu slope (0.1)
  const bf16* zero;     // >= 128 zero bytes
  bf16* trash;          // >= 1 KiB
  // ragged batch (mt_ragged.h, B <= RAG_MAXB): utterance b has lens[b] * lmul valid frames (zero padding past
  // them, tiles past them not computed); null: every utterance has L
  const int* lens;
  int lmul;
};

// Round-5 pair-kernel variants, each bit-identical to the kernel it replaces (mt_vpair_set_kernels): bit 0 the
// compile-time-K ring kernel (vpair_kernel<EF, 7 | 11>). All on by default; MT_VPAIRK=<mask> in the environment (read
// once) or vpair_set_kernels() to change.
enum : int { VPK_CTK = 1, VPK_ALL = 1 };
int vpair_kernels();
int vpair_set_kernels(int mask);

// epilogue flags: 0 | VE_ACCUM | VE_DIV | VE_DUAL combinations (mt_vconv.h values)
bool vpair_supported(int C, int k, int d);
int launch_vpair(int ef, const VPairArgs& a, hipStream_t st);
// the 32-channel kernel (weights in the generic conv packing)
bool vpair32_supported(int k, int d);
int launch_vpair32(int ef, const VPairArgs& a, hipStream_t st);
// the 128-channel kernel (mt_vconv image [2][taps][128][64])
bool vpair128_supported(int k, int d);
int launch_vpair128(int ef, const VPairArgs& a, hipStream_t st);

}  // namespace mt
