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

// The compile-time K loop of the ring pair kernels (vpair_kernel<EF, K> and vpair128_kernel<EF, K>, K > 0): per wave
// and tile of S = 2 NS steps (NS per conv), in program order: step s stages the weights of step s + 2 (2 pieces; past
// the workgroup's last step: phantom copies of valid weights, never read) after its barrier, then step 0 the old-xs
// loads (VE_ACCUM, 2 FN) and conv2's steps the next tile's rows (NXP pieces, piece i at conv2 step i * XSP / NXP:
// spread among the MFMAs rather than one burst; a phantom copy of the last tile after it); the tile's epilogue stores
// NST after step S - 1. So every vmcnt count is a constant (tests/test_vcsched.py replays the same model for mt_vconv
// / mt_rbconv).
template <int EF, int NS_, int NXP_, int FN_, int XSP_ = NS_>
struct VpkSched {
  static constexpr int NS = NS_, S = 2 * NS, NXP = NXP_, XSP = XSP_;
  static_assert(XSP >= 1 && XSP <= NS, "rows spread over conv2's steps");
  static constexpr int NACC = (EF & VE_ACCUM) ? 2 * FN_ : 0;
  static constexpr int NST = 2 * FN_ * ((EF & VE_DUAL) && !(EF & VE_Y2ONLY) ? 2 : 1);
  static constexpr int md(int q) { return ((q % S) + S) % S; }
  static constexpr int xpieces(int q) {  // row pieces conv2's step q (tile step) issues
    int n = 0;
    for (int i = 0; i < NXP; ++i) n += (md(q) >= NS && i * XSP / NXP == md(q) - NS) ? 1 : 0;
    return n;
  }
  static constexpr int after_w(int q) {  // operations a step issues after its weight pieces
    return (md(q) == 0 ? NACC : 0) + xpieces(q) + (md(q) == S - 1 ? NST : 0);
  }
  static constexpr int xlast = NS + (NXP - 1) * XSP / NXP;  // the step issuing the last row piece
  static constexpr int step_ops(int q) { return 2 + after_w(q); }
  // top of step s: the weights of step v = s + 1 (read at this step's end when s + 1 is in the same conv), else s's
  static constexpr int wait(int s) {
    const int v = (s % NS) + 1 < NS ? s + 1 : s;
    int n = after_w(v - 2);
    for (int u = v - 1; u < s; ++u) n += step_ops(u);
    return n;
  }
  // the first tile's step 0: step 1's weights are the prologue's last operation
  static constexpr int wait_first0 = 0;
  // tile start: its rows (the last piece issued at the previous tile's step xlast, after that step's weights)
  static constexpr int xwait = 2 * (S - 1 - xlast) + NST;
  static constexpr int xwait_first = 4;              // the first tile: the prologue's rows, then weights of steps 0, 1
  static constexpr int accwait = 2 * (S - 1) + NXP;  // the epilogue's old-xs loads (step 0)
};

// Round-5 pair-kernel variants, each bit-identical to the kernel it replaces (mt_vpair_set_kernels): bit 0 the
// 64-channel compile-time-K ring kernel (vpair_kernel<EF, 7 | 11>), bit 1 the 128-channel one (vpair128_kernel<EF, 3>).
// All on by default; MT_VPAIRK=<mask> in the environment (read once) or vpair_set_kernels() to change.
enum : int { VPK_CTK = 1, VPK_CTK128 = 2, VPK_ALL = 3 };
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
