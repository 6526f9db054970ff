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
  // VE_POST (mt_vpair32): conv_post's [7][32] bf16 weights and bias, its lrelu slope, the [B][L] fp32 waveform
  const bf16* post_w;
  const float* post_b;
  float post_slope;
  float* wav;
};

// conv_post (32 -> 1 channel, k = 7, pad 3; hifigan/models.py:193-195) on MFMA, the one arithmetic of the bf16 path
// (post_conv_kernel, mt_vocoder.hip, and mt_vpair32's VE_POST epilogue). rows is an LDS image of v = bf16(lrelu(xs,
// 0.01)) with 64-byte rows (32 channels; 16-byte chunk q at slot q ^ ((row >> 1) & 2), zero outside the utterance).
// The seven taps are the A operand's rows (post_wtaps), so one MFMA over 16 rows gives every tap's partial sum of each
// row, D[t][n] = w[t] . v[r0 + n] (post_taps: one LDS read per row instead of one per tap and row); the output whose
// window starts at row r0 + o (frame r0 + o + 3 of the image) is sum_t D[t][o + t], gathered from two consecutive
// blocks by row rotations (post_combine).
__device__ __forceinline__ bf16x8 post_wtaps(const bf16* w, int lane) {  // lane % 16 = t < 7: w[t][8 (lane / 16) ..]
  bf16x8 v = {};
  if ((lane & 15) < 7) v = *reinterpret_cast<const bf16x8*>(w + (lane & 15) * 32 + 8 * (lane >> 4));
  return v;
}
__device__ __forceinline__ f32x4 post_taps(const char* rows, int r0, const bf16x8& wt, int lane) {
  const int r = r0 + (lane & 15);
  const bf16x8 bv = *reinterpret_cast<const bf16x8*>(rows + r * 64 + (((lane >> 4) ^ ((r >> 1) & 2)) * 16));
  return mfma16(wt, bv, f32x4{0.f, 0.f, 0.f, 0.f});
}
// element I of a post_taps result lives in 16-lane row g (tap 4 g + I): lane o of row 0 takes lane (o + I) & 15, of
// row 1 lane (o + 4 + I) & 15 (DPP row_ror:m moves lane l - m to lane l, so m = 16 - that shift)
// row 1's element 3 is tap 7, the A operand's zero row: its D = 0 x B is NaN wherever B holds a non-finite value
// (LDS rows past the image: post_conv_kernel's last block reads rows it never wrote), so that term is never taken
template <int I>
__device__ __forceinline__ float post_rot(float x) {
  const int v = __float_as_int(x);
  const int r = I == 0 ? v : __builtin_amdgcn_update_dpp(0, v, 0x120 + 16 - I, 0x1, 0xf, false);
  if constexpr (I == 3) return __int_as_float(r);
  return __int_as_float(__builtin_amdgcn_update_dpp(r, v, 0x120 + 12 - I, 0x2, 0xf, false));
}
// the 16 outputs of rows r0 .. r0 + 15 from da = post_taps(r0) and db = post_taps(r0 + 16): D[t][o + t] lies in da
// when o + t < 16, i.e. at a source lane l16 >= t, else in db (lane l16 = o + t - 16 < t), so only rows up to r0 + 21
// reach a kept sum. Sum order: taps 0..3 and 4..6 in order within rows 0 / 1, then row 0 + row 1; lanes 0..15 hold
// the block's sums
__device__ __forceinline__ float post_combine(const f32x4& da, const f32x4& db, int lane) {
  const int l16 = lane & 15, t0 = 4 * (lane >> 4);
  float s = post_rot<0>(l16 >= t0 ? da[0] : db[0]);
  s += post_rot<1>(l16 >= t0 + 1 ? da[1] : db[1]);
  s += post_rot<2>(l16 >= t0 + 2 ? da[2] : db[2]);
  s += post_rot<3>(l16 >= t0 + 3 ? da[3] : db[3]);
  const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(s), __float_as_uint(s), false, false);
  return __uint_as_float(r[0]) + __uint_as_float(r[1]);  // row 0: (taps 0..3) + (taps 4..6)
}
// conv_post's tanh, inline (tanhf is an out-of-line library call: a call sequence and its register saves in the
// epilogue): 1 - 2 / (2^(2 log2(e) x) + 1) on v_exp_f32 and v_rcp_f32, +-1 at the ends (2^x = inf / 0), absolute
// error ~2e-7 (the bf16 path's waveform is checked against the oracle at 1e-2)
__device__ __forceinline__ float post_tanh(float x) {
  const float e = __builtin_amdgcn_exp2f(x * 2.8853900817779268f);
  return 1.f - 2.f * __builtin_amdgcn_rcpf(e + 1.f);
}

// The compile-time K loop of the ring pair kernels (vpair_kernel<EF, K> and vpair128_kernel<EF, K>, K > 0): per wave
// the prologue stages the first tile's rows (NXP pieces), then the weights of steps 0 .. NWS - 2 (2 pieces each); per
// tile of S = 2 NS steps (NS per conv), in program order: step s stages the weights of step s + NWS - 1 (2 pieces; past
// the workgroup's last step: phantom copies of valid weights, never read) after its barrier, then step 0 the old-xs
// loads (VE_ACCUM, 2 FN) and conv2's steps the next tile's rows (NXP pieces, piece i at conv2 step i * XSP / NXP:
// spread among the MFMAs rather than one burst; a phantom copy of the last tile after it); the tile's epilogue stores
// NST after step S - 1. So every vmcnt count is a constant. Each instantiation a launcher uses is registered
// (VpkReg, families 2 / 3) and replayed on the CPU against an independent model of that issue order
// (tests/test_vcsched.py), the first-tile counts included.
template <int EF, int NS_, int NXP_, int FN_, int XSP_ = NS_, int NWS_ = 3>
struct VpkSched {
  static constexpr int NS = NS_, S = 2 * NS, NXP = NXP_, XSP = XSP_, NWS = NWS_;
  static_assert(XSP >= 1 && XSP <= NS, "rows spread over conv2's steps");
  // NWS >= 3: the weights a step's wait needs (its successor's) were issued at least one step earlier; NS >= 2: the
  // only weights the prologue stages that a wait after tile step 0 needs are step 1's, read at step 0's end
  static_assert(NWS >= 3 && NS >= 2, "ring depth / steps per conv");
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
  // top of step s: the weights of step v = s + 1 (read at this step's end when s + 1 is in the same conv), else s's;
  // step v's weights were issued first at step v - (NWS - 1)
  static constexpr int wait(int s) {
    const int v = (s % NS) + 1 < NS ? s + 1 : s;
    int n = after_w(v - (NWS - 1));
    for (int u = v - (NWS - 2); u < s; ++u) n += step_ops(u);
    return n;
  }
  // the prologue's weight steps 0 .. PW - 1 follow its rows
  static constexpr int PW = NWS - 1;
  // the first tile's step 0 needs step 1's weights (NS >= 2): the prologue's weight steps after step 1's
  static constexpr int wait_first0 = 2 * (PW - 2);
  // tile start: its rows (the last piece issued at the previous tile's step xlast, after that step's weights)
  static constexpr int xwait = 2 * (S - 1 - xlast) + NST;
  static constexpr int xwait_first = 2 * PW;         // the first tile: the prologue's rows, then its weight steps
  static constexpr int accwait = 2 * (S - 1) + NXP;  // the epilogue's old-xs loads (step 0)
};

// Registry record of a ring pair kernel's schedule (SchedReg's table, mt_vconv.h; tests/test_vcsched.py): family
// (2 mt_vpair C = 64, 3 mt_vpair128), NS, NXP, XSP, NACC, NST, NWS, EF, then 0s. Waits: w[1 + s] = wait(s) for the
// tile steps s = 0 .. S - 1; wf = {wait_first0, xwait, xwait_first, accwait}.
template <int FAM, class SCH, int EF>
struct VpkReg {
  static int waits(int* w, int* wf, int cap) {
    if (cap < SCH::S + 1 || cap < 4) return -1;
    w[0] = -1;
    for (int s = 0; s < SCH::S; ++s) w[s + 1] = SCH::wait(s);
    wf[0] = SCH::wait_first0;
    wf[1] = SCH::xwait;
    wf[2] = SCH::xwait_first;
    wf[3] = SCH::accwait;
    return SCH::S;
  }
  static const int reg;
};
template <int FAM, class SCH, int EF>
const int VpkReg<FAM, SCH, EF>::reg =
    sched_register({FAM, SCH::NS, SCH::NXP, SCH::XSP, SCH::NACC, SCH::NST, SCH::NWS, EF, 0, 0, 0}, &VpkReg::waits);

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
