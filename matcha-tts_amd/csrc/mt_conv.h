// Implicit-GEMM Conv1d on [B][T][C] activations (gfx950 MFMA), with fused prologues
// and epilogues. One kernel template covers every contraction on the synthesis path:
//   * Conv1d k/dilation/stride/pad (U-Net k3 convs, Downsample k3 s2, HiFi-GAN resblocks)
//   * Linear (k = 1): QKV / out / FF projections of the transformer blocks
//   * ConvTranspose1d (k = n*s) as a polyphase GEMM: GEMM row m = phase*C_out + co,
//     n = k/s taps over x[u-(n-1)..u], output frame = u*s + phase - pad.
// GEMM: M = output rows (channels x phases), N = output positions per utterance,
// K = taps x C_in. A = packed weights [Mpad][taps][cin_pad]; B = input rows staged
// (with halo) through LDS once per 64-byte channel chunk and reused by every tap.
#pragma once
#include "mt_common.h"

namespace mt {

// prologue flags (applied to every staged input element, in this order)
enum : int {
  PF_LN = 1,      // (x - mean[f]) * rstd[f]  (stats from rowstats(); gamma/beta folded into W)
  PF_GN = 2,      // mish(x * ga[b,c] + gs[b,c])                     (GroupNorm8 + Mish)
  PF_TB = 4,      // + tb[c]                                          (time-embedding bias)
  PF_LRELU = 8,   // leaky_relu(x, slope)
  PF_MASK = 16,   // * pmask[b, f]
};
// epilogue flags (v = acc + bias, then in this order)
enum : int {
  EF_SNAKE = 1,    // v + ibeta[c] * sin(v * alpha[c])^2            (SnakeBeta)
  EF_GNSTATS = 2,  // per-tile (sum, sumsq) of v per 32-channel group -> gn_out
  EF_GNADD = 4,    // v + mish(gy * ga + gs) * emask                 (ResnetBlock1D output)
  EF_MASK = 8,     // v * emask[b, f]
  EF_RESID = 16,   // v + resid
  EF_ACCUM = 32,   // y_old + v
  EF_DIV = 64,     // v / div
  EF_TANH = 128,   // tanh(v)
  EF_EULER = 256,  // Euler/midpoint update of z (fp32 master) + estimator-input slot
  EF_OUTF32 = 512, // store fp32 whatever the element type
  EF_DUAL = 1024,  // also store y2 = lrelu(round(v), slope): the activated copy a pre-activated consumer reads
  EF_RELU = 2048,  // max(v, 0) right after the bias                 (text encoder FFN / duration predictor)
  EF_FMASK = 4096, // v * emask as the LAST step                      ((x + proj(h)) * x_mask, prenet)
};

struct ConvArgs {
  // input: channels [0,c0) from x0 (row stride c0), [c0,cin) from x1 (row stride cin-c0)
  const void* x0;
  const void* x1;
  int c0, cin, Tin, B;
  // weights
  const void* w;        // [Mpad][taps][cin_pad] element type
  const float* bias;    // [M]
  int M, Mpad, cout, taps, dil, pad, stride, cin_pad;
  // output geometry: out frame = n*ups + (m / cout) - opad, channel = m % cout
  int Ncols, ups, opad, Tout;
  void* y;
  int ldy;
  void* y2;             // EF_DUAL: [B][Tout][ldy]
  // prologue params
  const float* pmask;   // [B][Tin]
  float slope;
  const float* ln_g;       // unused: LayerNorm gamma/beta are folded into the packed weights
  const float* ln_b;
  float ln_eps;
  const float* ln_stats;   // [B*Tin][2] per-frame (mean, rstd) from rowstats()
  const double* gn_in;  // [B][G][gn_ntiles][2] partial (sum, sumsq) of the GN'd tensor
  int gn_ntiles, gn_T;  // partial count per (b, group); frames of the GN'd tensor
  const float* gn_g;
  const float* gn_b;
  float gn_eps;
  const float* tb;      // [cin] (+ b * tb_ld for utterance b)
  int tb_ld;            // 0: one time bias for the batch
  // epilogue params
  const float* emask;   // [B][Tout]
  const void* resid;
  int ldr;
  float div;
  const float* snake_alpha;  // exp(alpha)
  const float* snake_ibeta;  // 1 / (exp(beta) + 1e-9)
  double* gn_out;            // [B][M/32][ntiles][2]
  const void* gy;            // GN'd tensor for EF_GNADD, [B][Tout][cout]
  float* zmaster;            // [B][Tout][cout] fp32
  void* xin_z;               // estimator input slot (element type), row stride ld_xin
  int ld_xin;
  float dt;
  int half_step;             // midpoint first half: inc = (pred*dt)*0.5
  int update_master;
  // ragged batch (the fp32 vocoder's per-utterance lengths, mt_ragged.h): utterance b's input has lens[b] * lmul
  // valid frames (zero padding past them); tiles past its output columns exit, outputs past them are not written
  const int* lens;
  int lmul;
  // 1: the tile configuration from the problem's per-utterance shape only, never from the batch size (the vocoder:
  // a row's result must not depend on how many other utterances share the launch; TSmall and TConv accumulate K in
  // different orders)
  int fixed_tile;
};

// Host launcher. Picks a tile configuration from (M, N), validates the geometry and
// launches on `stream`. Returns 0 or a negative error (mt_last_error()).
// *ntiles_out (optional) receives the per-utterance column-tile count (GN partials).
template <class E, int PF, int EF>
int launch_conv(const ConvArgs& a, hipStream_t stream, int* ntiles_out = nullptr);

// Runtime dispatch over the (PF, EF) combinations compiled in (used by the C ABI test
// entry point and by the drivers).
int launch_conv_dyn(int dtype, int pf, int ef, const ConvArgs& a, hipStream_t stream,
                    int* ntiles_out = nullptr);
// op-level entry (mt_op_conv1d): same kernels, separate symbols (TAG=1) for profiling
int launch_conv_op(int dtype, int pf, const ConvArgs& a, hipStream_t stream, int variant = -1);

// The bf16 decoder's final projection + ODE update (launch_conv<bf16, PF_GN | PF_MASK, EF_MASK | EF_EULER>'s
// arithmetic, bit-identical) on a dedicated kernel: the GroupNorm / Mish transform in registers, the weight image
// in LDS. Geometry: 1x1, C_in 256 -> 80 (n_feats), no ragged lengths (proj_euler_supported).
bool proj_euler_supported(const ConvArgs& a);
int launch_proj_euler(const ConvArgs& a, hipStream_t stream);

}  // namespace mt
