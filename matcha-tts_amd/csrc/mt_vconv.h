// Persistent LDS-DMA implicit-GEMM Conv1d for the wide HiFi-GAN stages (bf16, C_out % 128 == 0,
// C_in % 64 == 0, stride 1): the resblock convs of stages 1 and 2 (hifigan/models.py:90-97), which
// dominate the vocoder's MFMA work. Inputs arrive PRE-ACTIVATED (the producer's epilogue wrote
// lrelu(x) next to x), so every operand byte goes global -> LDS by `global_load_lds_dwordx4` with no
// VGPR round trip and no prologue transform (see mt_vconv.hip for the pipeline).
#pragma once
#include <type_traits>

#include "mt_common.h"

namespace mt {

// epilogue flags: v = acc + bias, then in this order
enum : int {
  VE_RESID = 1,  // v += resid                        (ResBlock1 `xt + x`, models.py:96)
  VE_ACCUM = 2,  // v = y_old + v                     (`xs += ...`, models.py:189-192)
  VE_DIV = 4,    // v = v / div                       (`xs / num_kernels`, models.py:193)
  VE_ACT = 8,    // y = lrelu(round(v))               (conv1: only lrelu(xt) is ever consumed)
  VE_DUAL = 16,  // y = round(v), y2 = lrelu(round(v)) (chain state + the next conv1's input)
  VE_LN = 32,    // LayerNorm of the input folded in: acc := rstd[n] * (acc - mean[n] * wsum[m])
                 // (gamma folded into W, beta into the bias at pack time; model.py:733-741)
  VE_SNAKE = 64, // v + ibeta[m] * sin(v * alpha[m])^2 after the bias (SnakeBeta, model.py:580-609)
  VE_MASK = 128, // v * mask[frame] as the last step (a masked copy for consumers that read x * mask)
  VE_GNSTATS = 256,  // per-(utterance, 32-channel group) partial sum / sum of squares of v (fp64) -> gn_out
  VE_ROWSTATS = 512, // per frame and 64-channel slab: (mean, M2 = sum of squared deviations) of the stored
                     // values -> row_out (the next LayerNorm's statistics, consumed with VE_LNP; Welford /
                     // Chan form, no E[x^2] - mean^2 cancellation)
  VE_LNP = 1024,     // with VE_LN: ln_stats holds VE_ROWSTATS partials [frames][cin/64] instead of (mean, rstd)
  VE_RELU = 2048,    // max(v, 0) after the bias (text-encoder FFN, model.py:119-130)
  VE_PMASK = 4096,   // placed output: v * emask[output frame], frame = element / mask_div
  VE_ACTIN = 16384,  // mt_rbconv, with VE_ACT: the input is the RAW chain state; lrelu is applied to each staged row
                     // chunk in LDS (a pass over the chunk one step before its first use), so no producer writes an
                     // activated copy (VE_DUAL) for it
  VE_Y2ONLY = 32768, // with VE_DUAL: store y2 only (the raw y is dead: the vocoder's stage output, whose next
                     // upsampler reads lrelu(y) alone); mt_rbconv and the 64-channel ring pairs; every other kernel
                     // drops the flag and stores y as well (its launcher strips it)
  VE_POST = 131072,  // mt_vpair32 only, with VE_ACCUM | VE_DIV on the last stage's final pair: the stage output xs feeds
                     // conv_post (hifigan/models.py:193-195: tanh(conv_post(lrelu(xs, 0.01)))) in the same launch and the
                     // waveform is stored instead of xs (post_taps, mt_vpair.h)
  VE_SPLIT6 = 65536, // split-bf16 mode (VConvArgs::f32 == 2) only: the fp32 result is stored as its 3-way bf16 split
                     // h1 + h2 + h3 in the 6-plane layout [frames][6 M] = (h1, h1, h1, h2, h2, h3), the next split conv's
                     // input
  VE_GNRES = 8192,   // 1x1 only, with VE_RESID: the residual is the RAW input of a GroupNorm(M/32) + Mish + mask,
                     // applied here: resid := bf16(mish(GN(resid)) * emask[frame]) with the statistics merged
                     // per tile from the producer's VE_GNSTATS partials (ResnetBlock1D block2 -> + res(x),
                     // model.py:777-790; replaces a separate gn_apply pass)
};

// Compile-time K-loop schedule (mt_vconv CTN / CTT kernels and mt_rbconv). RL: the rows of a chunk are published
// RL steps before its first step (1; 2 for mt_rbconv's VE_ACTIN, whose in-LDS pass over them runs in between). Per
// loader wave and step s of a
// tile of S = NCH * TAPS steps, in program order: [row pieces of chunk c + NXB - 1, spread over taps t < TX of chunk
// c] [WPW weight pieces of step s + NW - 1] [NST epilogue stores on the tile's last step]. The epilogue's loads and
// any store whose issue depends on the data (statistics outputs) are left out of the counts: operations left out
// only make a wait stricter, and the epilogue's loads have completed before its stores (the compiler waits for them).
template <int NCH, int TAPS, int NW, int NXB, int TX, int WPW, int XPW, int NST, int RL = 1>
struct VcSched {
  static constexpr int S = NCH * TAPS;
  static constexpr int md(int v) { return ((v % S) + S) % S; }
  static constexpr int xr(int s) {
    const int t = s % TAPS;
    int n = 0;
    if (t < TX)
      for (int i = 0; i < XPW; ++i) n += (i * TX / XPW == t) ? 1 : 0;
    return n;
  }
  static constexpr int ops(int s) { return xr(s) + WPW + (s == S - 1 ? NST : 0); }
  static constexpr int after_w(int s) { return s == S - 1 ? NST : 0; }
  // VMEM operations issued after the group (rows / weights) of step v, up to the wait at the top of step s
  static constexpr int count(int v, bool rows, int s) {
    int n = (rows ? WPW : 0) + after_w(md(v));
    for (int u = v + 1; u < s; ++u) n += ops(md(u));
    return n;
  }
  // the wait at the top of step s (s = -1: the prologue's) publishes step s + 1: its weights (staged at step
  // s + 2 - NW) and, when it starts a chunk, that chunk's rows (their last pieces staged at step vx)
  static constexpr int wait(int s) {
    int n = count(s + 2 - NW, false, s);
    if ((s + RL) % TAPS == 0) {
      const int vx = ((s + RL) / TAPS - (NXB - 1)) * TAPS + TX - 1;
      const int nx = count(vx, true, s);
      n = n < nx ? n : nx;
    }
    return n;
  }
  static constexpr int v0 = (1 - NW) < (-(NXB - 1) * TAPS) ? (1 - NW) : (-(NXB - 1) * TAPS);
  // The prologue stages only what tile 0 needs, in virtual-step order v0 .. -1 (rows of chunks >= 0, weights of
  // steps >= 0; no stores): pops(v) operations at virtual step v. The first tile's waits whose data came from the
  // prologue count those instead of a previous tile's (wait_first; equal to wait(s) elsewhere).
  static constexpr int vfloor(int v) { return v >= 0 ? v / TAPS : -((-v + TAPS - 1) / TAPS); }
  static constexpr int prows(int v) { return vfloor(v) + NXB - 1 >= 0 ? xr(md(v)) : 0; }
  static constexpr int pw(int v) { return v + NW - 1 >= 0 ? WPW : 0; }
  static constexpr int pops(int v) { return prows(v) + pw(v); }
  static constexpr int count_first(int v, bool rows, int s) {
    if (v >= 0) return count(v, rows, s);
    int n = rows ? pw(v) : 0;
    for (int u = v + 1; u < 0; ++u) n += pops(u);
    for (int u = 0; u < s; ++u) n += ops(u);
    return n;
  }
  static constexpr int wait_first(int s) {
    int n = count_first(s + 2 - NW, false, s);
    if ((s + RL) % TAPS == 0) {
      const int vx = ((s + RL) / TAPS - (NXB - 1)) * TAPS + TX - 1;
      const int nx = count_first(vx, true, s);
      n = n < nx ? n : nx;
    }
    return n;
  }
};

// Host-side registry of the compile-time K-loop schedules the library instantiates, for the CPU schedule test
// (tests/test_vcsched.py replays each against its own model of the kernels' issue order). A kernel's host launcher
// odr-uses SchedReg<...>::reg, whose initializer records the schedule when the library is loaded.
constexpr int SCHED_FIELDS = 11;  // family (0 mt_vconv CT, 1 mt_rbconv), NCH, TAPS, NW, NXB, TX, WPW, XPW, NST, RL,
                                  // prologue wait (the count the kernel's prologue waits with)
using SchedWaits = int (*)(int* wait, int* wait_first, int cap);  // s = -1 .. S-1 -> entries 0 .. S; returns S
int sched_register(const int (&rec)[SCHED_FIELDS], SchedWaits waits);
int sched_count();
int sched_get(int i, int* rec, int* wait, int* wait_first, int cap);  // -> S, or -1
template <int FAM, int NCH, int TAPS, int NW, int NXB, int TX, int WPW, int XPW, int NST, int RL, int PW>
struct SchedReg {
  using SCH = VcSched<NCH, TAPS, NW, NXB, TX, WPW, XPW, NST, RL>;
  static int waits(int* w, int* wf, int cap) {
    if (cap < SCH::S + 1) return -1;
    for (int s = -1; s < SCH::S; ++s) {
      w[s + 1] = SCH::wait(s);
      wf[s + 1] = SCH::wait_first(s);
    }
    return SCH::S;
  }
  static const int reg;
};
template <int FAM, int NCH, int TAPS, int NW, int NXB, int TX, int WPW, int XPW, int NST, int RL, int PW>
const int SchedReg<FAM, NCH, TAPS, NW, NXB, TX, WPW, XPW, NST, RL, PW>::reg =
    sched_register({FAM, NCH, TAPS, NW, NXB, TX, WPW, XPW, NST, RL, PW}, &SchedReg::waits);

// compile-time loop: f(integral_constant<int, I>) for I in [I0, N)
template <int I, int N, class F>
__device__ __forceinline__ void vc_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    vc_for<I + 1, N>(f);
  }
}

template <int N>
__device__ __forceinline__ void vc_wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
}

struct VConvArgs {
  const bf16* x;      // [B][L][c0], already activated: channels [0, c0)
  const bf16* x1;     // [B][L][cin - c0]: channels [c0, cin) (a skip concatenation), or null
  int B, L, cin, c0;  // c0 = cin for one source; a multiple of 64
  const bf16* w;      // [cin/64][taps][Mpad][64]
  const float* bias;  // [M]
  int M, Mpad, taps, dil, pad;
  bf16* y;            // [B][L][M]
  bf16* y2;           // [B][L][M] (VE_DUAL)
  const bf16* resid;  // [B][L][M] (VE_RESID)
  float div, slope;
  const bf16* zero;   // >= 128 zero bytes: source of the conv's zero padding rows
  bf16* trash;        // >= 1 KiB writable: destination of the stores of frames past L
  const float* ln_stats;     // [B*L][2] (mean, rstd) of the input frames (VE_LN)
  const float* wsum;         // [M] row sums of the packed (gamma-folded, bf16) weights (VE_LN)
  const float* snake_alpha;  // [M] exp(alpha) (VE_SNAKE)
  const float* snake_ibeta;  // [M] 1 / (exp(beta) + 1e-9)
  const float* emask;        // [B*L] frame mask (VE_MASK)
  double* gn_out;            // [B][M/32][vconv_gn_parts(B, L, M)][2] (VE_GNSTATS)
  float* row_out;            // [B*L][M/64][2] (mean, M2) per 64-channel slab (VE_ROWSTATS)
  float ln_eps;              // VE_LNP
  int probe;                 // launch-probe site of k >= 2 launches (0: PROBE_VCONV, < 0: none)
  // Output placement (all 0 = the plain [B][L][M] layout). ConvTranspose1d as a polyphase conv
  // (rows = phase x C_out) writes column n, row m to element n * ldy + m - yshift of its utterance,
  // kept when it lies in [0, ylim); plain / dual epilogues only.
  int Lout;            // output columns per utterance
  int ldy;             // elements between consecutive columns of y
  int yshift;
  int ylim;
  long long ystride;   // elements per utterance of y
  int mask_div;        // VE_PMASK: output elements per frame
  int gn_parts;        // VE_GNSTATS: partial slots the consumer will merge (0: unchecked); must equal
                       // what this launch writes
  // VE_GNRES: the residual's GroupNorm
  const double* gn_in;       // [gn_B][M/32][gn_in_parts][2] (sum, sum of squares) of the raw residual
  int gn_in_parts, gn_T, gn_B;  // partial slots per (utterance, group), frames per utterance, utterances
  const float* gn_gamma;     // [M]
  const float* gn_beta;      // [M]
  float gn_eps;
  // 1: fp32 operands and output (x, w, y, resid, trash hold floats; w is the vconv_repack_f32 image); epilogues
  // 0 / VE_RELU / VE_MASK / VE_RESID and their combinations only; one source, plain [B][L][M] output.
  // 2: split-bf16 ("fp32x3"): x is the 6-plane bf16 split of an fp32 input ([B][L][6 cin0], planes h1 h1 h1 h2 h2 h3 of
  // x = h1 + h2 + h3, each h the bf16 rounding of what the previous parts leave), w the vconv_repack_split6 image
  // (planes W1 W2 W3 W1 W2 W1), cin = 6 cin0: one bf16 MFMA K loop sums the six products x1 W1 + x1 W2 + x1 W3 + x2 W1
  // + x2 W2 + x3 W1 in fp32 (fp32-level accuracy on the bf16 MFMA pipe); the epilogue is the fp32 mode's (resid, y
  // fp32), or with VE_SPLIT6 the 6-plane split of the result
  int f32;
  // diagnostic builds (-DVCONV_TS) only: per-workgroup phase timestamps (s_memrealtime, 100 MHz) of this launch go
  // to ts[(ts_slot * 256 + workgroup) * 4 + 0..3]; set by launch_vconv, unused otherwise
  unsigned long long* ts;
  int ts_slot;
  // ragged batch (mt_ragged.h; k >= 2, bf16, B <= RAG_MAXB): utterance b's valid input frames are lens[b] * lmul
  // (device ints); frames past them read as zero padding and column tiles past them are not computed. null: every
  // utterance has L frames
  const int* lens;
  int lmul;
  int xcd_tiles;  // set by launch_vconv: 1 = XCD-major tile ownership (mt_vconv.hip), 0 = round-robin walk
};

// LayerNorm (mean, rstd) of a 256-channel frame from its 4 slab partials (mean_i, M2_i), 64 values each,
// packed (m0, q0, m1, q1), (m2, q2, m3, q3): Chan's merge, var = M2 / 256
__device__ __forceinline__ float2 ln_merge4(f32x4 p01, f32x4 p23, float eps) {
#pragma clang fp contract(off)  // the same bits at every call site (mt_vconv's LN epilogues, mt_ffn)
  const float mean = 0.25f * ((p01[0] + p01[2]) + (p23[0] + p23[2]));
  const float d0 = p01[0] - mean, d1 = p01[2] - mean, d2 = p23[0] - mean, d3 = p23[2] - mean;
  const float m2 = (p01[1] + p01[3]) + (p23[1] + p23[3]) + 64.f * ((d0 * d0 + d1 * d1) + (d2 * d2 + d3 * d3));
  return float2{mean, rsqrtf(m2 * (1.f / 256.f) + eps)};
}

// partial-sum slots per (utterance, group) that VE_GNSTATS writes: column tiles x waves across columns
int vconv_gn_parts(int B, int L, int M);
// an upper bound of vconv_gn_parts over B (workspace sizing)
int vconv_gn_parts_max(int L);
// shortest utterance VE_GNRES accepts (shorter: run gn_apply, then a plain VE_RESID conv)
int vconv_gnres_min_frames();

bool vconv_supported(int cin, int cout, int k, int dil, int stride);
// packed bytes of the [cin/64][taps][Mpad][64] image
size_t vconv_packed_bytes(int cin, int cout, int k);
// [Mpad0][taps][cin_pad] (pack_conv layout, bf16) -> [cin/64][taps][Mpad][64]
// cin_src < cin: the image's channels [cin_src, cin) are zero (an input zero-padded to a multiple of 64)
int vconv_repack(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st,
                 int cin_src = -1);
int launch_vconv(int ef, const VConvArgs& a, hipStream_t st);
// mt_rbconv: the HiFi-GAN wide-stage ResBlock convs (C_in = C_out in {128, 256}, k in {3, 7, 11}) on a K loop scheduled
// at compile time; launch_vconv dispatches to it (MT_RBCONV=0: off). Same results as the mt_vconv kernel, bit for bit.
bool rbconv_handles(int ef, const VConvArgs& a);
int launch_rbconv(int ef, const VConvArgs& a, int G, hipStream_t st);
int rbconv_set(int enable);  // -> the previous setting
// VE_ACTIN (conv1 reads the raw chain state and activates its rows in LDS; conv2 writes no activated copy): 1 (the
// default) or 0 (MT_ACTIN=0 in the environment); bit-identical either way; -> the previous setting
int rbconv_actin_set(int enable);
int rbconv_actin_on();
// the compile-time K loop of the decoder's / upsamplers' convs (1, default) or the runtime-cursor loop (0); -> previous
int vconv_set_ct(int enable);
// the process-wide kernel selection above as one value (a key of the decoder's captured graphs)
int vconv_path_id();
// fp32 mode (VConvArgs::f32): [Mpad0][taps][cin_pad] fp32 -> [cin/32][taps][Mpad][32] fp32
bool vconv_supported_f32(int cin, int cout, int k, int stride);
size_t vconv_packed_bytes_f32(int cin, int cout, int k);
int vconv_repack_f32(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st);
// split-bf16 mode (VConvArgs::f32 == 2): [Mpad0][taps][cin_pad] fp32 -> bf16 image [6 cin / 64][taps][cout][64] of the
// weight planes W1 W2 W3 W1 W2 W1 (W = W1 + W2 + W3, each part the bf16 rounding of what the previous parts leave)
size_t vconv_packed_bytes_split6(int cin, int cout, int k);
int vconv_repack_split6(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st);
// the 3-way bf16 split of one fp32 value: h1 = RNE(v), h2 = RNE(v - h1), h3 = RNE(v - h1 - h2) (differences exact)
__device__ __forceinline__ void split3_bf16(float v, bf16& h1, bf16& h2, bf16& h3) {
  h1 = (bf16)v;
  const float r1 = v - (float)h1;
  h2 = (bf16)r1;
  h3 = (bf16)(r1 - (float)h2);
}
// image of a k = 3, stride 2, pad 1 conv (generic [Mpad0][3][cin_pad] source) as a 2-tap stride-1 conv over
// frame pairs (2C input channels): run it with L = T/2, cin = 2C, taps = 2, pad = 1 on the same [T][C] rows
int vconv_repack_s2(const void* src, int cin_pad, int C, int cout, void* dst, hipStream_t st);
// wsum[m] = sum over (chunk, tap, channel) of the packed bf16 image (VE_LN)
int vconv_wsum(const void* img, int cin, int taps, int cout, float* wsum, hipStream_t st);

}  // namespace mt
