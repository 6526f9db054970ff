// Host-side model descriptions shared by the decoder (U-Net estimator + CFM solver) and
// the HiFi-GAN vocoder drivers. A model lists the reference state_dict tensors it needs
// (names and shapes, canonical order) and the byte layout of its packed weight buffer.
// The caller (PyTorch) owns every device buffer; these objects hold host metadata only.
#pragma once
#include <memory>
#include <string>
#include <vector>

#include "mt_conv.h"
#include "mt_misc.h"
#include "mt_vconv.h"

namespace mt {

struct ParamList {
  std::vector<std::string> names;
  std::vector<std::vector<long long>> shapes;
  int add(const std::string& n, std::vector<long long> s) {
    names.push_back(n);
    shapes.push_back(std::move(s));
    return (int)names.size() - 1;
  }
};

struct Packer {
  size_t off = 0;
  size_t take(size_t bytes) {
    const size_t o = off;
    off += (bytes + 255) & ~(size_t)255;
    return o;
  }
};

// A packed GEMM layer (Conv1d / Linear / ConvTranspose1d) — see mt_conv.h for the mapping.
struct GemmW {
  int kind = 0;  // 0 Conv1d / Linear, 1 ConvTranspose1d
  int cin = 0, cout = 0, k = 1, s = 1, pad = 0, dil = 1;
  int M = 0, Mpad = 0, taps = 1, cin_pad = 0, gpad = 0, ups = 1, opad = 0;
  std::vector<int> wsrc;  // weight params (several = rows stacked, e.g. Q|K|V)
  int bsrc = -1;          // bias param or -1 (zeros)
  std::vector<int> bsrcs; // stacked biases, one per weight param (overrides bsrc), e.g. q|k|v
  int ln_g = -1, ln_b = -1;  // LayerNorm (on the input channels) folded into W and bias
  size_t w_off = 0, b_off = 0;
  size_t v_off = 0;  // vconv image [cin/64][taps][Mpad128][64] (bf16 HiFi-GAN convs, mt_vconv.h)
  bool vc = false;
  int vrows = 0;     // ConvTranspose on vconv: polyphase rows per image (M / vrows images back to back)
  int vcin = 0;      // vconv image input channels when cin is zero-padded to a multiple of 64 (0: cin)
};

GemmW make_conv(int cout, int cin, int k, int stride, int pad, int dil, std::vector<int> w, int b,
                int esize, Packer& pk);
GemmW make_convT(int cin, int cout, int k, int s, int pad, int w, int b, int esize, Packer& pk);
int pack_gemm(const GemmW& g, int dtype, const float* const* params, char* P, hipStream_t st);
// output geometry for an input of Tin frames
void gemm_geom(const GemmW& g, int Tin, int* Tout, int* Ncols);
// ConvArgs with the weight/geometry fields of g filled in
ConvArgs gemm_args(const GemmW& g, const char* P, int B, int Tin);
size_t align256(size_t x);

// Decoder kernel variants, each bit-identical to the launches it replaces (mt_decoder_set_kernels): DECK_PROJ the
// final projection + ODE update on proj_euler_kernel (mt_conv.hip) instead of the generic conv kernel. On by
// default; MT_DECK=<mask> in the environment (read once) or dec_set_kernels() to change.
enum : int { DECK_PROJ = 1, DECK_ALL = 1 };
int dec_kernels();
int dec_set_kernels(int mask);  // -> the previous mask

// -------------------------------------------------------------------------------------
// U-Net estimator (model.py:834-1048) + CFM solver (model.py:1084-1109)
// -------------------------------------------------------------------------------------
struct Decoder {
  int c_cond = 160, n_mid = 2, n_blocks = 1, heads = 2, dtype = BF16;
  static constexpr int C = 256, TE = 1024, NF = 80;
  int inner = 128, n_res = 0, esize = 2;
  ParamList params;
  size_t packed_bytes = 0;

  struct Res {
    int dim_in;
    GemmW c1, c2, res;
    int gn1g, gn1b, gn2g, gn2b, mlp_w, mlp_b;
    size_t gn1_off, gn2_off, mlp_w_off, mlp_b_off;
  };
  struct TB {
    int ln1g, ln1b, ln3g, ln3b, alpha, beta;
    size_t ln1_off, ln3_off, snake_off;
    size_t wsq_off = 0, wsf_off = 0;  // vconv: row sums of the LN-folded qkv / ff1 images
    GemmW qkv, out, ff1, ff2;
  };
  size_t zero_off = 0;  // 256 zero bytes (vconv padding rows)
  // bf16: 1 = the ResnetBlock convs, down1 / up1 and the final block conv also run on mt_vconv (their
  // inputs are then kept masked by their producers), 0 = generic conv kernel for those (A/B, tests)
  int vconv = 1;
  // vconv path: block 2's GroupNorm + Mish + mask folded into the res conv's epilogue (VE_GNRES); 0: a separate
  // gn_apply pass (mt_decoder_set_vconv mode 2, A/B and tests)
  int gnres = 1;
  std::vector<Res> res;                // down0, down1, mid..., up0, up1
  std::vector<std::vector<TB>> tbs;    // per resnet
  GemmW down0, down1, up0, up1, fconv, fproj;
  int fgn_g, fgn_b, t1w, t1b, t2w, t2b, freq;
  size_t fgn_off, t1w_off, t1b_off, t2w_off, t2b_off, freq_off;

  int init(int c_cond, int n_mid, int n_blocks, int heads, int dtype);
  int pack(const float* const* p, void* packed, hipStream_t st) const;
  size_t workspace_bytes(int B, int T, int S) const;

  struct Work {
    char *xin, *H0, *H1, *XA, *XB, *XC, *U, *XF, *y1, *y2, *qkv, *ob, *ff, *trash;
    float *zm, *m1, *emb, *h1, *h2, *tb, *lns;
    double *gn1, *gn2;
    float* apart;  // attention key-split slots
    float* lnp;    // per frame, per 64-channel slab (sum, sum of squares): LayerNorm partials (vconv VE_ROWSTATS)
    float* upart;  // query-independent attention: per (utterance, slice) masked sums of the normalised rows
    float* mst;    // the solve's staged copy of the caller's mask (graph replays read only the workspace)
    int tb_ld;     // 0: one time bias per evaluation; n_res * C: one per utterance (step_times)
    const float* m0;
    // every utterance has padded frames at the full- / half-resolution level (the caller's max_valid < T /
    // <= T - 2): the transformer blocks there take the query-independent attention path
    bool uni0 = false, uni1 = false;
    // debug taps (mt_decoder_set_taps; honoured by step() only): fp32 [B][C][T_l] copies of the block outputs
    // the reference fixture G2 records (down0_res, down0_tb, mid1_tb, up0_out, up1_tb)
    float* const* taps = nullptr;
  };
  Work carve(void* ws, int B, int T, int S) const;
  int time_embed(const char* P, const Work& w, const TimeSched& ts, int S, hipStream_t st,
                 const float* t_dev = nullptr) const;

  struct Euler {
    float dt;
    int half_step, update_master;
  };
  template <class E>
  int eval(const char* P, const Work& w, int B, int T, int ev, const Euler& eu, hipStream_t st) const;
  template <class E>
  int resnet(const char* P, const Work& w, const Res& R, const void* x0, const void* x1, int c0, int cin,
             bool x_masked, void* out, const float* mask, int B, int Tl, const float* tb, bool* row_stats,
             hipStream_t st) const;
  // row_stats: w.lnp already holds the LayerNorm partials of x (written by the producing conv)
  template <class E>
  // uni: the query-independent attention path (every utterance padded at this level)
  int tblock(const char* P, const Work& w, const TB& t, void* x, const float* mask, bool mask_out, bool row_stats,
             bool uni, int B, int Tl, hipStream_t st) const;
  bool vc(const GemmW& g) const { return vconv && g.vc; }
  // decoder input row stride: zero-padded to a multiple of 64 channels (and stored masked) on the vconv path
  int xld() const { return (vconv && dtype == BF16) ? (c_cond + 63) / 64 * 64 : c_cond; }
  VConvArgs vargs(const GemmW& g, const char* P, const Work& w, const void* x, int B, int Tl, void* y) const;

  int init_inputs(const Work& w, const float* z, float temperature, const float* mu_y, const float* spks,
                  int B, int T, hipStream_t st) const;
  // max_valid: the most valid (mask = 1) frames of any utterance (0: unknown)
  int solve(const void* packed, const float* z_noise, float temperature, const float* mu_y,
            const float* mask, const float* spks, int B, int T, int n_steps, int solver, float* z_out,
            void* ws, size_t ws_bytes, hipStream_t st, int max_valid = 0) const;
  // 1 (default): the query-independent attention path when the caller's max_valid allows it; 0: always the
  // general Q.K^T path (A/B, tests)
  int uniform_attn = 1;
  // 1 (default): solve() replays its evaluation chain (time embedding + every estimator evaluation, ~550
  // launches for 10 Euler steps) as a captured hipGraph, keyed by (packed, workspace, geometry, path flags);
  // 0: launches it directly. Bypassed while a launch probe or the launch log is armed.
  int graphs = 1;
  static constexpr int N_TAPS = 5;
  float* taps[N_TAPS] = {};
  int tap(const Work& w, int i, const void* src, int B, int Tl, hipStream_t st) const;
  struct GraphCache;
  mutable std::shared_ptr<GraphCache> gcache;
  // the solve's evaluation chain: time embedding + n_steps Euler / midpoint steps on stream st
  int solve_chain(const char* P, const Work& w, const TimeSched& ts, int S, int B, int T, int n_steps, int solver,
                  hipStream_t st) const;
  // the cached executable graph of solve_chain for this key, captured on first use
  int chain_graph(const char* P, const Work& w, const TimeSched& ts, int S, int B, int T, int n_steps, int solver,
                  const void* ws, hipGraphExec_t* out) const;
  int step(const void* packed, const float* x, const float* mu_y, const float* mask, const float* spks,
           float t, int B, int T, float* out, void* ws, size_t ws_bytes, hipStream_t st) const;
  int step_times(const void* packed, const float* x, const float* mu_y, const float* mask, const float* spks,
                 const float* t_dev, int B, int T, float* out, void* ws, size_t ws_bytes, hipStream_t st) const;
};

// -------------------------------------------------------------------------------------
// Text encoder + duration predictor (model.py:148-535), mt_encoder.hip
// -------------------------------------------------------------------------------------
struct Encoder {
  int n_vocab = 0, C = 192, F = 768, heads = 2, layers = 6, k = 3, n_spks = 1, spk_dim = 0, W = 192;
  int DF = 256, dpk = 3, prenet = 1, dtype = F32, esize = 4, dk = 96;
  int mfma_attn = 1;  // bf16, dk = 96: the attention core on MFMA (enc_attn_mfma96_kernel); 0: the fp32-VALU kernel
  int f32vc = 1;      // fp32: convs on mt_vconv's fp32 mode (1, default) or the generic conv kernel (0; A/B, tests)
  int split = 0;      // fp32: the FFN convs on mt_vconv's split-bf16 mode (VConvArgs::f32 == 2; encoder precision
                      // "fp32x3": fp32-level products on the bf16 MFMA pipe) instead of exact fp32 MFMA
  ParamList params;
  size_t packed_bytes = 0;
  int emb = -1;
  size_t emb_off = 0;
  struct Pre {
    GemmW conv;
    int g, b;
    size_t ln_off;
  };
  std::vector<Pre> pre;
  GemmW pre_proj;
  struct Layer {
    GemmW qkv, o, f1, f2;
    int n1g, n1b, n2g, n2b;
    size_t n1_off, n2_off;
    size_t s1_off = 0, s2_off = 0;  // fp32: the FFN convs' split-bf16 images (vconv_repack_split6), 0 if none
  };
  std::vector<Layer> lay;
  size_t ezero_off = 0;  // 256 zero bytes (vconv padding rows) when the FFN convs run on vconv (bf16)
  GemmW proj_m, dp1, dp2, dpp;
  int dn1g, dn1b, dn2g, dn2b, theta;
  size_t dn1_off, dn2_off, theta_off;

  int init(int n_vocab, int n_channels, int filter_channels, int heads, int layers, int kernel, int n_spks,
           int spk_dim, int dp_filter, int dp_kernel, int prenet, int dtype);
  int pack(const float* const* p, void* packed, hipStream_t st) const;
  size_t workspace_bytes(int B, int Tx) const;
  int forward(const void* packed, const long long* ids, const long long* xlen, const float* spks, int B, int Tx,
              float* mu, float* logw, float* xmask, int* oov, void* ws, size_t ws_bytes, hipStream_t st) const;
  template <class E>
  int forward_t(const char* P, const long long* ids, const long long* xlen, const float* spks, int B, int Tx,
                float* mu, float* logw, float* xmask, int* oov, char* ws, hipStream_t st) const;
};

// -------------------------------------------------------------------------------------
// HiFi-GAN Generator (hifigan/models.py:148-206)
// -------------------------------------------------------------------------------------
// conv_post folded into the last stage's final pair (mt_vpair32 VE_POST; 1, the default) or its own launch (0):
// bit-identical; process-wide, returns the previous setting (MT_POSTFOLD=0 in the environment: off)
int vocoder_post_fold();
int vocoder_set_post_fold(int enable);

struct Vocoder {
  int resblock = 1, dtype = BF16, esize = 2;
  int fuse = 1;  // fused ResBlock stages (mt_rbfuse) where supported
  int vconv = 2; // LDS-DMA persistent convs (mt_vconv): 1 = C >= 128 stages, 2 = also C = 64 (per layer)
  // the 128-, 64- and 32-channel stages' ResBlock pairs as one launch each (mt_vpair128 / mt_vpair / mt_vpair32;
  // needs vconv >= 2). The 128-channel stage: 1 = its k = 3 resblock fused, 4 = all fused, 2 = none (per layer)
  int pair = 1;
  size_t zero_off = 0;  // 256 zero bytes in the packed buffer (vconv padding rows)
  bool any_vc = false;
  std::vector<int> up_rates, up_kernels, rb_kernels;
  std::vector<std::vector<int>> rb_dils;
  int up_init = 512, n_mels = 80;
  ParamList params;
  size_t packed_bytes = 0;
  GemmW pre, post;
  std::vector<GemmW> ups;
  // resblocks[i*nk+j]: first convs (c1 / convs), second convs (c2, resblock 1 only)
  std::vector<std::vector<GemmW>> rb1, rb2;

  int init(int resblock, const std::vector<int>& up_rates, const std::vector<int>& up_kernels, int up_init,
           const std::vector<int>& rb_kernels, const std::vector<std::vector<int>>& rb_dils, int dtype);
  int pack(const float* const* p, void* packed, hipStream_t st) const;
  bool stage_vc(int i) const;  // stage i runs its ResBlock convs through mt_vconv
  bool rb_vp(int i, int j) const;  // resblock j of stage i as fused pairs (mt_vpair128 / mt_vpair)
  bool stage_vp(int i) const;  // ... every resblock as fused pairs: the stage input needs no activated copy
  bool stage_vp32(int i) const;  // a 32-channel stage as fused pairs (mt_vpair32, generic weight packing)
  // stage i's ResBlocks as one fused-pair launch per pair: X -> XS (+ lrelu(XS) in RA when act_out)
  // wav (non-null, the last stage under post_fold): the final pair runs conv_post in its epilogue (VE_POST) and writes
  // the waveform instead of xs
  int pair_resblock(const char* P, int i, int j, int B, int L, const char* X, char* XS, char* Tb, char* R,
                    char* RA, char* trash, bool act_out, hipStream_t st, const int* lens = nullptr,
                    float* wav = nullptr) const;
  int pair_chain(const char* P, int i, int B, int L, const char* X, char* XS, char* Tb, char* R, char* RA,
                 char* trash, bool act_out, hipStream_t st, const int* lens = nullptr, float* wav = nullptr) const;
  // stage i (the last, a 32-channel pair stage, conv_post 32 -> 1 with k = 7) folds conv_post into its final pair
  bool post_fold(int i) const;
  // frames per mel frame at the input of upsampler i (the product of the first i upsampling rates)
  int rate_upto(int i) const;
  size_t frame_elems() const;  // max over stages of (samples per mel frame) x channels
  size_t workspace_bytes(int B, int T) const;
  // lens (device ints, or null): ragged batch, utterance b vocoded at its own lens[b] mel frames (mt_ragged.h);
  // its samples past 256 lens[b] are zero
  int forward(const void* packed, const float* mel, int B, int T, float* wav, void* ws, size_t ws_bytes,
              hipStream_t st, const int* lens = nullptr) const;
  bool ragged_supported() const;  // every stage on the bf16 vconv / pair path
  template <class E>
  int forward_t(const char* P, const float* mel, int B, int T, float* wav, char* ws, hipStream_t st,
                const int* lens) const;
  // the per-layer resblocks of wide stage i read the raw chain state (mt_rbconv VE_ACTIN): no activated copies
  bool stage_actin(int i, int B, int L, const int* lens) const;
  int stage_vconv(const char* P, int i, int B, int L, const char* X, const char* XA, char* XS, char* Tb, char* R,
                  char* RA, char* trash, bool act_out, hipStream_t st, const int* lens = nullptr) const;
  // upsampler i runs on vconv: its input lrelu(xs) is written by the producer (conv_pre / stage i-1)
  bool ups_vc(int i) const;
  int ups_vconv(const char* P, int i, int B, int L, const char* xa, char* X, char* XA, bool dual, char* trash,
                hipStream_t st, const int* lens = nullptr) const;
};

}  // namespace mt
