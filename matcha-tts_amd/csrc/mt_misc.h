#pragma once
#include "mt_common.h"

namespace mt {

// solver evaluation times, passed by value to the time-embedding kernel
struct TimeSched {
  static constexpr int MAX = 128;
  float t[MAX];
};

int pack_conv(int dtype, const float* W, int kind, int cout, int cin, int k, int s, int row0, int Mrows,
              int Mpad, int taps, int cin_pad, void* out, hipStream_t st, const float* colscale = nullptr);
int rowstats(int dtype, const void* x, int rows, int C, float eps, float* stats, hipStream_t st);
int fold_bias(const float* W, const float* beta, int M, int K, float* out, hipStream_t st);
int pack_vec(const float* src, int period, int n, int op, float* out, hipStream_t st);

int bct_to_btc(int dtype, const float* src, int B, int C, int T, float scale, void* dst, int ld, int coff,
               hipStream_t st);
int btc_to_bct(int dtype, const void* src, int ld, int coff, int B, int C, int T, float* dst,
               hipStream_t st);
int spk_fill(int dtype, const float* spks, int B, int C, int T, void* dst, int ld, int coff, hipStream_t st);
int mask_half(const float* m0, int B, int T0, float* m1, hipStream_t st);
// dst[r][0..C) = src[r][0..C) (row strides ld_src / ld_dst, element type by dtype)
int copy_rows(int dtype, const void* src, int ld_src, int rows, int C, void* dst, int ld_dst, hipStream_t st);
// x[r][c] *= mask[r]
int mask_rows(int dtype, void* x, int rows, int C, const float* mask, hipStream_t st);

// ResnetBlock1D block tail (GroupNorm(8) -> Mish [-> + time bias] -> * mask, model.py Block1D/ResnetBlock1D)
// for bf16 rows y[b][t][C] whose GroupNorm partial sums (fp64 (sum, sumsq) per (b, 32-channel group,
// part), nparts per group) a conv epilogue produced: h = (mish(y * ga[b,c] + gs[b,c]) + tb[c]) * mask[b,t]
// tb_ld: elements between utterances' time biases (0: one shared vector)
int gn_apply(const void* y, int B, int T, int C, const double* part, int nparts, const float* gamma,
             const float* beta, float eps, const float* tb, int tb_ld, const float* mask, void* h, hipStream_t st);

// t_dev (optional): the S times in device memory instead of ts
int sinus_embed(const TimeSched& ts, int S, const float* freq, int half, float* emb, hipStream_t st,
                const float* t_dev = nullptr);
int rowdot(const float* x, int ldx, const float* W, const float* bias, float* y, int ldy, int yoff, int S,
           int O, int I, int pre, int post, hipStream_t st);
// n segments of O outputs each, segment j: y[s][yoff[j] + o] = post(b[j][o] + W[j][o] . pre(x[s])), one launch
constexpr int ROWDOT_MAXSEG = 8;
struct RowdotSegs {
  const float* W[ROWDOT_MAXSEG];
  const float* b[ROWDOT_MAXSEG];
  int yoff[ROWDOT_MAXSEG];
  int n;
};
int rowdot_segs(const float* x, int ldx, const RowdotSegs& sg, float* y, int ldy, int S, int O, int I, int pre,
                int post, hipStream_t st);

int durations(const float* logw, const float* xmask, float ls, int B, int Tx, float* w_ceil, float* cum,
              long long* ylen, hipStream_t st);
int alignment(const float* cum, const long long* ylen, int B, int Tx, int T, const float* mu, int C, float* attn,
              float* mu_y, float* y_mask, hipStream_t st);
int denorm_crop(const float* z, const float* mean, const float* stdv, int B, int C, int T, int Ty, float* mel,
                hipStream_t st);

// part (optional): key-split slots (attention_part_bytes, sized for the largest T launched on it);
// with it an unpadded utterance's keys are split over several workgroups + a merge launch
// Monotonic Alignment Search (mt_mas.hip, train_standalone.py:280-325)
size_t mas_workspace_bytes(int B, int Tx, int Ty);
int maximum_path(const float* value, const int* t_xs, const int* t_ys, int B, int Tx, int Ty, float* out,
                 void* ws, size_t ws_bytes, hipStream_t st);

int launch_attention(int dtype, const void* qkv, const float* mask, void* out, int B, int T, int heads,
                     hipStream_t stream, float* part = nullptr);
size_t attention_part_bytes(int B, int T, int heads);
// query-independent attention + out-projection + residual of utterances that ALL have padded frames at this
// level (the reference's mask fill, model.py:697; mt_attn.hip): x [B][T][256] bf16 updated in place to x + attn1(x),
// row_out [B*T][4][2] the per-slab (mean, M2) of the result; wqkv / bqkv the LN-folded QKV vconv image (mq = 384
// rows) and bias, wout / bout the out-projection image and bias; part: uniform_attention_floats(B) floats.
// Three launches: masked sums of the normalised rows over uniform_part_slices(T) frame slices per utterance; per
// utterance the merge and the two GEMVs (o_b); x += o_b with the row statistics over the same slices.
constexpr int UNI_PSMAX = 32;  // most masked-sum slices per utterance (the workspace holds B x 32 x 260 floats)
int uniform_part_slices(int T);
size_t uniform_attention_floats(int B);  // workspace of launch_uniform_attention's `part`: slice sums + o_b
// apply = false: the first two launches only; o_b ([B][256] floats) is left at uniform_attention_ovec(part, B) for a
// consumer that adds it itself (mt_ffn)
int launch_uniform_attention(void* x, const float* mask, int B, int T, const void* wqkv, int mq, const float* bqkv,
                             const void* wout, const float* bout, float* part, float* row_out, hipStream_t st,
                             bool apply = true);
const float* uniform_attention_ovec(const float* part, int B);

// the XCD-aligned block order of the decoder's streaming kernels (mt_common.h xcd_chunk; MT_XCD_TILES=0 turns it
// and mt_vconv's XCD-major tile walk off)
int xcd_remap_enabled();
// ... for a launch streaming `bytes` of activations: only while they fit the XCDs' L2 (the decoder at B = 32: CFM
// solve 8.70 -> 8.47 ms with mt_vconv's XCD-major walk; at B = 256 the round-robin order is faster)
inline int xcd_remap_for(size_t bytes) { return xcd_remap_enabled() && bytes <= (24u << 20) ? 1 : 0; }
}  // namespace mt
