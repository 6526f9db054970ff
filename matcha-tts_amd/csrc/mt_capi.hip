// C ABI (include/matcha_hip.h) over the decoder / vocoder drivers and the op kernels.
#include <string.h>

#include <new>

#include "../../include/matcha_hip.h"
#include "mt_ffn.h"
#include "mt_model.h"
#include "mt_vconv.h"
#include "mt_vpair.h"
#include "mt_probe.h"
#include "mt_train.h"

namespace mt {
const char* last_error();
int denoise(const float* audio, int B, int L, const float* bias_spec, float strength, float* out, void* ws,
            size_t ws_bytes, hipStream_t st, const int* lens = nullptr, int lmul = 1);
size_t denoise_workspace_bytes(int B, int L);
// timing-experiment macros each kernel file was built with (0 in a production build)
int vconv_exp_flags();
int rbconv_exp_flags();
int ffn_exp_flags();
int vpair_exp_flags();
int stft_magnitude(const float* audio, int B, int L, float* mag, hipStream_t st);
int log_mel(const float* audio, int B, int L, const float* basis, float mean, float stdv, float* mel, hipStream_t st);
}  // namespace mt

struct mt_encoder {
  mt::Encoder e;
};
struct mt_decoder {
  mt::Decoder d;
};
struct mt_vocoder {
  mt::Vocoder v;
};

using mt::set_error;

static int param_name(const mt::ParamList& L, int i, char* buf, int buflen) {
  MT_REQUIRE(i >= 0 && i < (int)L.names.size(), "param index %d out of range", i);
  MT_REQUIRE(buf && buflen > (int)L.names[i].size(), "param name buffer too small");
  memcpy(buf, L.names[i].c_str(), L.names[i].size() + 1);
  return 0;
}
static int param_shape(const mt::ParamList& L, int i, int64_t* shape, int maxdim) {
  MT_REQUIRE(i >= 0 && i < (int)L.names.size(), "param index %d out of range", i);
  const auto& s = L.shapes[i];
  MT_REQUIRE((int)s.size() <= maxdim, "shape buffer too small");
  for (size_t k = 0; k < s.size(); ++k) shape[k] = s[k];
  return (int)s.size();
}

extern "C" {

const char* mt_last_error(void) { return mt::last_error(); }
int mt_abi_version(void) { return 1; }
int mt_vpair_set_kernels(int mask) { return mt::vpair_set_kernels(mask); }
int mt_vocoder_set_post_fold(int enable) { return mt::vocoder_set_post_fold(enable); }
int mt_sched_count(void) { return mt::sched_count(); }
int mt_sched_get(int i, int* rec, int* wait, int* wait_first, int cap) {
  MT_REQUIRE(rec && wait && wait_first, "null buffer");
  const int S = mt::sched_get(i, rec, wait, wait_first, cap);
  MT_REQUIRE(S >= 0, "schedule %d: out of range or cap %d too small", i, cap);
  return S;
}
int mt_build_experiments(void) {
  // bit 0: mt_vconv (VCONV_EXP / VCONV_TS), 1: mt_rbconv (RB_EXP), 2: mt_ffn (FFN_EXP), 3: the pair kernels (VPAIR_EXP)
  return (mt::vconv_exp_flags() ? 1 : 0) | (mt::rbconv_exp_flags() ? 2 : 0) | (mt::ffn_exp_flags() ? 4 : 0) |
         (mt::vpair_exp_flags() ? 8 : 0);
}

// ---- decoder ----
int mt_encoder_create(int n_vocab, int n_channels, int filter_channels, int n_heads, int n_layers, int kernel_size,
                      int n_spks, int spk_emb_dim, int dp_filter_channels, int dp_kernel_size, int prenet, int dtype,
                      mt_encoder** out) {
  MT_REQUIRE(out, "null out");
  mt_encoder* h = new (std::nothrow) mt_encoder();
  MT_REQUIRE(h, "out of host memory");
  int rc = h->e.init(n_vocab, n_channels, filter_channels, n_heads, n_layers, kernel_size, n_spks, spk_emb_dim,
                     dp_filter_channels, dp_kernel_size, prenet, dtype);
  if (rc) {
    delete h;
    return rc;
  }
  *out = h;
  return 0;
}
void mt_encoder_destroy(mt_encoder* e) { delete e; }
int mt_encoder_num_params(const mt_encoder* e) { return e ? (int)e->e.params.names.size() : -1; }
int mt_encoder_param_name(const mt_encoder* e, int i, char* buf, int buflen) {
  MT_REQUIRE(e, "null encoder");
  return param_name(e->e.params, i, buf, buflen);
}
int mt_encoder_param_shape(const mt_encoder* e, int i, int64_t* shape, int maxdim) {
  MT_REQUIRE(e, "null encoder");
  return param_shape(e->e.params, i, shape, maxdim);
}
size_t mt_encoder_packed_bytes(const mt_encoder* e) { return e ? e->e.packed_bytes : 0; }
int mt_encoder_pack(const mt_encoder* e, const float* const* params, void* packed, void* stream) {
  MT_REQUIRE(e && params && packed, "encoder_pack: null argument");
  return e->e.pack(params, packed, (hipStream_t)stream);
}
size_t mt_encoder_workspace_bytes(const mt_encoder* e, int B, int Tx) { return e ? e->e.workspace_bytes(B, Tx) : 0; }
int mt_encoder_set_mfma_attention(mt_encoder* e, int enable) {
  MT_REQUIRE(e, "null encoder");
  e->e.mfma_attn = enable ? 1 : 0;
  return 0;
}
int mt_encoder_set_vconv(mt_encoder* e, int enable) {
  MT_REQUIRE(e, "null encoder");
  e->e.f32vc = enable ? 1 : 0;
  return 0;
}
int mt_encoder_set_split(mt_encoder* e, int enable) {
  MT_REQUIRE(e, "null encoder");
  MT_REQUIRE(!enable || e->e.dtype == mt::F32, "encoder_set_split: the split-bf16 FFN is an fp32-encoder mode");
  e->e.split = enable ? 1 : 0;
  return 0;
}
int mt_encoder_forward(const mt_encoder* e, const void* packed, const int64_t* x, const int64_t* x_lengths,
                       const float* spks, int B, int Tx, float* mu, float* logw, float* x_mask, int32_t* oov,
                       void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(e && packed, "encoder_forward: null argument");
  return e->e.forward(packed, (const long long*)x, (const long long*)x_lengths, spks, B, Tx, mu, logw, x_mask, oov, ws,
                      ws_bytes, (hipStream_t)stream);
}

int mt_decoder_create(int c_cond, int n_mid, int n_blocks, int heads, int dtype, mt_decoder** out) {
  MT_REQUIRE(out, "null out");
  mt_decoder* h = new (std::nothrow) mt_decoder();
  MT_REQUIRE(h, "out of host memory");
  int rc = h->d.init(c_cond, n_mid, n_blocks, heads, dtype);
  if (rc) {
    delete h;
    return rc;
  }
  *out = h;
  return 0;
}
void mt_decoder_destroy(mt_decoder* d) { delete d; }
int mt_decoder_num_params(const mt_decoder* d) { return d ? (int)d->d.params.names.size() : -1; }
int mt_decoder_param_name(const mt_decoder* d, int i, char* buf, int buflen) {
  MT_REQUIRE(d, "null decoder");
  return param_name(d->d.params, i, buf, buflen);
}
int mt_decoder_param_shape(const mt_decoder* d, int i, int64_t* shape, int maxdim) {
  MT_REQUIRE(d, "null decoder");
  return param_shape(d->d.params, i, shape, maxdim);
}
int mt_decoder_set_vconv(mt_decoder* d, int enable) {
  MT_REQUIRE(d, "null decoder");
  MT_REQUIRE(enable >= 0 && enable <= 2, "decoder_set_vconv: mode %d", enable);
  d->d.vconv = enable ? 1 : 0;
  d->d.gnres = enable == 1 ? 1 : 0;
  return 0;
}
size_t mt_decoder_packed_bytes(const mt_decoder* d) { return d ? d->d.packed_bytes : 0; }
int mt_decoder_pack(const mt_decoder* d, const float* const* params, void* packed, void* stream) {
  MT_REQUIRE(d && params && packed, "decoder_pack: null argument");
  return d->d.pack(params, packed, (hipStream_t)stream);
}
size_t mt_cfm_workspace_bytes(const mt_decoder* d, int B, int T, int n_timesteps, int solver) {
  if (!d) return 0;
  return d->d.workspace_bytes(B, T, solver == 1 ? 2 * n_timesteps : n_timesteps);
}
int mt_cfm_solve(const mt_decoder* d, const void* packed, const float* z_noise, float temperature,
                 const float* mu_y, const float* mask, const float* spks, int B, int T, int n_timesteps,
                 int solver, float* z_out, void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(d && packed && z_noise && mu_y && mask && z_out && ws, "cfm_solve: null argument");
  return d->d.solve(packed, z_noise, temperature, mu_y, mask, spks, B, T, n_timesteps, solver, z_out, ws,
                    ws_bytes, (hipStream_t)stream);
}
int mt_cfm_solve_bounded(const mt_decoder* d, const void* packed, const float* z_noise, float temperature,
                         const float* mu_y, const float* mask, const float* spks, int B, int T, int max_valid,
                         int n_timesteps, int solver, float* z_out, void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(d && packed && z_noise && mu_y && mask && z_out && ws, "cfm_solve: null argument");
  return d->d.solve(packed, z_noise, temperature, mu_y, mask, spks, B, T, n_timesteps, solver, z_out, ws,
                    ws_bytes, (hipStream_t)stream, max_valid);
}
int mt_decoder_set_uniform_attention(mt_decoder* d, int enable) {
  MT_REQUIRE(d, "null decoder");
  d->d.uniform_attn = enable ? 1 : 0;
  return 0;
}
int mt_decoder_set_graphs(mt_decoder* d, int enable) {
  MT_REQUIRE(d, "null decoder");
  d->d.graphs = enable ? 1 : 0;
  return 0;
}
int mt_decoder_set_taps(mt_decoder* d, float* const* taps, int n) {
  MT_REQUIRE(d, "null decoder");
  MT_REQUIRE(n >= 0 && n <= mt::Decoder::N_TAPS, "decoder_set_taps: %d taps (at most %d)", n, mt::Decoder::N_TAPS);
  for (int i = 0; i < mt::Decoder::N_TAPS; ++i) d->d.taps[i] = (taps && i < n) ? taps[i] : nullptr;
  return 0;
}
size_t mt_decoder_step_workspace_bytes(const mt_decoder* d, int B, int T) {
  return d ? d->d.workspace_bytes(B, T, 1) : 0;
}
int mt_decoder_step(const mt_decoder* d, const void* packed, const float* x, const float* mu_y,
                    const float* mask, const float* spks, float t, int B, int T, float* out, void* ws,
                    size_t ws_bytes, void* stream) {
  MT_REQUIRE(d && packed && x && mu_y && mask && out && ws, "decoder_step: null argument");
  return d->d.step(packed, x, mu_y, mask, spks, t, B, T, out, ws, ws_bytes, (hipStream_t)stream);
}

size_t mt_decoder_step_times_workspace_bytes(const mt_decoder* d, int B, int T) {
  return d ? d->d.workspace_bytes(B, T, B) : 0;
}
int mt_decoder_step_times(const mt_decoder* d, const void* packed, const float* x, const float* mu_y,
                          const float* mask, const float* spks, const float* t, int B, int T, float* out, void* ws,
                          size_t ws_bytes, void* stream) {
  MT_REQUIRE(d && packed && x && mu_y && mask && t && out && ws, "decoder_step_times: null argument");
  return d->d.step_times(packed, x, mu_y, mask, spks, t, B, T, out, ws, ws_bytes, (hipStream_t)stream);
}

// ---- vocoder ----
int mt_vocoder_create(int resblock, int n_ups, const int* up_rates, const int* up_kernels, int up_init,
                      int n_kernels, const int* rb_kernels, int n_dils, const int* rb_dils, int dtype,
                      mt_vocoder** out) {
  MT_REQUIRE(out && up_rates && up_kernels && rb_kernels && rb_dils && n_ups > 0 && n_kernels > 0 &&
                 n_dils > 0,
             "vocoder_create: bad arguments");
  std::vector<int> ur(up_rates, up_rates + n_ups), uk(up_kernels, up_kernels + n_ups);
  std::vector<int> rk(rb_kernels, rb_kernels + n_kernels);
  std::vector<std::vector<int>> rd;
  for (int j = 0; j < n_kernels; ++j) rd.emplace_back(rb_dils + j * n_dils, rb_dils + (j + 1) * n_dils);
  mt_vocoder* h = new (std::nothrow) mt_vocoder();
  MT_REQUIRE(h, "out of host memory");
  int rc = h->v.init(resblock, ur, uk, up_init, rk, rd, dtype);
  if (rc) {
    delete h;
    return rc;
  }
  *out = h;
  return 0;
}
void mt_vocoder_destroy(mt_vocoder* v) { delete v; }
int mt_vocoder_num_params(const mt_vocoder* v) { return v ? (int)v->v.params.names.size() : -1; }
int mt_vocoder_param_name(const mt_vocoder* v, int i, char* buf, int buflen) {
  MT_REQUIRE(v, "null vocoder");
  return param_name(v->v.params, i, buf, buflen);
}
int mt_vocoder_param_shape(const mt_vocoder* v, int i, int64_t* shape, int maxdim) {
  MT_REQUIRE(v, "null vocoder");
  return param_shape(v->v.params, i, shape, maxdim);
}
int mt_vocoder_set_fusion(mt_vocoder* v, int enable) {
  MT_REQUIRE(v, "null vocoder");
  v->v.fuse = enable ? 1 : 0;
  return 0;
}
int mt_vocoder_set_vconv(mt_vocoder* v, int enable) {
  MT_REQUIRE(v, "null vocoder");
  v->v.vconv = enable < 0 ? 0 : enable;
  return 0;
}
int mt_vocoder_set_pair(mt_vocoder* v, int enable) {
  MT_REQUIRE(v, "null vocoder");
  v->v.pair = enable < 0 ? 0 : enable;
  return 0;
}
size_t mt_vocoder_packed_bytes(const mt_vocoder* v) { return v ? v->v.packed_bytes : 0; }
int mt_vocoder_pack(const mt_vocoder* v, const float* const* params, void* packed, void* stream) {
  MT_REQUIRE(v && params && packed, "vocoder_pack: null argument");
  return v->v.pack(params, packed, (hipStream_t)stream);
}
size_t mt_vocoder_workspace_bytes(const mt_vocoder* v, int B, int T) {
  return v ? v->v.workspace_bytes(B, T) : 0;
}
int mt_vocoder_forward(const mt_vocoder* v, const void* packed, const float* mel, int B, int T, float* wav,
                       void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(v && packed && mel && wav && ws, "vocoder_forward: null argument");
  return v->v.forward(packed, mel, B, T, wav, ws, ws_bytes, (hipStream_t)stream);
}

int mt_vocoder_ragged_supported(const mt_vocoder* v) { return v && v->v.ragged_supported() ? 1 : 0; }

int mt_vocoder_forward_ragged(const mt_vocoder* v, const void* packed, const float* mel, int B, int T,
                              const int32_t* lens, float* wav, void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(v && packed && mel && lens && wav && ws, "vocoder_forward_ragged: null argument");
  return v->v.forward(packed, mel, B, T, wav, ws, ws_bytes, (hipStream_t)stream, lens);
}

// ---- index path ----
int mt_durations(const float* logw, const float* x_mask, float length_scale, int B, int Tx, float* w_ceil,
                 float* cum, int64_t* y_lengths, void* stream) {
  MT_REQUIRE(logw && x_mask && w_ceil && cum && y_lengths, "durations: null argument");
  return mt::durations(logw, x_mask, length_scale, B, Tx, w_ceil, cum, (long long*)y_lengths,
                       (hipStream_t)stream);
}
int mt_alignment(const float* cum, const int64_t* y_lengths, int B, int Tx, int T, const float* mu, int C,
                 float* attn, float* mu_y, float* y_mask, void* stream) {
  MT_REQUIRE(cum && (mu || !mu_y) && (y_lengths || !y_mask), "alignment: null argument");
  return mt::alignment(cum, (const long long*)y_lengths, B, Tx, T, mu, C, attn, mu_y, y_mask,
                       (hipStream_t)stream);
}
int mt_denorm_crop(const float* z, const float* mean, const float* stdv, int B, int C, int T, int Ty,
                   float* mel, void* stream) {
  MT_REQUIRE(z && mean && stdv && mel, "denorm_crop: null argument");
  return mt::denorm_crop(z, mean, stdv, B, C, T, Ty, mel, (hipStream_t)stream);
}

// ---- denoiser ----
size_t mt_denoise_workspace_bytes(int B, int L) { return mt::denoise_workspace_bytes(B, L); }
int mt_denoise(const float* audio, int B, int L, const float* bias_spec, float strength, float* out, void* ws,
               size_t ws_bytes, void* stream) {
  MT_REQUIRE(audio && bias_spec && out, "denoise: null argument");
  return mt::denoise(audio, B, L, bias_spec, strength, out, ws, ws_bytes, (hipStream_t)stream);
}

int mt_denoise_ragged(const float* audio, int B, int L, const int32_t* lens, int lmul, const float* bias_spec,
                      float strength, float* out, void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(audio && lens && bias_spec && out, "denoise_ragged: null argument");
  return mt::denoise(audio, B, L, bias_spec, strength, out, ws, ws_bytes, (hipStream_t)stream, lens, lmul);
}

size_t mt_maximum_path_workspace_bytes(int B, int Tx, int Ty) { return mt::mas_workspace_bytes(B, Tx, Ty); }
int mt_maximum_path(const float* neg_cent, const int32_t* t_xs, const int32_t* t_ys, int B, int Tx, int Ty,
                    float* paths, void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(neg_cent && t_xs && t_ys && paths, "maximum_path: null argument");
  return mt::maximum_path(neg_cent, t_xs, t_ys, B, Tx, Ty, paths, ws, ws_bytes, (hipStream_t)stream);
}

int mt_stft_magnitude(const float* audio, int B, int L, float* mag, void* stream) {
  MT_REQUIRE(audio && mag, "stft_magnitude: null argument");
  return mt::stft_magnitude(audio, B, L, mag, (hipStream_t)stream);
}

int mt_log_mel(const float* audio, int B, int L, const float* mel_basis, float mel_mean, float mel_std, float* mel,
               void* stream) {
  MT_REQUIRE(audio && mel_basis && mel, "log_mel: null argument");
  return mt::log_mel(audio, B, L, mel_basis, mel_mean, mel_std, mel, (hipStream_t)stream);
}

// ---- op level ----
size_t mt_op_conv1d_workspace_bytes(int dtype, int cin, int cout, int k, int stride, int transposed) {
  mt::Packer pk;
  const int es = dtype == MT_DTYPE_BF16 ? 2 : 4;
  if (transposed)
    mt::make_convT(cin, cout, k, stride, 0, 0, 1, es, pk);
  else
    mt::make_conv(cout, cin, k, stride, 0, 1, {0}, 1, es, pk);
  return pk.off;
}
int mt_op_conv1d_tile(int variant, int dtype, const void* x, int B, int Tin, int cin, const float* W, const float* bias,
                 int cout, int k, int stride, int pad, int dil, int transposed, float slope, void* y, int Tout,
                 void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(x && W && y && ws, "op_conv1d: null argument");
  hipStream_t st = (hipStream_t)stream;
  const int es = dtype == MT_DTYPE_BF16 ? 2 : 4;
  mt::Packer pk;
  mt::GemmW g = transposed ? mt::make_convT(cin, cout, k, stride, pad, 0, bias ? 1 : -1, es, pk)
                           : mt::make_conv(cout, cin, k, stride, pad, dil, {0}, bias ? 1 : -1, es, pk);
  MT_REQUIRE(ws_bytes >= pk.off, "op_conv1d: workspace %zu < %zu", ws_bytes, pk.off);
  const float* params[2] = {W, bias};
  const bool reuse = variant >= 0x1000 - 1;  // variant + 0x1000: weights already packed in ws (timing)
  if (reuse) variant -= 0x1000;
  if (!reuse) {
    int rc = mt::pack_gemm(g, dtype, params, (char*)ws, st);
    if (rc) return rc;
  }
  mt::ConvArgs a = mt::gemm_args(g, (const char*)ws, B, Tin);
  MT_REQUIRE(a.Tout == Tout, "op_conv1d: Tout %d != expected %d", Tout, a.Tout);
  a.x0 = x;
  a.y = y;
  a.slope = slope;
  return mt::launch_conv_op(dtype, slope >= 0.f ? mt::PF_LRELU : 0, a, st, variant);
}
int mt_op_conv1d(int dtype, const void* x, int B, int Tin, int cin, const float* W, const float* bias,
                 int cout, int k, int stride, int pad, int dil, int transposed, float slope, void* y, int Tout,
                 void* ws, size_t ws_bytes, void* stream) {
  return mt_op_conv1d_tile(-1, dtype, x, B, Tin, cin, W, bias, cout, k, stride, pad, dil, transposed, slope, y,
                           Tout, ws, ws_bytes, stream);
}
size_t mt_op_vconv_workspace_bytes(int cin, int cout, int k) {
  mt::Packer pk;
  mt::GemmW g = mt::make_conv(cout, cin, k, 1, 0, 1, {0}, 1, 2, pk);
  pk.take(mt::vconv_packed_bytes(cin, cout, k));
  pk.take(256);
  pk.take(4096);
  (void)g;
  return pk.off;
}
int mt_vconv_set_rbconv(int enable) { return mt::rbconv_set(enable); }
int mt_vconv_set_ct(int enable) { return mt::vconv_set_ct(enable); }
int mt_ffn_set(int enable) { return mt::ffn_set(enable); }
int mt_vconv_set_actin(int enable) { return mt::rbconv_actin_set(enable); }
int mt_ffn_set_min_frames(int frames) { return mt::ffn_set_min_frames(frames); }
int mt_decoder_set_kernels(int mask) { return mt::dec_set_kernels(mask); }
int mt_op_vconv(const void* x, int B, int L, int cin, const float* W, const float* bias, int cout, int k, int dil,
                int ef, const void* resid, void* y, void* y2, float slope, float div, const int32_t* lens, int pack,
                void* ws, size_t ws_bytes, void* stream) {
  MT_REQUIRE(x && W && bias && y && ws, "op_vconv: null argument");
  MT_REQUIRE(mt::vconv_supported(cin, cout, k, dil, 1), "op_vconv: unsupported conv %dx%d k%d d%d", cin, cout, k, dil);
  hipStream_t st = (hipStream_t)stream;
  mt::Packer pk;
  mt::GemmW g = mt::make_conv(cout, cin, k, 1, dil * (k - 1) / 2, dil, {0}, 1, 2, pk);
  const size_t v_off = pk.take(mt::vconv_packed_bytes(cin, cout, k));
  const size_t z_off = pk.take(256);
  const size_t t_off = pk.take(4096);
  MT_REQUIRE(ws_bytes >= pk.off, "op_vconv: workspace %zu < %zu", ws_bytes, pk.off);
  const float* params[2] = {W, bias};
  char* P = (char*)ws;
  int rc;
  if (pack) {
    if ((rc = mt::pack_gemm(g, MT_DTYPE_BF16, params, P, st))) return rc;
    if ((rc = mt::vconv_repack(P + g.w_off, g.Mpad, g.taps, g.cin_pad, cin, cout, P + v_off, st))) return rc;
    if ((rc = mt::pack_vec(nullptr, 1, 64, 0, (float*)(P + z_off), st))) return rc;
  }
  mt::VConvArgs a{};
  a.x = (const mt::bf16*)x;
  a.B = B;
  a.L = L;
  a.cin = cin;
  a.w = (const mt::bf16*)(P + v_off);
  a.bias = (const float*)(P + g.b_off);
  a.M = a.Mpad = cout;
  a.taps = k;
  a.dil = dil;
  a.pad = g.pad;
  a.y = (mt::bf16*)y;
  a.y2 = (mt::bf16*)y2;
  a.resid = (const mt::bf16*)resid;
  a.slope = slope;
  a.div = div;
  a.zero = (const mt::bf16*)(P + z_off);
  a.trash = (mt::bf16*)(P + t_off);
  a.lens = (const int*)lens;
  a.lmul = 1;
  return mt::launch_vconv(ef, a, st);
}
int mt_op_attention(int dtype, const void* qkv, const float* mask, void* out, int B, int T, int heads,
                    void* stream) {
  MT_REQUIRE(qkv && mask && out, "op_attention: null argument");
  return mt::launch_attention(dtype, qkv, mask, out, B, T, heads, (hipStream_t)stream);
}

int mt_probe_start(int site, int max_launches) { return mt::probe_start(site, max_launches); }
int mt_probe_pause(int paused) { return mt::probe_pause(paused != 0); }
int mt_probe_detail(int cap, double* ms, double* flops, double* bytes, int* tags) {
  return mt::probe_detail(cap, ms, flops, bytes, tags);
}

int mt_probe_stop(int* launches, double* total_ms, double* flops, double* bytes, double peak_flops, double peak_bw,
                  double* roof_ms) {
  return mt::probe_stop(launches, total_ms, flops, bytes, peak_flops, peak_bw, roof_ms);
}

// ---- training-step primitives (fp32) ----
int mtt_gemm(int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda, long long sA,
             const float* B, int ldb, long long sB, float beta, float* C, int ldc, long long sC, int batch,
             const float* bias, const float* row_mask, float* ws, size_t ws_bytes, void* stream) {
  return mtt_gemm_ex(0, transA, transB, M, N, K, alpha, A, lda, sA, B, ldb, sB, beta, C, ldc, sC, batch, bias,
                     row_mask, ws, ws_bytes, stream);
}
int mtt_gemm_ex(int opfmt, int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda,
                long long sA, const float* B, int ldb, long long sB, float beta, float* C, int ldc, long long sC,
                int batch, const float* bias, const float* row_mask, float* ws, size_t ws_bytes, void* stream) {
  mt::GemmF32 g{transA, transB, M, N, K, alpha, beta, A, lda, sA, B, ldb, sB, C, ldc, sC, batch, bias, row_mask, ws,
                ws_bytes / sizeof(float), opfmt};
  return mt::gemm_f32(g, (hipStream_t)stream);
}
size_t mtt_gemm_workspace_bytes(int M, int N, int K, int batch) {
  return mt::gemm_f32_workspace_floats(M, N, K, batch) * sizeof(float);
}
int mtt_im2col(const float* x, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
               float* cols, void* stream) {
  return mt::im2col(x, mask, B, T, C, k, stride, pad, dil, Tout, cols, (hipStream_t)stream);
}
int mtt_col2im(const float* dcols, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil,
               int Tout, float* dx, int accumulate, void* stream) {
  return mt::col2im(dcols, mask, B, T, C, k, stride, pad, dil, Tout, dx, accumulate, (hipStream_t)stream);
}
int mtt_ew(int op, size_t n, const float* a, const float* b, const float* c, float* out, float alpha, float beta,
           size_t d0, size_t m0, size_t s0, size_t d1, size_t m1, size_t s1, int accumulate, void* stream) {
  mt::EwArgs e{op, n, a, b, c, out, alpha, beta, d0, m0, s0, d1, m1, s1, accumulate};
  return mt::ew(e, (hipStream_t)stream);
}
int mtt_copy_cols(const float* src, int lds, int soff, float* dst, int ldd, int doff, int rows, int n, int accumulate,
                  void* stream) {
  return mt::copy_cols(src, lds, soff, dst, ldd, doff, rows, n, accumulate, (hipStream_t)stream);
}
int mtt_seq_mask(const int64_t* lengths, int B, int T, float* out, void* stream) {
  return mt::seq_mask((const long long*)lengths, B, T, out, (hipStream_t)stream);
}
size_t mtt_colsum_scratch_floats(int rows, int C, int seg) { return mt::colsum_scratch_floats(rows, C, seg); }
int mtt_colsum(const float* a, const float* b, int rows, int C, int seg, float* out, int accumulate, float* scratch,
               void* stream) {
  return mt::colsum(a, b, rows, C, seg, out, accumulate, scratch, (hipStream_t)stream);
}
int mtt_sum(const float* a, const float* b, size_t n, float* out, float* scratch, void* stream) {
  return mt::sum_all(a, b, n, out, scratch, (hipStream_t)stream);
}
int mtt_dropout(const float* a, size_t n, float p, unsigned seed, float* out, void* stream) {
  return mt::dropout(a, n, p, seed, out, (hipStream_t)stream);
}
int mtt_groupnorm_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, int G, float eps,
                      float* y, float* mean, float* rstd, void* stream) {
  return mt::groupnorm_fwd(x, gamma, beta, B, T, C, G, eps, y, mean, rstd, (hipStream_t)stream);
}
int mtt_groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int B,
                      int T, int C, int G, float* dx, float* dgamma_part, float* dbeta_part, void* stream) {
  return mt::groupnorm_bwd(dy, x, gamma, mean, rstd, B, T, C, G, dx, dgamma_part, dbeta_part, (hipStream_t)stream);
}
int mtt_layernorm_fwd(const float* x, const float* gamma, const float* beta, int rows, int C, float eps, float* y,
                      float* mean, float* rstd, void* stream) {
  return mt::layernorm_fwd(x, gamma, beta, rows, C, eps, y, mean, rstd, (hipStream_t)stream);
}
int mtt_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                      int rows, int C, float* dx, void* stream) {
  return mt::layernorm_bwd(dy, x, gamma, mean, rstd, rows, C, dx, (hipStream_t)stream);
}
int mtt_snake_fwd(const float* x, const float* log_alpha, const float* log_beta, size_t n, int C, float* y,
                  void* stream) {
  return mt::snake_fwd(x, log_alpha, log_beta, n, C, y, (hipStream_t)stream);
}
int mtt_snake_bwd(const float* x, const float* log_alpha, const float* log_beta, const float* dy, size_t n, int C,
                  float* dx, float* galpha, float* gbeta, void* stream) {
  return mt::snake_bwd(x, log_alpha, log_beta, dy, n, C, dx, galpha, gbeta, (hipStream_t)stream);
}
int mtt_softmax_fwd(const float* s, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk, float scale,
                    int mode, float* p, void* stream) {
  return mt::softmax_fwd(s, kmask, qmask, BH, H, Tq, Tk, scale, mode, p, (hipStream_t)stream);
}
int mtt_softmax_bwd(const float* p, const float* dp, const float* kmask, const float* qmask, int BH, int H, int Tq,
                    int Tk, float scale, float* ds, void* stream) {
  return mt::softmax_bwd(p, dp, kmask, qmask, BH, H, Tq, Tk, scale, ds, (hipStream_t)stream);
}
int mtt_rope(float* x, int B, int T, int H, int dh, int d, const float* theta, int inverse, void* stream) {
  return mt::rope(x, B, T, H, dh, d, theta, inverse, (hipStream_t)stream);
}
int mtt_embed_fwd(const int64_t* ids, size_t ntok, const float* table, int C, float scale, float* out, void* stream) {
  return mt::embed_fwd((const long long*)ids, ntok, table, C, scale, out, (hipStream_t)stream);
}
int mtt_embed_bwd(const int64_t* ids, size_t ntok, const float* dout, int V, int C, float scale, float* dtable,
                  void* stream) {
  return mt::embed_bwd((const long long*)ids, ntok, dout, V, C, scale, dtable, (hipStream_t)stream);
}
int mtt_adam(float* p, const float* g, float* m, float* v, size_t n, const float* gscale, float lr, float beta1,
             float beta2, float eps, int step, void* stream) {
  return mt::adam_step(p, g, m, v, n, gscale, lr, beta1, beta2, eps, step, (hipStream_t)stream);
}
int mtt_clip_factor(const float* sumsq, float max_norm, float inv_world, float* out, float* norm_out, void* stream) {
  return mt::clip_factor(sumsq, max_norm, inv_world, out, norm_out, (hipStream_t)stream);
}
int mtt_unscale(float* g, size_t n, float inv_scale, float* found, float* scratch, void* stream) {
  return mt::unscale_found_inf(g, n, inv_scale, found, scratch, (hipStream_t)stream);
}

int mt_vconv_log_start(int capacity) { return mt::vclog_start(capacity); }
int mt_vconv_log_stop(int32_t* records, int capacity) { return mt::vclog_stop(records, capacity); }

}  // extern "C"
