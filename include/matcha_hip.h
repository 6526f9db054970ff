/*
 * matcha_hip.h — C ABI of the MI355X-native (gfx950) Matcha-TTS synthesis path.
 *
 * The reference (Lounes78/matcha-tts) has no native code and no FFI: its hot path is the
 * PyTorch module call surface that main.py uses. Each entry point below replaces the ATen
 * work under one of those calls (reference file:line in /root/reference):
 *
 *   mt_durations + mt_alignment  <- MatchaTTS.synthesize duration/index path  model.py:1273-1289
 *                                   (sequence_mask :42-46, generate_path :64-76)
 *   mt_cfm_solve                 <- CFM.forward / BASECFM.forward Euler|midpoint loop
 *                                   model.py:1084-1109, 1136-1145, estimator Decoder.forward :964-1048
 *   mt_decoder_step              <- one Decoder.forward (estimator) call  model.py:964-1048
 *   mt_denorm_crop               <- denormalize + crop  model.py:106-125, 1295-1298
 *   mt_vocoder_forward           <- hifigan.models.Generator.forward  hifigan/models.py:181-197
 *   mt_denoise                   <- hifigan.denoiser.Denoiser.forward hifigan/denoiser.py:62-68
 *   mt_vocoder_forward_ragged,   <- the reference pipeline's per-utterance vocoder + denoiser calls (one utterance
 *   mt_denoise_ragged               per call, mel cropped to its y_length: main.py:181-198,
 *                                   MOS_audiou_generator.ipynb:265-277) for a whole padded batch in one launch chain
 *   mt_maximum_path              <- train_standalone.maximum_path train_standalone.py:280-325 (MAS)
 *
 * Conventions
 *  - Every pointer argument is DEVICE memory owned by the caller (PyTorch), except the
 *    host-side handles and name/shape buffers. The library never allocates device memory
 *    and keeps no global device state.
 *  - `stream` is a hipStream_t passed as void*; all work is enqueued on it, asynchronously.
 *  - Tensors use the reference layouts at the boundary: mel/mu/z [B][80][T] fp32, masks
 *    [B][1][T] fp32 (0/1), wav [B][1][L] fp32. Internally activations are [B][T][C].
 *  - Return 0 on success; a negative value on error, with a message in mt_last_error()
 *    (thread-local).
 *  - dtype selects the arithmetic of the conv/GEMM/attention kernels: MT_DTYPE_F32 (exact fp32
 *    MFMA, parity mode) or MT_DTYPE_BF16 (bf16 MFMA, fp32 accumulate, perf mode). Norm
 *    statistics, the time-embedding MLP and the ODE state are always fp32.
 */
#ifndef MATCHA_HIP_H
#define MATCHA_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MT_DTYPE_F32 0
#define MT_DTYPE_BF16 1
#define MT_SOLVER_EULER 0
#define MT_SOLVER_MIDPOINT 1

const char* mt_last_error(void);
int mt_abi_version(void);
/* Nonzero when this library is a timing-experiment build (tools/exp_build.sh), whose kernels drop work and
 * compute WRONG results: bit 0 mt_vconv (VCONV_EXP, or the VCONV_TS diagnostic build), 1 mt_rbconv (RB_EXP),
 * 2 mt_ffn (FFN_EXP), 3 the pair kernels (VPAIR_EXP). A production build returns 0; smoke() and bench.py refuse
 * anything else. */
int mt_build_experiments(void);
/* The compile-time K-loop schedules this library instantiates (mt_vconv's CT loops and mt_rbconv; test support for
 * tests/test_vcsched.py, host only): mt_sched_count() records; mt_sched_get(i, rec[11], wait, wait_first, cap) fills
 * rec = {family, NCH, TAPS, NW, NXB, TX, WPW, XPW, NST, RL, prologue wait} and the vmcnt counts the kernel waits with
 * at the top of steps s = -1 .. S-1 (entries 0 .. S; wait_first: the first tile's), returns S (negative: error). */
int mt_sched_count(void);
int mt_sched_get(int i, int* rec, int* wait, int* wait_first, int cap);

/* ---------------------------------------------------------------------------------------
 * Text encoder + duration predictor (TextEncoder.forward, model.py:517-535; Encoder :428-439,
 * RoPE MultiHeadAttention :294-364, ConvReluNorm prenet :171-208, DurationPredictor :210-229).
 * Replaces the host PyTorch encoder that MatchaTTS.synthesize (model.py:1273) calls.
 * Parameters are named relative to the TextEncoder module ("emb.weight",
 * "encoder.attn_layers.0.conv_q.weight", "proj_w.norm_1.gamma", ...); "_rope_theta" is the fp32
 * table 1/10000^(arange(0, d, 2)/d), d = int(head_dim * 0.5), of model.py:258-265.
 * forward: x int64 [B][Tx] token ids, x_lengths int64 [B], spks fp32 [B][spk_emb_dim] (n_spks > 1)
 * -> mu fp32 [B][80][Tx], logw fp32 [B][1][Tx], x_mask fp32 [B][1][Tx].
 * ------------------------------------------------------------------------------------- */
typedef struct mt_encoder mt_encoder;
int mt_encoder_create(int n_vocab, int n_channels, int filter_channels, int n_heads, int n_layers, int kernel_size,
                      int n_spks, int spk_emb_dim, int dp_filter_channels, int dp_kernel_size, int prenet, int dtype,
                      mt_encoder** out);
void mt_encoder_destroy(mt_encoder* e);
int mt_encoder_num_params(const mt_encoder* e);
int mt_encoder_param_name(const mt_encoder* e, int i, char* buf, int buflen);
int mt_encoder_param_shape(const mt_encoder* e, int i, int64_t* shape, int maxdim);
size_t mt_encoder_packed_bytes(const mt_encoder* e);
int mt_encoder_pack(const mt_encoder* e, const float* const* params, void* packed, void* stream);
size_t mt_encoder_workspace_bytes(const mt_encoder* e, int B, int Tx);
/* 96-dim heads: the self-attention core on MFMA (1, default; bf16: probabilities enter P.V as bf16; fp32: exact-fp32
 * v_mfma_f32_16x16x4_f32 throughout) or on the fp32-VALU kernel (0). */
int mt_encoder_set_mfma_attention(mt_encoder* e, int enable);
/* fp32: 1 (default) runs the prenet / attention-projection / FFN / duration-predictor convs on mt_vconv's fp32 mode
 * (LDS-DMA staging, exact-fp32 MFMA); 0 = the generic implicit-GEMM kernel (A/B, tests). Same arithmetic. */
int mt_encoder_set_vconv(mt_encoder* e, int enable);
/* fp32 encoder: 1 runs the FFN convs (model.py:375-393; TextEncoder precision "fp32x3") in mt_vconv's split-bf16 mode:
 * every fp32 operand is the sum of three bf16 parts and each fp32 product the sum of the six bf16 MFMA products whose
 * parts reach 2^-16, accumulated in fp32 (the reference's fp32 to a few ulp, at 16x the fp32 MFMA rate per product);
 * 0 (default) = exact fp32 MFMA. Not a bf16 encoder: its logw stays within 1e-5 of the fp32 reference. */
int mt_encoder_set_split(mt_encoder* e, int enable);
/* oov (nullable, device int32): set to 0, then to 1 when any id of x (padding included) lies outside [0, n_vocab):
 * nn.Embedding's IndexError (model.py:522); the caller raises at its next host sync. The embedding reads a clamped
 * row for such an id, so the launch itself stays in bounds. */
int mt_encoder_forward(const mt_encoder* e, const void* packed, const int64_t* x, const int64_t* x_lengths,
                       const float* spks, int B, int Tx, float* mu, float* logw, float* x_mask, int32_t* oov,
                       void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * U-Net estimator + CFM solver. Hyper-parameters are those of main.py:67-76
 * (channels=(256,256), attention_head_dim=64); c_cond = 2*n_feats (+ spk_emb_dim).
 * ------------------------------------------------------------------------------------- */
typedef struct mt_decoder mt_decoder;
int mt_decoder_create(int c_cond, int n_mid_blocks, int n_blocks, int num_heads, int dtype,
                      mt_decoder** out);
void mt_decoder_destroy(mt_decoder* d);
/* Reference state_dict tensors the packer needs, in canonical order, named relative to the
 * estimator (e.g. "down_blocks.0.0.block1.block.0.weight"); "_sinus_freq" is the fp32
 * frequency table exp(arange(c_cond/2) * -ln(1e4)/(c_cond/2-1)) of model.py:757-759. */
int mt_decoder_num_params(const mt_decoder* d);
int mt_decoder_param_name(const mt_decoder* d, int i, char* buf, int buflen);
int mt_decoder_param_shape(const mt_decoder* d, int i, int64_t* shape, int maxdim); /* -> ndim */
/* bf16: 1 (default) runs the ResnetBlock1D convs, the stride-1 down/up convs and the final block
 * conv on the LDS-DMA persistent conv (mt_vconv; producers keep those inputs masked, block 1's
 * GroupNorm+Mish applied by a separate pass, block 2's inside the res conv's epilogue); 2 = the same with
 * block 2's GroupNorm+Mish as a separate pass too; 0 = generic conv kernel with the GN/mask prologues.
 * Same math as mt_decoder_step / mt_cfm_solve (model.py ResnetBlock1D, Block1D, Decoder.forward). */
int mt_decoder_set_vconv(mt_decoder* d, int enable);
size_t mt_decoder_packed_bytes(const mt_decoder* d);
/* params[i]: device fp32 tensor in reference layout for parameter i. */
int mt_decoder_pack(const mt_decoder* d, const float* const* params, void* packed, void* stream);

size_t mt_cfm_workspace_bytes(const mt_decoder* d, int B, int T, int n_timesteps, int solver);
/* z_noise: randn [B,80,T] (z = z_noise*temperature, model.py:1085); mu_y [B,80,T]; mask [B,1,T];
 * spks [B,spk_dim] or NULL; z_out [B,80,T] (may alias z_noise). T must be even. */
int mt_cfm_solve(const mt_decoder* d, const void* packed, const float* z_noise, float temperature,
                 const float* mu_y, const float* mask, const float* spks, int B, int T,
                 int n_timesteps, int solver, float* z_out, void* ws, size_t ws_bytes, void* stream);

/* The same solve with the caller's bound on valid frames: max_valid = the most mask = 1 frames of any utterance
 * (model.py:1278's y_max; 0 = unknown). When max_valid < T every utterance has padded frames at full resolution
 * (and at max_valid <= T - 2 also at half resolution, mask[:, ::2]); the reference then fills every masked key
 * with +3.4e38 (model.py:697), so each utterance's attention is the same row for all queries — the uniform
 * mean of its masked V rows — and those transformer blocks skip Q / K / the per-frame softmax and
 * out-projection (a masked mean + two GEMVs per utterance). Same results as mt_cfm_solve up to rounding. */
int mt_cfm_solve_bounded(const mt_decoder* d, const void* packed, const float* z_noise, float temperature,
                         const float* mu_y, const float* mask, const float* spks, int B, int T, int max_valid,
                         int n_timesteps, int solver, float* z_out, void* ws, size_t ws_bytes, void* stream);
/* 1 (default): mt_cfm_solve_bounded takes the query-independent attention path where max_valid allows it;
 * 0: always the general Q.K^T path (A/B, tests) */
int mt_decoder_set_uniform_attention(mt_decoder* d, int enable);
/* 1 (default): mt_cfm_solve / mt_cfm_solve_bounded replay the evaluation chain (time embedding + every estimator
 * evaluation) as a captured hipGraph, cached per (packed, workspace, B, T, steps, solver, path flags); the caller's
 * mask is staged into the workspace first, so replays read no caller pointer. 0: direct launches. Bypassed while a
 * launch probe or the launch log is armed. Same results either way. */
int mt_decoder_set_graphs(mt_decoder* d, int enable);
/* Debug taps honoured by mt_decoder_step only: taps[i] (device fp32 [B,256,T_l], or NULL) receives a copy of
 * the block output the reference fixture records with forward hooks — 0 down_blocks[0][0] (ResnetBlock1D),
 * 1 down_blocks[0][1][0] (BasicTransformerBlock, channel-major), 2 mid_blocks[-1][1][0] (T/2), 3 up_blocks[0][2]
 * (Upsample1D, masked), 4 up_blocks[1][1][0] (model.py:984-1043). n <= 5; NULL / n = 0 clears them. */
int mt_decoder_set_taps(mt_decoder* d, float* const* taps, int n);

size_t mt_decoder_step_workspace_bytes(const mt_decoder* d, int B, int T);
/* one estimator evaluation: out = Decoder.forward(x, mask, mu_y, t, spks) [B,80,T] */
int mt_decoder_step(const mt_decoder* d, const void* packed, const float* x, const float* mu_y,
                    const float* mask, const float* spks, float t, int B, int T, float* out, void* ws,
                    size_t ws_bytes, void* stream);
/* the same with one time per utterance, t [B] fp32 in device memory (Decoder.forward with a [B] t as
 * CFM.compute_loss calls it, model.py:1147-1162) */
size_t mt_decoder_step_times_workspace_bytes(const mt_decoder* d, int B, int T);
int mt_decoder_step_times(const mt_decoder* d, const void* packed, const float* x, const float* mu_y,
                          const float* mask, const float* spks, const float* t, int B, int T, float* out,
                          void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * HiFi-GAN Generator (hifigan/models.py:148-206). Parameters are the folded weights
 * ("conv_pre.weight", "ups.0.weight", "resblocks.4.convs1.1.weight", ...) i.e. after
 * remove_weight_norm (hifigan/models.py:199-206).
 * ------------------------------------------------------------------------------------- */
typedef struct mt_vocoder mt_vocoder;
/* rb_dils: n_kernels x n_dils row-major */
int mt_vocoder_create(int resblock, int n_ups, const int* up_rates, const int* up_kernels,
                      int up_init_channel, int n_kernels, const int* rb_kernels, int n_dils,
                      const int* rb_dils, int dtype, mt_vocoder** out);
void mt_vocoder_destroy(mt_vocoder* v);
int mt_vocoder_num_params(const mt_vocoder* v);
int mt_vocoder_param_name(const mt_vocoder* v, int i, char* buf, int buflen);
int mt_vocoder_param_shape(const mt_vocoder* v, int i, int64_t* shape, int maxdim);
size_t mt_vocoder_packed_bytes(const mt_vocoder* v);
/* fused ResBlock stages for the 32/64-channel stages in bf16 (default on; bit-identical to the
 * per-layer path, which 0 selects) */
int mt_vocoder_set_fusion(mt_vocoder* v, int enable);
/* LDS-DMA persistent convs (mt_vconv) for the bf16 ResBlock1 stages with C % 64 == 0: inputs
 * pre-activated by their producers, same rounding points as the generic per-layer path. mode 1:
 * the stages the fused ResBlock kernel does not serve (C = 128, 256); mode 2 (default, measured
 * faster): also the 64-channel stage instead of the fused kernel; 0: the generic per-layer kernel. Replaces the same
 * convs as mt_vocoder_forward (hifigan/models.py:90-97, 187-192). */
int mt_vocoder_set_vconv(mt_vocoder* v, int mode);
/* bf16, vconv mode 2: ResBlock pairs (conv_{k,d} -> lrelu -> conv_{k,1} -> + x, hifigan/models.py:90-97) each as
 * ONE launch with the intermediate on chip and the input activation applied on chip. 1 (default): the 64- and
 * 32-channel stages' pairs and the 128-channel stage's k = 3 resblock; 4: every 128-channel pair too; 2: none of
 * the 128-channel stage; 0: every pair as two per-layer launches. Same bits in every mode. */
int mt_vocoder_set_pair(mt_vocoder* v, int enable);
int mt_vocoder_pack(const mt_vocoder* v, const float* const* params, void* packed, void* stream);
size_t mt_vocoder_workspace_bytes(const mt_vocoder* v, int B, int T);
/* mel [B,80,T] fp32 -> wav [B,1,T*prod(up_rates)] fp32 */
int mt_vocoder_forward(const mt_vocoder* v, const void* packed, const float* mel, int B, int T,
                       float* wav, void* ws, size_t ws_bytes, void* stream);
/* Ragged batch: utterance b is vocoded at its own lens[b] mel frames (int32, device; frames past it are the
 * zero padding a batch-1 call of that length sees), so wav[b][0, 256 lens[b]) equals Generator.forward on
 * mel[b:b+1, :, :lens[b]] alone; wav[b] past it is zero and columns past lens[b] are not computed. Needs the bf16
 * vconv / pair path on every stage (the defaults) and B <= 512. */
int mt_vocoder_forward_ragged(const mt_vocoder* v, const void* packed, const float* mel, int B, int T,
                              const int32_t* lens, float* wav, void* ws, size_t ws_bytes, void* stream);
/* 1 when mt_vocoder_forward_ragged runs with this handle's precision and path modes, else 0 */
int mt_vocoder_ragged_supported(const mt_vocoder* v);

/* ---------------------------------------------------------------------------------------
 * Duration -> alignment index path (bit-exact given logw).
 * ------------------------------------------------------------------------------------- */
/* w_ceil = ceil(exp(logw)*x_mask*length_scale) [B,Tx]; cum = cumsum(w_ceil) [B,Tx];
 * y_lengths = max(sum(w_ceil), 1) int64 [B]. */
int mt_durations(const float* logw, const float* x_mask, float length_scale, int B, int Tx,
                 float* w_ceil, float* cum, int64_t* y_lengths, void* stream);
/* attn [B,1,Tx,T] one-hot path (may be NULL); mu_y[b,c,j] = mu[b,c,token(j)] [B,C,T] (may be NULL);
 * y_mask [B,1,T] = (j < y_lengths[b]) (may be NULL) */
int mt_alignment(const float* cum, const int64_t* y_lengths, int B, int Tx, int T, const float* mu, int C,
                 float* attn, float* mu_y, float* y_mask, void* stream);
/* mel[b,c,t] = z[b,c,t]*std[c] + mean[c] for t < Ty; z [B,C,T] -> mel [B,C,Ty] */
int mt_denorm_crop(const float* z, const float* mean, const float* std, int B, int C, int T, int Ty,
                   float* mel, void* stream);

/* ---------------------------------------------------------------------------------------
 * Denoiser (hifigan/denoiser.py): STFT n_fft 1024 / hop 256 / Hann, magnitude - strength*bias,
 * clamp >= 0, iSTFT. audio [B,L] -> out [B, 256*(L/256)]; bias_spec [513].
 * ------------------------------------------------------------------------------------- */
size_t mt_denoise_workspace_bytes(int B, int L);
int mt_denoise(const float* audio, int B, int L, const float* bias_spec, float strength, float* out,
               void* ws, size_t ws_bytes, void* stream);
/* Ragged batch: row b denoised as an utterance of lens[b] * lmul samples (int32, device; its own reflect padding
 * and 1 + samples / 256 frames, as a one-utterance call); out[b] past those samples is zero. */
int mt_denoise_ragged(const float* audio, int B, int L, const int32_t* lens, int lmul, const float* bias_spec,
                      float strength, float* out, void* ws, size_t ws_bytes, void* stream);
/* |STFT| (same framing) of every frame: mag [B][1+L/256][513] (bias spectrum, denoiser.py:57-60) */
int mt_stft_magnitude(const float* audio, int B, int L, float* mag, void* stream);

/* ---------------------------------------------------------------------------------------
 * Log-mel featurizer (§8f rank 4), replacing train_standalone.py:164-201 `mel_spectrogram(y, 1024, 80,
 * 22050, 256, 1024, fmin, fmax, center=False)` + `normalize(mel, mel_mean, mel_std)` (:204-210,
 * hifigan/meldataset.py:52-89): reflect pad 384 | STFT 1024/256 Hann, center=False | sqrt(|S|^2 + 1e-9) |
 * mel_basis . | log(clamp(., 1e-5)) | (. - mel_mean) / mel_std.
 * audio [B][L] fp32 (L > 384), mel_basis [80][513] fp32 (librosa slaney filters, host-computed) ->
 * mel [B][80][F] fp32, F = (L - 256) / 256 + 1.
 * ------------------------------------------------------------------------------------- */
int mt_log_mel(const float* audio, int B, int L, const float* mel_basis, float mel_mean, float mel_std, float* mel,
               void* stream);

/* ---------------------------------------------------------------------------------------
 * Training-side (§8f rank 3): Monotonic Alignment Search, replacing train_standalone.py:280-325
 * `maximum_path(neg_cent, mask)` (a device->host copy + CPU numba/Python DP in the reference) with
 * its exact recurrence as a GPU anti-diagonal wavefront. neg_cent [B][Tx][Ty] fp32, t_xs / t_ys [B]
 * int32 (the mask's token / frame counts) -> paths [B][Tx][Ty] fp32 one-hot per frame column inside
 * [0,t_x) x [0,t_y), zero elsewhere. Tx <= 1024.
 * ------------------------------------------------------------------------------------- */
size_t mt_maximum_path_workspace_bytes(int B, int Tx, int Ty);
int mt_maximum_path(const float* neg_cent, const int32_t* t_xs, const int32_t* t_ys, int B, int Tx, int Ty,
                    float* paths, void* ws, size_t ws_bytes, void* stream);

/* ---------------------------------------------------------------------------------------
 * Training step (§8f rank 3): fp32 primitives the CFM training step (train_standalone.py:623-707,
 * MatchaLightningModule.forward / training_step / configure_optimizers; model.py:1147-1162 compute_loss)
 * is built from, forward and backward (matcha_hip/train.py composes them). Activations are [rows][C]
 * row-major fp32 device buffers. No reduction uses atomics (bitwise reproducible).
 * ------------------------------------------------------------------------------------- */
/* C[z] = (alpha op(A[z]) op(B[z]) + beta C[z] + bias[n]) * row_mask[z][m]; op(A) M x K, op(B) K x N; z < batch,
 * strides in elements; bias [N] and row_mask [batch][M] optional (NULL). Exact-fp32 MFMA (32x32x2 f32); a long K over
 * few output tiles is split into slices whose partials (in the caller's workspace) are summed in slice order
 * (deterministic). */
int mtt_gemm(int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda, long long sA,
             const float* B, int ldb, long long sB, float beta, float* C, int ldc, long long sC, int batch,
             const float* bias, const float* row_mask, float* ws, size_t ws_bytes, void* stream);
/* mtt_gemm with the operands rounded (RNE) to a 16-bit format before 16-bit MFMA with fp32 accumulation:
 * opfmt 0 none (= mtt_gemm), 1 fp16 (the reference Trainer's precision="16-mixed", train_standalone.py:868, under
 * which autocast runs conv1d / linear / matmul on fp16 operands), 2 bf16 ("bf16-mixed"). The output stays fp32. */
int mtt_gemm_ex(int opfmt, int transA, int transB, int M, int N, int K, float alpha, const float* A, int lda,
                long long sA, const float* B, int ldb, long long sB, float beta, float* C, int ldc, long long sC,
                int batch, const float* bias, const float* row_mask, float* ws, size_t ws_bytes, void* stream);
/* device workspace mtt_gemm uses to split a long K over slices (0: never splits this shape); with less, it runs
 * unsplit */
size_t mtt_gemm_workspace_bytes(int M, int N, int K, int batch);
/* conv1d columns: cols[(b*Tout+o)][c*k+tap] = x[b][t][c] * mask[b][t], t = o*stride-pad+tap*dil (a torch Conv1d weight
 * [Cout][Cin][k] is then the GEMM operand as stored; mask [B][T] optional: the reference's conv(x * mask)); col2im is
 * its adjoint, dx[b][t][c] (+)= mask[b][t] * sum of the columns that read (b, t, c) */
int mtt_im2col(const float* x, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
               float* cols, void* stream);
int mtt_col2im(const float* dcols, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil,
               int Tout, float* dx, int accumulate, void* stream);
/* out[i] (+)= op(a[i], b[((i/d0)%m0)*s0 + ((i/d1)%m1)*s1], c[i]); op: 0 alpha a + beta b, 1 alpha a b,
 * 2 mish(a), 3 c mish'(a), 4 silu(a), 5 c silu'(a), 6 relu(a), 7 c [a>0], 8 exp(a), 9 (a-b)^2, 10 sin(a),
 * 11 cos(a), 12 log(alpha + a), 13 alpha / a */
int mtt_ew(int op, size_t n, const float* a, const float* b, const float* c, float* out, float alpha, float beta,
           size_t d0, size_t m0, size_t s0, size_t d1, size_t m1, size_t s1, int accumulate, void* stream);
/* dst[r][doff+j] (+)= src[r][soff+j], r < rows, j < n (channel concat / split; lds, ldd row strides) */
int mtt_copy_cols(const float* src, int lds, int soff, float* dst, int ldd, int doff, int rows, int n, int accumulate,
                  void* stream);
/* sequence_mask (model.py:42-46, train_standalone.py:328-333): out[b][t] = t < lengths[b], fp32 [B][T] */
int mtt_seq_mask(const int64_t* lengths, int B, int T, float* out, void* stream);
/* out[s][c] (+)= sum over rows r of segment s (seg rows each) of a[r][c] (* b[r][c]); scratch >=
 * mtt_colsum_scratch_floats(rows, C, seg) floats */
size_t mtt_colsum_scratch_floats(int rows, int C, int seg);
int mtt_colsum(const float* a, const float* b, int rows, int C, int seg, float* out, int accumulate, float* scratch,
               void* stream);
/* out[0] = sum_i a[i] (* b[i]); scratch >= 1024 floats */
int mtt_sum(const float* a, const float* b, size_t n, float* out, float* scratch, void* stream);
/* dropout(p) with a counter-based hash mask of (seed, index): out = a * keep / (1 - p); the backward is the same
 * call on the gradient with the same seed */
int mtt_dropout(const float* a, size_t n, float p, unsigned seed, float* out, void* stream);
/* torch.nn.GroupNorm over x [B][T][C] (model.py:764-775); backward writes dx and per-(b, c) partials of the
 * gamma / beta gradients [B][C] (reduce with mtt_colsum) */
int mtt_groupnorm_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, int G, float eps,
                      float* y, float* mean, float* rstd, void* stream);
int mtt_groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int B,
                      int T, int C, int G, float* dx, float* dgamma_part, float* dbeta_part, void* stream);
/* LayerNorm over the C channels of each row (decoder nn.LayerNorm, encoder channel LayerNorm model.py:148-166) */
int mtt_layernorm_fwd(const float* x, const float* gamma, const float* beta, int rows, int C, float eps, float* y,
                      float* mean, float* rstd, void* stream);
int mtt_layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd,
                      int rows, int C, float* dx, void* stream);
/* SnakeBeta (model.py:580-609) on [n/C][C]; backward: dx and per-element log-alpha / log-beta gradient terms */
int mtt_snake_fwd(const float* x, const float* log_alpha, const float* log_beta, size_t n, int C, float* y,
                  void* stream);
int mtt_snake_bwd(const float* x, const float* log_alpha, const float* log_beta, const float* dy, size_t n, int C,
                  float* dx, float* galpha, float* gbeta, void* stream);
/* row softmax of scale*s [BH][Tq][Tk] with masked keys (kmask [B][Tk] == 0) or masked queries (qmask [B][Tq],
 * may be NULL) := +3.4e38 (mode 0, decoder model.py:697) or -1e4 (mode 1, encoder model.py:353) */
int mtt_softmax_fwd(const float* s, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk, float scale,
                    int mode, float* p, void* stream);
int mtt_softmax_bwd(const float* p, const float* dp, const float* kmask, const float* qmask, int BH, int H, int Tq,
                    int Tk, float scale, float* ds, void* stream);
/* RoPE in place on x [B][T][H*dh] (first d features of each head), inverse = 1 for the backward */
int mtt_rope(float* x, int B, int T, int H, int dh, int d, const float* theta, int inverse, void* stream);
int mtt_embed_fwd(const int64_t* ids, size_t ntok, const float* table, int C, float scale, float* out, void* stream);
int mtt_embed_bwd(const int64_t* ids, size_t ntok, const float* dout, int V, int C, float scale, float* dtable,
                  void* stream);
/* torch.optim.Adam step (lr, betas, eps; no weight decay) with grad scaled by *gscale (clip / world) */
int mtt_adam(float* p, const float* g, float* m, float* v, size_t n, const float* gscale, float lr, float beta1,
             float beta2, float eps, int step, void* stream);
/* clip factor for a flat gradient holding the SUM over `world` ranks: norm = sqrt(*sumsq) * inv_world (the norm of
 * the DDP-averaged gradient), out = min(1, max_norm / (norm + 1e-6)) * inv_world (torch.nn.utils.clip_grad_norm_) */
int mtt_clip_factor(const float* sumsq, float max_norm, float inv_world, float* out, float* norm_out, void* stream);
/* torch.cuda.amp.GradScaler.unscale_ ("16-mixed", train_standalone.py:868): g *= inv_scale in place, and
 * *found = the number of non-finite elements of g as stored, checked before the multiply (the per-element
 * found-inf check of torch._amp_foreach_non_finite_check_and_unscale_); scratch >= 1024 floats */
int mtt_unscale(float* g, size_t n, float inv_scale, float* found, float* scratch, void* stream);

/* ---------------------------------------------------------------------------------------
 * Op-level entry points (per-kernel parity tests)
 * ------------------------------------------------------------------------------------- */
/* y = conv(act(x)), x [B][Tin][Cin], y [B][Tout][Cout] in dtype; W fp32 reference layout
 * (Conv1d [Cout][Cin][k]; transposed: ConvTranspose1d [Cin][Cout][k]); slope < 0: no act. */
size_t mt_op_conv1d_workspace_bytes(int dtype, int cin, int cout, int k, int stride, int transposed);
int mt_op_conv1d(int dtype, const void* x, int B, int Tin, int cin, const float* W, const float* bias,
                 int cout, int k, int stride, int pad, int dil, int transposed, float slope, void* y,
                 int Tout, void* ws, size_t ws_bytes, void* stream);
/* same with a fixed tile variant (in-process A/B timing; lrelu prologue only; -1 = automatic;
 * variant + 0x1000 reuses the weights a previous call packed into ws) */
int mt_op_conv1d_tile(int variant, int dtype, const void* x, int B, int Tin, int cin, const float* W,
                      const float* bias, int cout, int k, int stride, int pad, int dil, int transposed,
                      float slope, void* y, int Tout, void* ws, size_t ws_bytes, void* stream);
/* Op-level entry of mt_vconv (tests / A-B timing): bf16 x [B][L][cin] already activated, fp32
 * W [cout][cin][k], bias [cout], padding dil*(k-1)/2 ("same"), epilogue flags ef: 1 + resid,
 * 2 accumulate into y, 4 / div, 8 y = lrelu(v), 16 also y2 = lrelu(v); lens (nullable, device int32 [B]): the
 * ragged batch, utterance b valid for its first lens[b] frames. pack = 0 reuses the weights a
 * previous call with the same ws packed (timing). One ResBlock1 conv of hifigan/models.py:90-97. */
size_t mt_op_vconv_workspace_bytes(int cin, int cout, int k);
int mt_op_vconv(const void* x, int B, int L, int cin, const float* W, const float* bias, int cout, int k, int dil,
                int ef, const void* resid, void* y, void* y2, float slope, float div, const int32_t* lens, int pack,
                void* ws, size_t ws_bytes, void* stream);
/* The HiFi-GAN wide-stage ResBlock convs (C_in = C_out in {128, 256}, k in {3, 7, 11}) run on mt_rbconv, a variant
 * of mt_vconv whose K loop is scheduled at compile time (1, the default; bit-identical results) or on the generic
 * mt_vconv kernel (0). Process-wide; returns the previous setting. */
int mt_vconv_set_rbconv(int enable);
/* The decoder's convs and the upsamplers run mt_vconv with their K loop unrolled at compile time for their
 * (C_in, taps) (1, the default; bit-identical results) or with the runtime-cursor loop (0). Process-wide; returns
 * the previous setting. */
int mt_vconv_set_ct(int enable);
/* Round-5 ResBlock pair kernels (mask; each bit-identical to the kernel it replaces): bit 0 the 64-channel k = 7 / 11
 * pairs' compile-time K loop, bit 1 the 128-channel k = 3 pairs' one. Default 3 (MT_VPAIRK=<mask> in the
 * environment); process-wide; returns the previous mask. */
int mt_vpair_set_kernels(int mask);
/* conv_post (hifigan/models.py:193-195) in the epilogue of the last stage's final ResBlock pair (1, the default: the stage
 * output xs is never stored) or as its own launch after it (0). Both run the same MFMA arithmetic (bit-identical).
 * Process-wide; returns the previous setting (MT_POSTFOLD=0 in the environment: off). */
int mt_vocoder_set_post_fold(int enable);
/* The stage 1-2 ResBlock conv1s (mt_rbconv) read the raw chain state and apply its leaky ReLU to their staged rows in
 * LDS, so the producing convs store no activated copy (1, the default; bit-identical results), or read an activated
 * copy the producers store (0). Process-wide; returns the previous setting. */
int mt_vconv_set_actin(int enable);
/* The bf16 decoder's transformer FeedForward (LayerNorm, Linear 256 -> 1024, SnakeBeta, Linear 1024 -> 256, + x) as
 * one fused launch whose 1024-wide intermediate stays on chip (3, the default; 1 / 2 other schedules of the same
 * kernel; bit-identical results) or as two mt_vconv GEMM launches (0). Process-wide; returns the previous setting. */
int mt_ffn_set(int enable);
/* ... on decoder levels of at least `frames` frames (B x T at that level; default 16384); returns the previous value */
int mt_ffn_set_min_frames(int frames);
/* Decoder kernel variants (mask; each bit-identical to the launches it replaces): bit 0 the final projection + ODE
 * update (final_proj of mish(GroupNorm) * mask, z += dt * v) on a dedicated kernel instead of the generic conv
 * kernel. Default 1 (MT_DECK=<mask> in the environment); process-wide; returns the previous mask. */
int mt_decoder_set_kernels(int mask);
/* qkv [B][T][3*heads*64], mask [B][T] -> out [B][T][heads*64], reference mask semantics */
int mt_op_attention(int dtype, const void* qkv, const float* mask, void* out, int B, int T, int heads,
                    void* stream);

/* ---------------------------------------------------------------------------------------
 * Launch probe (measurement only; no reference counterpart). Arms HIP events around every
 * launch of one kernel site, on the stream the kernel is launched on, so a benchmark can time
 * that kernel inside its own timed region. Sites: 1 = fused 64-channel HiFi-GAN ResBlock stage,
 * 2 = fused 32-channel stage, 3 = every HiFi-GAN ResBlock conv launch on mt_vconv and every fused conv-pair
 * launch (mt_vpair / mt_vpair32, priced as its two convs), 4 = the
 * decoder's k >= 2 mt_vconv launches. mt_probe_stop synchronizes the recorded events and returns the
 * number of launches, their summed duration, the algorithmic FLOPs and layer-boundary bytes they did
 * (every conv reads its input once and writes its output once, + its weights), and
 * roof_ms = sum over launches of max(FLOPs / peak_flops, bytes / peak_bw) (peaks in FLOP/s, B/s).
 * mt_probe_pause(1) stops recording (launches run unprobed) until mt_probe_pause(0); mt_probe_start
 * arms the probe unpaused. A benchmark probes a sample of its timed steps this way, since each event
 * pair adds a few microseconds of idle before the launch it brackets.
 * ------------------------------------------------------------------------------------- */
#define MT_PROBE_RBFUSE_C64 1
#define MT_PROBE_RBFUSE_C32 2
#define MT_PROBE_VCONV 3
#define MT_PROBE_VCONV_DEC 4
int mt_probe_start(int site, int max_launches);
int mt_probe_pause(int paused);
/* per recorded launch: duration (ms), algorithmic FLOPs and bytes, kernel tag (0 mt_vconv, 1 mt_vpair,
 * 2 mt_vpair32, 3 mt_rbfuse); synchronizes the events; call before mt_probe_stop. Returns the count written. */
int mt_probe_detail(int cap, double* ms, double* flops, double* bytes, int* tags);
int mt_probe_stop(int* launches, double* total_ms, double* flops, double* bytes, double peak_flops, double peak_bw,
                  double* roof_ms);

/* Launch log of the persistent LDS-DMA conv (test coverage only; no reference counterpart). While
 * armed, every mt_vconv launch appends 11 int32: epilogue flags, rows per tile (BM), frames per tile
 * (BN), 1x1 pipeline flag, output tiles, grid size (tiles > grid: workgroups walk several tiles), taps,
 * output channels, input channels, utterances, frames per utterance. stop returns the record count. */
#define MT_VCONV_LOG_FIELDS 11
int mt_vconv_log_start(int capacity);
int mt_vconv_log_stop(int32_t* records, int capacity);

#ifdef __cplusplus
}
#endif
#endif /* MATCHA_HIP_H */
