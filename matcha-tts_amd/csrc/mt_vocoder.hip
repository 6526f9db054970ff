// HiFi-GAN Generator driver (hifigan/models.py:148-206; ResBlock1 :90-97, ResBlock2 :133-138).
//
//   mel [B,80,T] fp32 -> [B][T][80] -> conv_pre k7 -> per stage i:
//     lrelu(0.1) -> ConvTranspose1d (polyphase GEMM) -> X
//     for resblock j: chain of (lrelu -> conv(k, d) -> lrelu -> conv(k, 1) -> + x) pairs,
//                     the last conv of the chain accumulates into XS (xs += ...; / nk fused)
//   -> lrelu(0.01) -> conv_post k7 -> tanh -> wav [B,1,256T] fp32
// Buffers (each B x T x frame_elems elements): XS (stage input / resblock sum), X (upsampled),
// Tb (first conv of a pair), R (resblock chain state, updated in place).
#include <algorithm>
#include <type_traits>

#include "mt_model.h"
#include "mt_ragged.h"
#include "mt_rbfuse.h"
#include "mt_vconv.h"
#include "mt_vpair.h"

namespace mt {

// conv_post (hifigan/models.py:194-196) for bf16 C = 32: tanh(conv_k7(lrelu(x, 0.01)) + b), one output channel.
// 256 samples per workgroup: their 262 input rows staged once in LDS as bf16(lrelu(x)), the image post_taps reads
// (mt_vpair.h; mt_vpair32's VE_POST epilogue runs the same arithmetic on its own tile).
constexpr int PC_N = 256;
// Ragged batch (lens != null): utterance b has Lb = lens[b] * lmul samples; rows past Lb are zero padding and its
// samples past Lb are written as zeros.
__global__ __launch_bounds__(256) void post_conv_kernel(const bf16* __restrict__ x, int L,
                                                        const bf16* __restrict__ w, const float* __restrict__ bias,
                                                        float slope, float* __restrict__ out, const int* lens,
                                                        int lmul) {
  // v = bf16(lrelu(x, slope)) of frames f0 - 3 .. f0 + PC_N + 2 (zero outside [0, Lb)) as post_taps's LDS image:
  // 64-byte rows, 16-byte chunk q at slot q ^ ((row >> 1) & 2); each wave then runs 4 blocks of 16 frames on MFMA
  // (rows up to 64 wave + 79 are read: the last 10 never reach a kept sum)
  __shared__ __attribute__((aligned(16))) char rows[(PC_N + 16) * 64];
  const int b = blockIdx.y, f0 = blockIdx.x * PC_N, tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const bf16* xb = x + (size_t)b * L * 32;
  const int Lb = lens ? min(max(lens[b] * lmul, 0), L) : L;
  if (f0 >= Lb) {  // wholly past the utterance
    if (f0 + tid < L) out[(size_t)b * L + f0 + tid] = 0.f;
    return;
  }
  for (int e = tid; e < (PC_N + 6) * 4; e += 256) {
    const int r = e >> 2, q = e & 3;
    const int f = f0 - 3 + r;
    u32x4 v = {0u, 0u, 0u, 0u};
    if (f >= 0 && f < Lb) {
      v = *reinterpret_cast<const u32x4*>(xb + (size_t)f * 32 + q * 8);
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = lrelu_pk_sel(v[j], slope);
    }
    *reinterpret_cast<u32x4*>(rows + r * 64 + ((q ^ ((r >> 1) & 2)) * 16)) = v;
  }
  const bf16x8 wt = post_wtaps(w, lane);
  __syncthreads();
  const float bs = bias[0];
  f32x4 dp = post_taps(rows, wave * (PC_N / 4), wt, lane);
#pragma unroll
  for (int j = 0; j < PC_N / 64; ++j) {
    const int r0 = wave * (PC_N / 4) + 16 * j;
    const f32x4 dn = post_taps(rows, r0 + 16, wt, lane);
    const float s = post_combine(dp, dn, lane);
    dp = dn;
    const int f = f0 + r0 + lane;
    const float th = post_tanh(s + bs);
    if (lane < 16 && f < L) out[(size_t)b * L + f] = f < Lb ? th : 0.f;
  }
}

// rows [lens[b], T) of utterance b of a [B][T][C] tensor := 0 (a ragged batch's zero padding)
template <class E>
__global__ void zero_tail_rows_kernel(E* __restrict__ x, int T, int C, const int* __restrict__ lens) {
  const int b = blockIdx.y;
  const int Lb = min(max(lens[b], 0), T);
  E* xb = x + (size_t)b * T * C;
  for (size_t e = (size_t)Lb * C + blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < (size_t)T * C;
       e += (size_t)gridDim.x * blockDim.x)
    xb[e] = (E)0.f;
}

static int zero_tail_rows(int dtype, void* x, int B, int T, int C, const int* lens, hipStream_t st) {
  const dim3 grid(std::max(1, std::min(64, (T * C + 255) / 256)), B);
  if (dtype == BF16) hipLaunchKernelGGL(zero_tail_rows_kernel<bf16>, grid, dim3(256), 0, st, (bf16*)x, T, C, lens);
  else hipLaunchKernelGGL(zero_tail_rows_kernel<float>, grid, dim3(256), 0, st, (float*)x, T, C, lens);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int Vocoder::init(int resblock_, const std::vector<int>& ur, const std::vector<int>& uk, int up_init_,
                  const std::vector<int>& rk, const std::vector<std::vector<int>>& rd, int dtype_) {
  MT_REQUIRE(resblock_ == 1 || resblock_ == 2, "vocoder: resblock must be 1 or 2");
  MT_REQUIRE(ur.size() == uk.size() && !ur.empty(), "vocoder: upsample config");
  MT_REQUIRE(rk.size() == rd.size() && !rk.empty(), "vocoder: resblock config");
  MT_REQUIRE(dtype_ == F32 || dtype_ == BF16, "vocoder: dtype");
  resblock = resblock_;
  up_rates = ur;
  up_kernels = uk;
  up_init = up_init_;
  rb_kernels = rk;
  rb_dils = rd;
  dtype = dtype_;
  esize = dtype == BF16 ? 2 : 4;
  params = ParamList();
  ups.clear();
  rb1.clear();
  rb2.clear();
  Packer pk;
  ParamList& L = params;
  {
    int w = L.add("conv_pre.weight", {up_init, n_mels, 7});
    int b = L.add("conv_pre.bias", {up_init});
    pre = make_conv(up_init, n_mels, 7, 1, 3, 1, {w}, b, esize, pk);
  }
  int ch = up_init;
  for (size_t i = 0; i < ur.size(); ++i) {
    const int cin = up_init >> i, cout = up_init >> (i + 1);
    MT_REQUIRE(uk[i] % ur[i] == 0 && (uk[i] - ur[i]) % 2 == 0,
               "vocoder: upsample kernel %d must be a multiple of rate %d", uk[i], ur[i]);
    MT_REQUIRE(cout % 32 == 0 || cout % 4 == 0, "vocoder: channels");
    const std::string p = "ups." + std::to_string(i);
    int w = L.add(p + ".weight", {cin, cout, uk[i]});
    int b = L.add(p + ".bias", {cout});
    ups.push_back(make_convT(cin, cout, uk[i], ur[i], (uk[i] - ur[i]) / 2, w, b, esize, pk));
    ch = cout;
  }
  const int nk = (int)rk.size();
  for (size_t i = 0; i < ur.size(); ++i) {
    const int c = up_init >> (i + 1);
    for (int j = 0; j < nk; ++j) {
      const std::string p = "resblocks." + std::to_string(i * nk + j);
      std::vector<GemmW> v1, v2;
      const int k = rk[j];
      for (size_t q = 0; q < rd[j].size(); ++q) {
        const int d = rd[j][q];
        if (resblock == 1) {
          int w1 = L.add(p + ".convs1." + std::to_string(q) + ".weight", {c, c, k});
          int b1 = L.add(p + ".convs1." + std::to_string(q) + ".bias", {c});
          v1.push_back(make_conv(c, c, k, 1, (k * d - d) / 2, d, {w1}, b1, esize, pk));
        } else {
          int w1 = L.add(p + ".convs." + std::to_string(q) + ".weight", {c, c, k});
          int b1 = L.add(p + ".convs." + std::to_string(q) + ".bias", {c});
          v1.push_back(make_conv(c, c, k, 1, (k * d - d) / 2, d, {w1}, b1, esize, pk));
        }
      }
      if (resblock == 1) {
        for (size_t q = 0; q < rd[j].size(); ++q) {
          int w2 = L.add(p + ".convs2." + std::to_string(q) + ".weight", {c, c, k});
          int b2 = L.add(p + ".convs2." + std::to_string(q) + ".bias", {c});
          v2.push_back(make_conv(c, c, k, 1, (k - 1) / 2, 1, {w2}, b2, esize, pk));
        }
      }
      rb1.push_back(v1);
      rb2.push_back(v2);
    }
  }
  // wide bf16 ResBlock1 stages: every conv of the stage through mt_vconv (its own weight image)
  any_vc = false;
  if (dtype == BF16 && resblock == 1) {
    for (size_t i = 0; i < ur.size(); ++i) {
      bool ok = true;
      for (int j = 0; j < nk; ++j)
        for (size_t q = 0; q < rb1[i * nk + j].size(); ++q) {
          const GemmW& a = rb1[i * nk + j][q];
          const GemmW& b = rb2[i * nk + j][q];
          ok = ok && vconv_supported(a.cin, a.cout, a.k, a.dil, a.s) && vconv_supported(b.cin, b.cout, b.k, b.dil, b.s);
        }
      if (!ok) continue;
      for (int j = 0; j < nk; ++j)
        for (auto* v : {&rb1[i * nk + j], &rb2[i * nk + j]})
          for (GemmW& g : *v) {
            g.vc = true;
            g.v_off = pk.take(vconv_packed_bytes(g.cin, g.cout, g.k));
          }
      any_vc = true;
    }
    if (any_vc) {
      zero_off = pk.take(256);
      // upsamplers as polyphase convs (rows = phase x C_out, <= 1024 rows per image)
      for (GemmW& g : ups) {
        const int ng = (g.M + 1023) / 1024;
        const int rows = g.M / ng;
        if (g.M % ng || g.cout % 8 || !vconv_supported(g.cin, rows, g.taps, 1, 1)) continue;
        g.vc = true;
        g.vrows = rows;
        g.v_off = pk.take((size_t)ng * vconv_packed_bytes(g.cin, rows, g.taps));
      }
    }
  }
  {
    int w = L.add("conv_post.weight", {1, ch, 7});
    int b = L.add("conv_post.bias", {1});
    post = make_conv(1, ch, 7, 1, 3, 1, {w}, b, esize, pk);
  }
  packed_bytes = pk.off;
  return 0;
}

int Vocoder::pack(const float* const* p, void* packed, hipStream_t st) const {
  char* P = (char*)packed;
  int rc;
  if ((rc = pack_gemm(pre, dtype, p, P, st))) return rc;
  for (const GemmW& g : ups) {
    if ((rc = pack_gemm(g, dtype, p, P, st))) return rc;
    if (!g.vc) continue;
    for (int gi = 0; gi < g.M / g.vrows; ++gi) {
      const char* src = P + g.w_off + (size_t)gi * g.vrows * g.taps * g.cin_pad * esize;
      char* dst = P + g.v_off + (size_t)gi * vconv_packed_bytes(g.cin, g.vrows, g.taps);
      if ((rc = vconv_repack(src, g.vrows, g.taps, g.cin_pad, g.cin, g.vrows, dst, st))) return rc;
    }
  }
  for (size_t i = 0; i < rb1.size(); ++i) {
    for (const GemmW& g : rb1[i])
      if ((rc = pack_gemm(g, dtype, p, P, st))) return rc;
    for (const GemmW& g : rb2[i])
      if ((rc = pack_gemm(g, dtype, p, P, st))) return rc;
    for (auto* v : {&rb1[i], &rb2[i]})
      for (const GemmW& g : *v)
        if (g.vc && (rc = vconv_repack(P + g.w_off, g.Mpad, g.taps, g.cin_pad, g.cin, g.cout, P + g.v_off, st)))
          return rc;
  }
  if (any_vc && (rc = pack_vec(nullptr, 1, 64, 0, (float*)(P + zero_off), st))) return rc;
  return pack_gemm(post, dtype, p, P, st);
}

size_t Vocoder::frame_elems() const {
  size_t m = (size_t)up_init;  // conv_pre output
  size_t rate = 1;
  for (size_t i = 0; i < up_rates.size(); ++i) {
    rate *= up_rates[i];
    m = std::max(m, rate * (size_t)(up_init >> (i + 1)));
  }
  return m;
}

bool Vocoder::stage_vc(int i) const {
  const int nk = (int)rb_kernels.size();
  if (!(vconv && dtype == BF16 && resblock == 1 && !rb1[(size_t)i * nk].empty() && rb1[(size_t)i * nk][0].vc))
    return false;
  // stages the fused ResBlock kernel serves stay fused unless vconv mode 2 asks for the per-layer path
  const int C = rb1[(size_t)i * nk][0].cout;
  return vconv >= 2 || !(fuse && rbfuse_supported(dtype, C));
}

// resblock j of wide stage i as one fused-pair launch per pair. C = 128 (mt_vpair128) pays only where the pair is
// HBM-bound: pair mode 1 (default) fuses its k = 3 resblock, 4 every resblock, 2 none (measured per pair at B = 256:
// k = 3 3.9 ms fused vs 4.3 per layer, k = 7 / 11 7.0 / 10.3 fused vs 6.9 / 9.4 per layer)
bool Vocoder::rb_vp(int i, int j) const {
  if (!pair || vconv < 2 || !stage_vc(i)) return false;
  const int nk = (int)rb_kernels.size();
  for (size_t q = 0; q < rb1[(size_t)i * nk + j].size(); ++q) {
    const GemmW& a = rb1[(size_t)i * nk + j][q];
    const GemmW& b = rb2[(size_t)i * nk + j][q];
    const bool ok = a.cout == 128 ? (pair == 4 || (pair == 1 && a.k == 3)) && a.cin == 128 &&
                                        vpair128_supported(a.k, a.dil)
                                  : vpair_supported(a.cout, a.k, a.dil);
    if (!ok || b.k != a.k || b.dil != 1) return false;
  }
  return true;
}

bool Vocoder::stage_vp(int i) const {
  const int nk = (int)rb_kernels.size();
  for (int j = 0; j < nk; ++j)
    if (!rb_vp(i, j)) return false;
  return nk > 0;
}

bool Vocoder::stage_vp32(int i) const {
  const int nk = (int)rb_kernels.size();
  // (needs the zero rows and the trash area of a vconv model)
  if (!pair || !fuse || vconv < 2 || !any_vc || dtype != BF16 || resblock != 1 || rb1[(size_t)i * nk].empty()) return false;
  for (int j = 0; j < nk; ++j)
    for (size_t q = 0; q < rb1[(size_t)i * nk + j].size(); ++q) {
      const GemmW& a = rb1[(size_t)i * nk + j][q];
      const GemmW& b = rb2[(size_t)i * nk + j][q];
      for (const GemmW* g : {&a, &b})
        if (g->cin != 32 || g->cout != 32 || g->Mpad != 32 || g->cin_pad != 32 || g->taps != g->k) return false;
      if (!vpair32_supported(a.k, a.dil) || b.k != a.k || b.dil != 1) return false;
    }
  return true;
}

// One launch per pair (mt_vpair128 / mt_vpair / mt_vpair32); the chain state ping-pongs between R and Tb (a pair
// reads its input's halo, so it cannot write in place); the inputs' activations are applied in LDS.
// conv_post in the last stage's final pair (mt_vpair32 VE_POST): on by default; MT_POSTFOLD=0 in the environment or
// mt_vocoder_set_post_fold(0): the separate post_conv_kernel (the same post_taps arithmetic: bit-identical)
static int g_postfold = -1;
int vocoder_post_fold() {
  if (g_postfold < 0) {
    const char* e = getenv("MT_POSTFOLD");
    g_postfold = e && e[0] == '0' ? 0 : 1;
  }
  return g_postfold;
}
int vocoder_set_post_fold(int enable) {
  const int prev = vocoder_post_fold();
  g_postfold = enable ? 1 : 0;
  return prev;
}

bool Vocoder::post_fold(int i) const {
  const int nk = (int)rb_kernels.size();
  return vocoder_post_fold() && dtype == BF16 && i + 1 == (int)ups.size() && stage_vp32(i) && post.cin == 32 &&
         post.k == 7 && post.cout == 1 && nk > 0 && (rb_kernels[nk - 1] - 1) / 2 <= 5;
}

int Vocoder::pair_resblock(const char* P, int i, int j, int B, int L, const char* X, char* XS, char* Tb, char* R,
                           char* RA, char* trash, bool act_out, hipStream_t st, const int* lens, float* wav) const {
  const int nk = (int)rb_kernels.size();
  const int C = rb1[(size_t)i * nk][0].cout;
  const bool c32 = C == 32;
  int rc;
  const std::vector<GemmW>& c1 = rb1[(size_t)i * nk + j];
  const std::vector<GemmW>& c2 = rb2[(size_t)i * nk + j];
  const int np = (int)c1.size();
  const char* state = X;
  for (int q = 0; q < np; ++q) {
    const bool last = q == np - 1;
    VPairArgs a{};
    a.x = (const bf16*)state;
    a.B = B;
    a.L = L;
    a.w1 = (const bf16*)(P + (c32 ? c1[q].w_off : c1[q].v_off));
    a.b1 = (const float*)(P + c1[q].b_off);
    a.w2 = (const bf16*)(P + (c32 ? c2[q].w_off : c2[q].v_off));
    a.b2 = (const float*)(P + c2[q].b_off);
    a.taps = c1[q].k;
    a.dil = c1[q].dil;
    a.div = (float)nk;
    a.slope = 0.1f;
    a.zero = (const bf16*)(P + zero_off);
    a.trash = (bf16*)trash;
    a.lens = lens;
    a.lmul = rate_upto(i + 1);
    int ef = 0;
    if (!last) {
      a.y = (bf16*)((q & 1) ? Tb : R);
    } else {
      a.y = (bf16*)XS;
      if (j > 0) ef |= VE_ACCUM;
      if (j == nk - 1) ef |= VE_DIV;
      if (j == nk - 1 && act_out) {  // lrelu(xs) for the next upsampler
        a.y2 = (bf16*)RA;
        ef |= VE_DUAL | VE_Y2ONLY;  // the upsampler reads RA alone: the raw xs is dead (not stored)
      }
      if (j == nk - 1 && wav && c32 && !act_out && j > 0) {  // conv_post here; xs is not stored
        a.post_w = (const bf16*)(P + post.w_off);
        a.post_b = (const float*)(P + post.b_off);
        a.post_slope = 0.01f;
        a.wav = wav;
        ef |= VE_POST;
      }
    }
    if ((rc = c32 ? launch_vpair32(ef, a, st) : C == 128 ? launch_vpair128(ef, a, st) : launch_vpair(ef, a, st)))
      return rc;
    state = (const char*)a.y;
  }
  return 0;
}

int Vocoder::pair_chain(const char* P, int i, int B, int L, const char* X, char* XS, char* Tb, char* R, char* RA,
                        char* trash, bool act_out, hipStream_t st, const int* lens, float* wav) const {
  const int nk = (int)rb_kernels.size();
  int rc;
  for (int j = 0; j < nk; ++j)
    if ((rc = pair_resblock(P, i, j, B, L, X, XS, Tb, R, RA, trash, act_out, st, lens, wav))) return rc;
  return 0;
}

int Vocoder::rate_upto(int i) const {
  int r = 1;
  for (int u = 0; u < i && u < (int)up_rates.size(); ++u) r *= up_rates[(size_t)u];
  return r;
}

bool Vocoder::ups_vc(int i) const {
  return vconv && dtype == BF16 && ups[(size_t)i].vc && (i == 0 || stage_vc(i - 1));
}

// ConvTranspose1d(k = taps*s, stride s, pad p) on vconv: column n (n in [0, L+1)) of the polyphase conv
// computes rows (phase, c) = sum_t W[phase, c, t] . xa[n - (taps-1) + t]; it is output frame
// s*n + phase - p, i.e. element n * (s*C) + phase*C + c - p*C of the utterance's [Tout][C] output, and
// exactly the frames in [0, Tout) are kept (hifigan/models.py:184-186; the generic kernel's ConvT
// mapping, mt_conv.hip ups/opad)
int Vocoder::ups_vconv(const char* P, int i, int B, int L, const char* xa, char* X, char* XA, bool dual,
                       char* trash, hipStream_t st, const int* lens) const {
  const GemmW& g = ups[(size_t)i];
  int Tout = 0, Ncols = 0;
  gemm_geom(g, L, &Tout, &Ncols);
  int rc;
  for (int gi = 0; gi < g.M / g.vrows; ++gi) {
    VConvArgs a{};
    a.x = (const bf16*)xa;
    a.B = B;
    a.L = L;
    a.cin = g.cin;
    a.w = (const bf16*)(P + g.v_off + (size_t)gi * vconv_packed_bytes(g.cin, g.vrows, g.taps));
    a.bias = (const float*)(P + g.b_off) + (size_t)gi * g.vrows;
    a.M = a.Mpad = g.vrows;
    a.taps = g.taps;
    a.dil = 1;
    a.pad = g.gpad;
    a.y = (bf16*)X;
    a.y2 = (bf16*)XA;
    a.slope = 0.1f;
    a.div = 1.f;
    a.zero = (const bf16*)(P + zero_off);
    a.trash = (bf16*)trash;
    a.probe = -1;
    a.lens = lens;  // the input's valid frames (rate before this upsampler)
    a.lmul = rate_upto(i);
    a.Lout = Ncols;
    a.ldy = g.M;
    a.yshift = g.opad * g.cout - gi * g.vrows;
    a.ylim = Tout * g.cout;
    a.ystride = (long long)Tout * g.cout;
    if ((rc = launch_vconv(dual ? VE_DUAL : 0, a, st))) return rc;
  }
  return 0;
}

size_t Vocoder::workspace_bytes(int B, int T) const {
  const size_t big = align256((size_t)B * T * frame_elems() * esize);
  // + XA, RA: the activated copies the vconv stages read
  return (any_vc ? 6 * big + 4096 : 4 * big) + align256((size_t)B * T * n_mels * esize);
}

// One wide ResBlock1 stage through mt_vconv (bf16). Per resblock j, pair q (models.py:90-97):
//   Tb = lrelu(conv1(stateA))                         (VE_ACT: conv2 only ever reads lrelu(xt))
//   R, RA = conv2(Tb) + state, lrelu(.)               (VE_DUAL, pairs before the last)
//   XS (+)= conv2(Tb) + state (/ nk on the last resblock)  (last pair)
// Rounding points equal the generic per-layer path's: every stored tensor is rounded to bf16 and the
// activated copies are lrelu of the rounded values.
// every per-layer conv1 of stage i on mt_rbconv with VE_ACTIN (the launch arguments stage_vconv builds)
bool Vocoder::stage_actin(int i, int B, int L, const int* lens) const {
  if (!rbconv_actin_on() || !stage_vc(i) || stage_vp(i)) return false;
  const int nk = (int)rb_kernels.size();
  for (int j = 0; j < nk; ++j) {
    if (rb_vp(i, j)) continue;
    for (const GemmW& g : rb1[(size_t)i * nk + j]) {
      VConvArgs a{};
      a.B = B;
      a.L = L;
      a.cin = a.c0 = g.cin;
      a.M = a.Mpad = g.cout;
      a.taps = g.k;
      a.dil = g.dil;
      a.Lout = L;
      a.ldy = g.cout;
      a.ylim = L * g.cout;
      a.lens = lens;
      if (!rbconv_handles(VE_ACT | VE_ACTIN, a)) return false;
    }
  }
  return true;
}

int Vocoder::stage_vconv(const char* P, int i, int B, int L, const char* X, const char* XA, char* XS, char* Tb,
                         char* R, char* RA, char* trash, bool act_out, hipStream_t st, const int* lens) const {
  const int nk = (int)rb_kernels.size();
  const bf16* zero = (const bf16*)(P + zero_off);
  // VE_ACTIN: conv1 activates the raw chain state in LDS, so neither the upsampler (XA) nor conv2 (RA) stores an
  // activated copy for it (the same bits: lrelu of the stored bf16 values either way)
  const bool actin = stage_actin(i, B, L, lens);
  int rc;
  if (stage_vp(i)) return pair_chain(P, i, B, L, X, XS, Tb, R, RA, trash, act_out, st, lens);
  for (int j = 0; j < nk; ++j) {
    if (rb_vp(i, j)) {  // this resblock as fused pairs (from the raw X), the others per layer (from XA)
      if ((rc = pair_resblock(P, i, j, B, L, X, XS, Tb, R, RA, trash, act_out, st, lens))) return rc;
      continue;
    }
    const std::vector<GemmW>& c1 = rb1[(size_t)i * nk + j];
    const std::vector<GemmW>& c2 = rb2[(size_t)i * nk + j];
    const int np = (int)c1.size();
    const char* state = X;
    const char* stateA = XA;
    for (int q = 0; q < np; ++q) {
      const bool last = q == np - 1;
      VConvArgs a{};
      a.x = (const bf16*)(actin ? state : stateA);
      a.B = B;
      a.L = L;
      a.cin = c1[q].cin;
      a.w = (const bf16*)(P + c1[q].v_off);
      a.bias = (const float*)(P + c1[q].b_off);
      a.M = a.Mpad = c1[q].cout;
      a.taps = c1[q].k;
      a.dil = c1[q].dil;
      a.pad = c1[q].pad;
      a.y = (bf16*)Tb;
      a.slope = 0.1f;
      a.div = 1.f;
      a.zero = zero;
      a.trash = (bf16*)trash;
      a.lens = lens;
      a.lmul = rate_upto(i + 1);
      if ((rc = launch_vconv(actin ? VE_ACT | VE_ACTIN : VE_ACT, a, st))) return rc;
      VConvArgs b = a;
      b.x = (const bf16*)Tb;
      b.w = (const bf16*)(P + c2[q].v_off);
      b.bias = (const float*)(P + c2[q].b_off);
      b.taps = c2[q].k;
      b.dil = c2[q].dil;
      b.pad = c2[q].pad;
      b.resid = (const bf16*)state;
      b.div = (float)nk;
      int ef = VE_RESID;
      if (!last) {
        b.y = (bf16*)R;
        if (!actin) {
          b.y2 = (bf16*)RA;
          ef |= VE_DUAL;
        }
        state = R;
        stateA = RA;
      } else {
        b.y = (bf16*)XS;
        if (j > 0) ef |= VE_ACCUM;
        if (j == nk - 1) ef |= VE_DIV;
        if (j == nk - 1 && act_out) {  // lrelu(xs) for the next upsampler, in RA (this pair's conv1 read it)
          b.y2 = (bf16*)RA;
          ef |= VE_DUAL | VE_Y2ONLY;  // the upsampler reads RA alone: the raw xs is dead (not stored)
        }
      }
      if ((rc = launch_vconv(ef, b, st))) return rc;
    }
  }
  return 0;
}

template <class E>
int Vocoder::forward_t(const char* P, const float* mel, int B, int T, float* wav, char* ws,
                       hipStream_t st, const int* lens) const {
  int rc;
  const size_t big = align256((size_t)B * T * frame_elems() * esize);
  char* XS = ws;
  char* X = ws + big;
  char* Tb = ws + 2 * big;
  char* R = ws + 3 * big;
  char* xm = ws + 4 * big;
  char* XA = ws + 4 * big + align256((size_t)B * T * n_mels * esize);
  char* RA = XA + big;
  char* trash = RA + big;  // 4 KiB (vconv stores of frames past L)
  if ((rc = bct_to_btc(dtype, mel, B, n_mels, T, 1.f, xm, n_mels, 0, st))) return rc;
  // ragged: mel frames past each utterance's length are conv_pre's zero padding
  if (lens && (rc = zero_tail_rows(dtype, xm, B, T, n_mels, lens, st))) return rc;
  // generic (fp32) path: the waveform past each utterance is zero (its conv_post tiles there exit unwritten)
  if (lens && !std::is_same<E, bf16>::value)
    MT_CHECK_HIP(hipMemsetAsync(wav, 0, (size_t)B * T * rate_upto((int)ups.size()) * sizeof(float), st));
  // the generic kernel's ragged lengths (ConvArgs::lens) at the input rate of each conv
  auto rag = [&](ConvArgs& c, int rate) {
    c.lens = lens;
    c.lmul = rate;
    c.fixed_tile = 1;  // batch-invariant rows: the tile choice may not depend on B
  };
  {
    ConvArgs a = gemm_args(pre, P, B, T);
    a.x0 = xm;
    a.y = XS;
    rag(a, 1);
    bool dual = false;
    if constexpr (std::is_same<E, bf16>::value) dual = ups_vc(0);
    if (dual) {  // + lrelu(xs) in RA, the first upsampler's vconv input
      a.y2 = RA;
      a.slope = 0.1f;
      if ((rc = launch_conv<E, 0, EF_DUAL>(a, st))) return rc;
    } else if ((rc = launch_conv<E, 0, 0>(a, st))) {
      return rc;
    }
  }
  int L = T;
  const int nk = (int)rb_kernels.size();
  for (size_t i = 0; i < ups.size(); ++i) {
    ConvArgs u = gemm_args(ups[i], P, B, L);
    u.x0 = XS;
    u.y = X;
    u.slope = 0.1f;
    rag(u, rate_upto((int)i));
    const int C = ups[i].cout;
    bool done_up = false;
    if constexpr (std::is_same<E, bf16>::value) {
      const bool svc = stage_vc((int)i);
      // the stage's per-layer conv1s activate their input themselves (VE_ACTIN) or read XA = lrelu(X)
      const bool noxa = stage_vp((int)i) || (svc && stage_actin((int)i, B, u.Tout, lens));
      if (ups_vc((int)i)) {  // polyphase vconv from lrelu(xs) (RA); + XA = lrelu(X) for a vconv stage
        if ((rc = ups_vconv(P, (int)i, B, L, RA, X, XA, svc && !noxa, trash, st, lens))) return rc;
        done_up = true;
      }
      if (svc) {
        // X and XA = lrelu(X): the three resblocks' first convs read XA (or, VE_ACTIN, X), their residual X
        if (!done_up) {
          u.y2 = XA;
          if ((rc = noxa ? launch_conv<E, PF_LRELU, 0>(u, st) : launch_conv<E, PF_LRELU, EF_DUAL>(u, st)))
            return rc;
        }
        L = u.Tout;
        const bool act_out = i + 1 < ups.size() && ups_vc((int)i + 1);
        if ((rc = stage_vconv(P, (int)i, B, L, X, XA, XS, Tb, R, RA, trash, act_out, st, lens))) return rc;
        continue;
      }
    }
    if (!done_up && (rc = launch_conv<E, PF_LRELU, 0>(u, st))) return rc;
    L = u.Tout;
    if constexpr (std::is_same<E, bf16>::value) {
      if (stage_vp32((int)i)) {
        const bool act_out = i + 1 < ups.size() && ups_vc((int)i + 1);
        if (post_fold((int)i) && !act_out) {
          // conv_post in the final pair's epilogue (VE_POST): the pair walks only each utterance's live tiles, so
          // the samples past them are zeroed here (post_conv_kernel wrote those zeros itself)
          if (lens) MT_CHECK_HIP(hipMemsetAsync(wav, 0, (size_t)B * L * sizeof(float), st));
          return pair_chain(P, (int)i, B, L, X, XS, Tb, R, RA, trash, act_out, st, lens, wav);
        }
        if ((rc = pair_chain(P, (int)i, B, L, X, XS, Tb, R, RA, trash, act_out, st, lens))) return rc;
        continue;
      }
    }
    bool uniform = true;
    for (const auto& dl : rb_dils) uniform = uniform && dl.size() == rb_dils[0].size();
    if (fuse && resblock == 1 && nk <= 3 && rbfuse_supported(dtype, C) && uniform && rb_dils[0].size() <= 3) {
      // whole stage in one launch: y = (sum_j resblock_j(x)) / nk, intermediates in LDS
      RBArgs r{};
      r.x = X;
      r.y = XS;
      r.B = B;
      r.L = L;
      r.nk = nk;
      r.npair = (int)rb_dils[0].size();
      r.slope = 0.1f;
      r.div = (float)nk;
      int hm = 0;
      for (int j = 0; j < nk; ++j) {
        const int q = (rb_kernels[j] - 1) / 2;
        int h = 0;
        for (int d : rb_dils[j]) h += q * d + q;
        hm = std::max(hm, h);
      }
      r.hmax = hm;
      const int N = rbfuse_tile_n(C);
      for (int j = 0; j < nk; ++j) {
        const int q = (rb_kernels[j] - 1) / 2;
        r.k[j] = rb_kernels[j];
        int A = hm, Bv = hm + N;  // rows each conv must produce, from the output backwards
        for (int p = r.npair - 1; p >= 0; --p) {
          const int d = rb_dils[j][p];
          r.dil[j][p] = d;
          r.c1[j][p] = RBConv{P + rb1[i * nk + j][p].w_off, (const float*)(P + rb1[i * nk + j][p].b_off)};
          r.c2[j][p] = RBConv{P + rb2[i * nk + j][p].w_off, (const float*)(P + rb2[i * nk + j][p].b_off)};
          r.r2a[j][p] = A;
          r.r2b[j][p] = Bv;
          r.r1a[j][p] = A - q;
          r.r1b[j][p] = Bv + q;
          A -= q + q * d;
          Bv += q + q * d;
        }
      }
      if ((rc = launch_rbfuse(dtype, C, r, st))) return rc;
      continue;
    }
    for (int j = 0; j < nk; ++j) {
      const std::vector<GemmW>& c1 = rb1[i * nk + j];
      const std::vector<GemmW>& c2 = rb2[i * nk + j];
      const int np = (int)c1.size();
      const bool acc = j > 0, div = j == nk - 1;
      const char* state = X;  // chain state entering each pair
      for (int q = 0; q < np; ++q) {
        const bool last = q == np - 1;
        const char* xin = state;
        // ResBlock1: the second conv reads Tb, so R may be updated in place. ResBlock2's conv
        // reads the chain state itself (with a halo), so it ping-pongs R <-> Tb.
        char* dst = last ? XS : (resblock == 1 ? R : (state == R ? Tb : R));
        state = dst;
        const char* src = xin;
        if (resblock == 1) {
          ConvArgs a = gemm_args(c1[q], P, B, L);
          a.x0 = xin;
          a.y = Tb;
          a.slope = 0.1f;
          rag(a, rate_upto((int)i + 1));
          if ((rc = launch_conv<E, PF_LRELU, 0>(a, st))) return rc;
          src = Tb;
        }
        const GemmW& g = resblock == 1 ? c2[q] : c1[q];
        ConvArgs b = gemm_args(g, P, B, L);
        b.x0 = src;
        b.y = dst;
        b.slope = 0.1f;
        rag(b, rate_upto((int)i + 1));
        b.resid = xin;
        b.ldr = g.cout;
        b.div = (float)nk;
        if (!last) {
          rc = launch_conv<E, PF_LRELU, EF_RESID>(b, st);
        } else if (acc && div) {
          rc = launch_conv<E, PF_LRELU, EF_RESID | EF_ACCUM | EF_DIV>(b, st);
        } else if (acc) {
          rc = launch_conv<E, PF_LRELU, EF_RESID | EF_ACCUM>(b, st);
        } else if (div) {
          rc = launch_conv<E, PF_LRELU, EF_RESID | EF_DIV>(b, st);
        } else {
          rc = launch_conv<E, PF_LRELU, EF_RESID>(b, st);
        }
        if (rc) return rc;
      }
    }
  }
  if constexpr (std::is_same<E, bf16>::value) {
    if (post.cin == 32 && post.k == 7 && post.cout == 1) {
      hipLaunchKernelGGL(post_conv_kernel, dim3((L + PC_N - 1) / PC_N, B), dim3(256), 0, st, (const bf16*)XS, L,
                         (const bf16*)(P + post.w_off), (const float*)(P + post.b_off), 0.01f, wav, lens,
                         rate_upto((int)ups.size()));
      MT_CHECK_HIP(hipGetLastError());
      return 0;
    }
  }
  ConvArgs c = gemm_args(post, P, B, L);
  c.x0 = XS;
  c.y = wav;
  rag(c, rate_upto((int)ups.size()));
  c.ldy = 1;
  c.slope = 0.01f;
  return launch_conv<E, PF_LRELU, EF_TANH | EF_OUTF32>(c, st);
}

bool Vocoder::ragged_supported() const {
  if (dtype != BF16) return true;  // the generic per-layer kernel everywhere (ConvArgs::lens)
  if (resblock != 1 || post.cin != 32 || post.k != 7 || post.cout != 1) return false;
  for (size_t i = 0; i < ups.size(); ++i)
    if (!ups_vc((int)i) || !(stage_vc((int)i) || stage_vp32((int)i))) return false;
  return true;
}

int Vocoder::forward(const void* packed, const float* mel, int B, int T, float* wav, void* ws, size_t ws_bytes,
                     hipStream_t st, const int* lens) const {
  MT_REQUIRE(B > 0 && T > 0, "vocoder: empty input");
  MT_REQUIRE(ws_bytes >= workspace_bytes(B, T), "vocoder: workspace %zu < %zu", ws_bytes,
             workspace_bytes(B, T));
  MT_REQUIRE(!lens || (ragged_supported() && B <= RAG_MAXB),
             "vocoder: per-utterance lengths need the bf16 vconv / pair path on every stage and B <= %d", RAG_MAXB);
  if (dtype == BF16) return forward_t<bf16>((const char*)packed, mel, B, T, wav, (char*)ws, st, lens);
  return forward_t<float>((const char*)packed, mel, B, T, wav, (char*)ws, st, lens);
}

}  // namespace mt
