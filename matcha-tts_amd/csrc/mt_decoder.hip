// U-Net estimator + CFM ODE solver driver (model.py:834-1048, 1084-1109).
//
// One estimator evaluation = 54 kernel launches on the caller's stream (all activations
// [B][T][C] in the element type, GN/LN statistics and the Euler state in fp32):
//   ResnetBlock1D  = K1 conv3(x*m)+GN-partials | K2 conv3((mish(GN(y1))+tb)*m)+GN-partials |
//                    K3 res1x1(x*m) + mish(GN(y2))*m
//   Transformer    = QKV(LN1 prologue) | attention | out-proj(+x) | FF1(LN3, SnakeBeta) | FF2(+x)
//   final          = final_block conv3 + GN-partials | final_proj(mish(GN)*m)*m fused with the
//                    Euler/midpoint update z += pred*dt written to the fp32 master and to the
//                    estimator input slot for the next evaluation.
#include <math.h>
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "mt_ffn.h"
#include "mt_model.h"
#include "mt_probe.h"
#include "mt_vconv.h"

namespace mt {

size_t align256(size_t x) { return (x + 255) & ~(size_t)255; }

static int g_deck = -1;
int dec_kernels() {
  if (g_deck < 0) {
    const char* e = getenv("MT_DECK");
    g_deck = e ? atoi(e) & DECK_ALL : DECK_ALL;
  }
  return g_deck;
}
int dec_set_kernels(int mask) {
  const int prev = dec_kernels();
  g_deck = mask & DECK_ALL;
  return prev;
}

static int round_up(int x, int m) { return (x + m - 1) / m * m; }

GemmW make_conv(int cout, int cin, int k, int stride, int pad, int dil, std::vector<int> w, int b,
                int esize, Packer& pk) {
  GemmW g;
  g.kind = 0;
  g.cin = cin;
  g.cout = cout;
  g.k = k;
  g.s = stride;
  g.pad = pad;
  g.dil = dil;
  g.M = cout;
  g.Mpad = round_up(cout, 16);
  g.taps = k;
  g.cin_pad = round_up(cin, 64 / esize);
  g.gpad = pad;
  g.ups = 1;
  g.opad = 0;
  g.wsrc = std::move(w);
  g.bsrc = b;
  g.w_off = pk.take((size_t)g.Mpad * g.taps * g.cin_pad * esize);
  g.b_off = pk.take((size_t)g.M * sizeof(float));
  return g;
}

GemmW make_convT(int cin, int cout, int k, int s, int pad, int w, int b, int esize, Packer& pk) {
  GemmW g;
  g.kind = 1;
  g.cin = cin;
  g.cout = cout;
  g.k = k;
  g.s = s;
  g.pad = pad;
  g.dil = 1;
  g.M = s * cout;
  g.Mpad = round_up(g.M, 16);
  g.taps = k / s;
  g.cin_pad = round_up(cin, 64 / esize);
  g.gpad = g.taps - 1;
  g.ups = s;
  g.opad = pad;
  g.wsrc = {w};
  g.bsrc = b;
  g.w_off = pk.take((size_t)g.Mpad * g.taps * g.cin_pad * esize);
  g.b_off = pk.take((size_t)g.M * sizeof(float));
  return g;
}

int pack_gemm(const GemmW& g, int dtype, const float* const* params, char* P, hipStream_t st) {
  int rc;
  void* wdst = P + g.w_off;
  const float* colscale = g.ln_g >= 0 ? params[g.ln_g] : nullptr;
  if (g.kind == 0) {
    const int rows_per = g.cout / (int)g.wsrc.size();
    for (size_t i = 0; i < g.wsrc.size(); ++i) {
      rc = pack_conv(dtype, params[g.wsrc[i]], 0, rows_per, g.cin, g.k, 1, (int)i * rows_per, rows_per,
                     g.Mpad, g.taps, g.cin_pad, wdst, st, colscale);
      if (rc) return rc;
    }
    const int rest = g.Mpad - g.cout;  // zero pad rows
    if (rest > 0) {
      rc = pack_conv(dtype, nullptr, 0, 0, g.cin, g.k, 1, g.cout, rest, g.Mpad, g.taps, g.cin_pad, wdst, st);
      if (rc) return rc;
    }
  } else {
    rc = pack_conv(dtype, params[g.wsrc[0]], 1, g.cout, g.cin, g.k, g.s, 0, g.Mpad, g.Mpad, g.taps,
                   g.cin_pad, wdst, st);
    if (rc) return rc;
  }
  if (!g.bsrcs.empty()) {
    const int rows_per = g.cout / (int)g.bsrcs.size();
    for (size_t i = 0; i < g.bsrcs.size(); ++i) {
      rc = pack_vec(params[g.bsrcs[i]], rows_per, rows_per, 0, (float*)(P + g.b_off) + i * rows_per, st);
      if (rc) return rc;
    }
  } else {
    rc = pack_vec(g.bsrc >= 0 ? params[g.bsrc] : nullptr, g.cout, g.M, 0, (float*)(P + g.b_off), st);
    if (rc) return rc;
  }
  if (g.ln_b >= 0) {  // LN(x) = x_hat*gamma + beta  ->  W(gamma) x_hat + (b + W beta)
    const int rows_per = g.cout / (int)g.wsrc.size();
    for (size_t i = 0; i < g.wsrc.size(); ++i) {
      rc = fold_bias(params[g.wsrc[i]], params[g.ln_b], rows_per, g.cin, (float*)(P + g.b_off) + i * rows_per, st);
      if (rc) return rc;
    }
  }
  return 0;
}

void gemm_geom(const GemmW& g, int Tin, int* Tout, int* Ncols) {
  if (g.kind == 0) {
    *Tout = (Tin + 2 * g.pad - g.dil * (g.k - 1) - 1) / g.s + 1;
    *Ncols = *Tout;
  } else {
    *Tout = (Tin - 1) * g.s - 2 * g.pad + g.k;
    *Ncols = (*Tout - 1 + g.pad) / g.s + 1;
  }
}

ConvArgs gemm_args(const GemmW& g, const char* P, int B, int Tin) {
  ConvArgs a{};
  a.B = B;
  a.Tin = Tin;
  a.c0 = a.cin = g.cin;
  a.w = P + g.w_off;
  a.bias = (const float*)(P + g.b_off);
  a.M = g.M;
  a.Mpad = g.Mpad;
  a.cout = g.cout;
  a.taps = g.taps;
  a.dil = g.dil;
  a.pad = g.gpad;
  a.stride = g.kind == 0 ? g.s : 1;
  a.cin_pad = g.cin_pad;
  a.ups = g.ups;
  a.opad = g.opad;
  gemm_geom(g, Tin, &a.Tout, &a.Ncols);
  a.ldy = g.cout;
  a.slope = 0.1f;
  a.ln_eps = 1e-5f;
  a.gn_eps = 1e-5f;
  a.div = 1.f;
  return a;
}

// -------------------------------------------------------------------------------------
int Decoder::init(int c_cond_, int n_mid_, int n_blocks_, int heads_, int dtype_) {
  MT_REQUIRE(c_cond_ % 32 == 0 && c_cond_ >= 160, "decoder: c_cond %d must be a multiple of 32 >= 160",
             c_cond_);
  MT_REQUIRE(n_mid_ >= 0 && n_blocks_ >= 1 && heads_ >= 1 && heads_ <= 8, "decoder: bad config");
  MT_REQUIRE(dtype_ == F32 || dtype_ == BF16, "decoder: dtype");
  c_cond = c_cond_;
  n_mid = n_mid_;
  n_blocks = n_blocks_;
  heads = heads_;
  dtype = dtype_;
  esize = dtype == BF16 ? 2 : 4;
  inner = heads * 64;
  n_res = 4 + n_mid;
  Packer pk;
  ParamList& L = params;
  L = ParamList();
  res.clear();
  tbs.clear();
  const long long Cc = c_cond;

  t1w = L.add("time_mlp.linear_1.weight", {TE, Cc});
  t1b = L.add("time_mlp.linear_1.bias", {TE});
  t2w = L.add("time_mlp.linear_2.weight", {TE, TE});
  t2b = L.add("time_mlp.linear_2.bias", {TE});
  freq = L.add("_sinus_freq", {Cc / 2});  // exp(arange(half) * -ln(1e4)/(half-1)), host-computed
  t1w_off = pk.take((size_t)TE * Cc * 4);
  t1b_off = pk.take(TE * 4);
  t2w_off = pk.take((size_t)TE * TE * 4);
  t2b_off = pk.take(TE * 4);
  freq_off = pk.take(Cc / 2 * 4);

  // bf16 convs mt_vconv serves (stride 1, C_in % 64 == 0) get its [cin/64][taps][M][64] image too
  // (the first ResnetBlock reads x ‖ mu ‖ spk, c_cond channels: its image takes the input zero-padded to a
  // multiple of 64, which is how the vconv path stores that input)
  auto vcify = [&](GemmW& g) {
    const int ci = (g.cin + 63) / 64 * 64;
    if (dtype == BF16 && g.kind == 0 && vconv_supported(ci, g.cout, g.k, g.dil, g.s)) {
      g.vc = true;
      g.vcin = ci != g.cin ? ci : 0;
      g.v_off = pk.take(vconv_packed_bytes(ci, g.cout, g.k));
    }
  };
  auto add_res = [&](const std::string& p, int dim_in) {
    Res R;
    R.dim_in = dim_in;
    R.mlp_w = L.add(p + ".mlp.1.weight", {C, TE});
    R.mlp_b = L.add(p + ".mlp.1.bias", {C});
    int w1 = L.add(p + ".block1.block.0.weight", {C, dim_in, 3});
    int b1 = L.add(p + ".block1.block.0.bias", {C});
    R.gn1g = L.add(p + ".block1.block.1.weight", {C});
    R.gn1b = L.add(p + ".block1.block.1.bias", {C});
    int w2 = L.add(p + ".block2.block.0.weight", {C, C, 3});
    int b2 = L.add(p + ".block2.block.0.bias", {C});
    R.gn2g = L.add(p + ".block2.block.1.weight", {C});
    R.gn2b = L.add(p + ".block2.block.1.bias", {C});
    int wr = L.add(p + ".res_conv.weight", {C, dim_in, 1});
    int br = L.add(p + ".res_conv.bias", {C});
    R.c1 = make_conv(C, dim_in, 3, 1, 1, 1, {w1}, b1, esize, pk);
    R.c2 = make_conv(C, C, 3, 1, 1, 1, {w2}, b2, esize, pk);
    R.res = make_conv(C, dim_in, 1, 1, 0, 1, {wr}, br, esize, pk);
    vcify(R.c1);
    vcify(R.c2);
    vcify(R.res);
    R.gn1_off = pk.take(2 * C * 4);
    R.gn2_off = pk.take(2 * C * 4);
    R.mlp_w_off = pk.take((size_t)C * TE * 4);
    R.mlp_b_off = pk.take(C * 4);
    res.push_back(R);
  };
  auto add_tbs = [&](const std::string& p) {
    std::vector<TB> v;
    for (int j = 0; j < n_blocks; ++j) {
      const std::string q = p + "." + std::to_string(j);
      TB t;
      t.ln1g = L.add(q + ".norm1.weight", {C});
      t.ln1b = L.add(q + ".norm1.bias", {C});
      int wq = L.add(q + ".attn1.to_q.weight", {inner, C});
      int wk = L.add(q + ".attn1.to_k.weight", {inner, C});
      int wv = L.add(q + ".attn1.to_v.weight", {inner, C});
      int wo = L.add(q + ".attn1.to_out.0.weight", {C, inner});
      int bo = L.add(q + ".attn1.to_out.0.bias", {C});
      t.ln3g = L.add(q + ".norm3.weight", {C});
      t.ln3b = L.add(q + ".norm3.bias", {C});
      int w1 = L.add(q + ".ff.net.0.proj.weight", {TE, C});
      int b1 = L.add(q + ".ff.net.0.proj.bias", {TE});
      t.alpha = L.add(q + ".ff.net.0.alpha", {TE});
      t.beta = L.add(q + ".ff.net.0.beta", {TE});
      int w2 = L.add(q + ".ff.net.2.weight", {C, TE});
      int b2 = L.add(q + ".ff.net.2.bias", {C});
      t.qkv = make_conv(3 * inner, C, 1, 1, 0, 1, {wq, wk, wv}, -1, esize, pk);
      t.qkv.ln_g = t.ln1g;
      t.qkv.ln_b = t.ln1b;
      t.out = make_conv(C, inner, 1, 1, 0, 1, {wo}, bo, esize, pk);
      t.ff1 = make_conv(TE, C, 1, 1, 0, 1, {w1}, b1, esize, pk);
      t.ff1.ln_g = t.ln3g;
      t.ff1.ln_b = t.ln3b;
      t.ff2 = make_conv(C, TE, 1, 1, 0, 1, {w2}, b2, esize, pk);
      t.ln1_off = pk.take(2 * C * 4);
      t.ln3_off = pk.take(2 * C * 4);
      t.snake_off = pk.take(2 * TE * 4);
      if (dtype == BF16) {  // the transformer-block GEMMs run on mt_vconv's 1x1 pipeline
        for (GemmW* g : {&t.qkv, &t.out, &t.ff1, &t.ff2}) {
          g->vc = vconv_supported(g->cin, g->cout, 1, 1, 1);
          if (g->vc) g->v_off = pk.take(vconv_packed_bytes(g->cin, g->cout, 1));
        }
        t.wsq_off = pk.take((size_t)t.qkv.cout * 4);
        t.wsf_off = pk.take((size_t)t.ff1.cout * 4);
      }
      v.push_back(t);
    }
    tbs.push_back(v);
  };

  // down blocks (channels = (256, 256))
  add_res("down_blocks.0.0", c_cond);
  add_tbs("down_blocks.0.1");
  {
    int w = L.add("down_blocks.0.2.conv.weight", {C, C, 3});
    int b = L.add("down_blocks.0.2.conv.bias", {C});
    down0 = make_conv(C, C, 3, 2, 1, 1, {w}, b, esize, pk);
    if (dtype == BF16 && vconv_supported(2 * C, C, 2, 1, 1)) {  // stride 2 as a 2-tap conv over frame pairs
      down0.vc = true;
      down0.vcin = 2 * C;
      down0.v_off = pk.take(vconv_packed_bytes(2 * C, C, 2));
    }
  }
  add_res("down_blocks.1.0", C);
  add_tbs("down_blocks.1.1");
  {
    int w = L.add("down_blocks.1.2.weight", {C, C, 3});
    int b = L.add("down_blocks.1.2.bias", {C});
    down1 = make_conv(C, C, 3, 1, 1, 1, {w}, b, esize, pk);
    vcify(down1);
  }
  for (int i = 0; i < n_mid; ++i) {
    add_res("mid_blocks." + std::to_string(i) + ".0", C);
    add_tbs("mid_blocks." + std::to_string(i) + ".1");
  }
  add_res("up_blocks.0.0", 2 * C);
  add_tbs("up_blocks.0.1");
  {
    int w = L.add("up_blocks.0.2.conv.weight", {C, C, 4});
    int b = L.add("up_blocks.0.2.conv.bias", {C});
    up0 = make_convT(C, C, 4, 2, 1, w, b, esize, pk);
    if (dtype == BF16 && up0.M <= 1024 && vconv_supported(C, up0.M, up0.taps, 1, 1)) {  // polyphase, placed output
      up0.vc = true;
      up0.vrows = up0.M;
      up0.v_off = pk.take(vconv_packed_bytes(C, up0.M, up0.taps));
    }
  }
  add_res("up_blocks.1.0", 2 * C);
  add_tbs("up_blocks.1.1");
  {
    int w = L.add("up_blocks.1.2.weight", {C, C, 3});
    int b = L.add("up_blocks.1.2.bias", {C});
    up1 = make_conv(C, C, 3, 1, 1, 1, {w}, b, esize, pk);
    vcify(up1);
  }
  {
    int w = L.add("final_block.block.0.weight", {C, C, 3});
    int b = L.add("final_block.block.0.bias", {C});
    fgn_g = L.add("final_block.block.1.weight", {C});
    fgn_b = L.add("final_block.block.1.bias", {C});
    fconv = make_conv(C, C, 3, 1, 1, 1, {w}, b, esize, pk);
    vcify(fconv);
    fgn_off = pk.take(2 * C * 4);
    int wp = L.add("final_proj.weight", {NF, C, 1});
    int bp = L.add("final_proj.bias", {NF});
    fproj = make_conv(NF, C, 1, 1, 0, 1, {wp}, bp, esize, pk);
  }
  zero_off = pk.take(256);
  packed_bytes = pk.off;
  return 0;
}

int Decoder::pack(const float* const* p, void* packed, hipStream_t st) const {
  char* P = (char*)packed;
  int rc;
#define PK(expr) \
  if ((rc = (expr)) != 0) return rc
  PK(pack_vec(p[t1w], TE * c_cond, TE * c_cond, 0, (float*)(P + t1w_off), st));
  PK(pack_vec(p[t1b], TE, TE, 0, (float*)(P + t1b_off), st));
  PK(pack_vec(p[t2w], TE * TE, TE * TE, 0, (float*)(P + t2w_off), st));
  PK(pack_vec(p[t2b], TE, TE, 0, (float*)(P + t2b_off), st));
  PK(pack_vec(p[freq], c_cond / 2, c_cond / 2, 0, (float*)(P + freq_off), st));
  for (size_t r = 0; r < res.size(); ++r) {
    const Res& R = res[r];
    PK(pack_gemm(R.c1, dtype, p, P, st));
    PK(pack_gemm(R.c2, dtype, p, P, st));
    PK(pack_gemm(R.res, dtype, p, P, st));
    for (const GemmW* g : {&R.c1, &R.c2, &R.res})
      if (g->vc)
        PK(vconv_repack(P + g->w_off, g->Mpad, g->taps, g->cin_pad, g->vcin ? g->vcin : g->cin, g->cout,
                        P + g->v_off, st, g->cin));
    PK(pack_vec(p[R.gn1g], C, C, 0, (float*)(P + R.gn1_off), st));
    PK(pack_vec(p[R.gn1b], C, C, 0, (float*)(P + R.gn1_off) + C, st));
    PK(pack_vec(p[R.gn2g], C, C, 0, (float*)(P + R.gn2_off), st));
    PK(pack_vec(p[R.gn2b], C, C, 0, (float*)(P + R.gn2_off) + C, st));
    PK(pack_vec(p[R.mlp_w], C * TE, C * TE, 0, (float*)(P + R.mlp_w_off), st));
    PK(pack_vec(p[R.mlp_b], C, C, 0, (float*)(P + R.mlp_b_off), st));
    for (const TB& t : tbs[r]) {
      PK(pack_gemm(t.qkv, dtype, p, P, st));
      PK(pack_gemm(t.out, dtype, p, P, st));
      PK(pack_gemm(t.ff1, dtype, p, P, st));
      PK(pack_gemm(t.ff2, dtype, p, P, st));
      PK(pack_vec(p[t.ln1g], C, C, 0, (float*)(P + t.ln1_off), st));
      PK(pack_vec(p[t.ln1b], C, C, 0, (float*)(P + t.ln1_off) + C, st));
      PK(pack_vec(p[t.ln3g], C, C, 0, (float*)(P + t.ln3_off), st));
      PK(pack_vec(p[t.ln3b], C, C, 0, (float*)(P + t.ln3_off) + C, st));
      PK(pack_vec(p[t.alpha], TE, TE, 1, (float*)(P + t.snake_off), st));
      PK(pack_vec(p[t.beta], TE, TE, 2, (float*)(P + t.snake_off) + TE, st));
      for (const GemmW* g : {&t.qkv, &t.out, &t.ff1, &t.ff2})
        if (g->vc) PK(vconv_repack(P + g->w_off, g->Mpad, g->taps, g->cin_pad, g->cin, g->cout, P + g->v_off, st));
      if (t.qkv.vc) PK(vconv_wsum(P + t.qkv.v_off, t.qkv.cin, 1, t.qkv.cout, (float*)(P + t.wsq_off), st));
      if (t.ff1.vc) PK(vconv_wsum(P + t.ff1.v_off, t.ff1.cin, 1, t.ff1.cout, (float*)(P + t.wsf_off), st));
    }
  }
  PK(pack_vec(nullptr, 1, 64, 0, (float*)(P + zero_off), st));
  PK(pack_gemm(down0, dtype, p, P, st));
  if (down0.vc) PK(vconv_repack_s2(P + down0.w_off, down0.cin_pad, C, C, P + down0.v_off, st));
  PK(pack_gemm(down1, dtype, p, P, st));
  PK(pack_gemm(up0, dtype, p, P, st));
  if (up0.vc) PK(vconv_repack(P + up0.w_off, up0.vrows, up0.taps, up0.cin_pad, up0.cin, up0.vrows, P + up0.v_off, st));
  PK(pack_gemm(up1, dtype, p, P, st));
  PK(pack_gemm(fconv, dtype, p, P, st));
  PK(pack_vec(p[fgn_g], C, C, 0, (float*)(P + fgn_off), st));
  PK(pack_vec(p[fgn_b], C, C, 0, (float*)(P + fgn_off) + C, st));
  PK(pack_gemm(fproj, dtype, p, P, st));
  for (const GemmW* g : {&down1, &up1, &fconv})
    if (g->vc) PK(vconv_repack(P + g->w_off, g->Mpad, g->taps, g->cin_pad, g->cin, g->cout, P + g->v_off, st));
#undef PK
  return 0;
}

size_t Decoder::workspace_bytes(int B, int T, int S) const {
  const size_t BT = (size_t)B * T;
  // GroupNorm partial slots: generic conv tiles of 64 frames or vconv tiles x waves, whichever is more
  const size_t ntl = (size_t)std::max((T + 63) / 64, vconv_gn_parts_max(T));
  size_t n = 0;
  n += align256(BT * ((c_cond + 63) / 64 * 64) * esize);  // xin (row stride xld())
  n += 8 * align256(BT * C * esize);                  // H0 H1 XA XB XC U XF + y1
  n += align256(BT * C * esize);                      // y2
  n += align256(BT * 3 * inner * esize);              // qkv
  n += align256(BT * inner * esize);                  // ob
  n += align256(BT * TE * esize);                     // ff
  n += align256(BT * NF * 4);                         // zm
  n += align256(BT * 2 * 4);                          // lns (LayerNorm row stats)
  n += align256((size_t)B * ((T + 1) / 2) * 4);       // m1
  n += 2 * align256((size_t)B * 8 * ntl * 2 * 8);     // gn1 gn2
  n += align256((size_t)S * c_cond * 4);              // emb
  n += 2 * align256((size_t)S * TE * 4);              // h1 h2
  n += align256((size_t)S * n_res * C * 4);           // tb
  n += 4096;                                          // trash (vconv stores past the last frame)
  n += align256(attention_part_bytes(B, T, heads));   // attention key-split slots
  n += align256(BT * (C / 64) * 2 * 4);               // lnp
  n += align256(uniform_attention_floats(B) * 4);     // upart
  n += align256(BT * 4);                              // mst
  return n;
}

Decoder::Work Decoder::carve(void* ws, int B, int T, int S) const {
  const size_t BT = (size_t)B * T;
  const size_t ntl = (size_t)std::max((T + 63) / 64, vconv_gn_parts_max(T));
  char* p = (char*)ws;
  auto take = [&](size_t bytes) {
    char* r = p;
    p += align256(bytes);
    return r;
  };
  Work w;
  w.xin = take(BT * ((c_cond + 63) / 64 * 64) * esize);
  w.H0 = take(BT * C * esize);
  w.H1 = take(BT * C * esize);
  w.XA = take(BT * C * esize);
  w.XB = take(BT * C * esize);
  w.XC = take(BT * C * esize);
  w.U = take(BT * C * esize);
  w.XF = take(BT * C * esize);
  w.y1 = take(BT * C * esize);
  w.y2 = take(BT * C * esize);
  w.qkv = take(BT * 3 * inner * esize);
  w.ob = take(BT * inner * esize);
  w.ff = take(BT * TE * esize);
  w.zm = (float*)take(BT * NF * 4);
  w.lns = (float*)take(BT * 2 * 4);
  w.m1 = (float*)take((size_t)B * ((T + 1) / 2) * 4);
  w.gn1 = (double*)take((size_t)B * 8 * ntl * 2 * 8);
  w.gn2 = (double*)take((size_t)B * 8 * ntl * 2 * 8);
  w.emb = (float*)take((size_t)S * c_cond * 4);
  w.h1 = (float*)take((size_t)S * TE * 4);
  w.h2 = (float*)take((size_t)S * TE * 4);
  w.tb = (float*)take((size_t)S * n_res * C * 4);
  w.trash = take(4096);
  w.tb_ld = 0;
  w.apart = (float*)take(attention_part_bytes(B, T, heads));
  w.lnp = (float*)take(BT * (C / 64) * 2 * 4);
  w.upart = (float*)take(uniform_attention_floats(B) * 4);
  w.mst = (float*)take(BT * 4);
  w.m0 = nullptr;
  return w;
}

int Decoder::time_embed(const char* P, const Work& w, const TimeSched& ts, int S, hipStream_t st,
                        const float* t_dev) const {
  int rc;
  if ((rc = sinus_embed(ts, S, (const float*)(P + freq_off), c_cond / 2, w.emb, st, t_dev))) return rc;
  if ((rc = rowdot(w.emb, c_cond, (const float*)(P + t1w_off), (const float*)(P + t1b_off), w.h1, TE, 0, S,
                   TE, c_cond, 0, 1, st)))
    return rc;
  // h2 is only ever read through the ResnetBlocks' Mish (model.py mlp = Mish -> Linear): store mish(h2)
  if ((rc = rowdot(w.h1, TE, (const float*)(P + t2w_off), (const float*)(P + t2b_off), w.h2, TE, 0, S, TE, TE,
                   0, 2, st)))
    return rc;
  // every ResnetBlock's time projection (model.py mlp: Linear(TE, C) on mish(h2)) in one launch per 8 blocks
  for (int r0 = 0; r0 < n_res; r0 += ROWDOT_MAXSEG) {
    RowdotSegs sg{};
    sg.n = std::min(ROWDOT_MAXSEG, n_res - r0);
    for (int j = 0; j < sg.n; ++j) {
      sg.W[j] = (const float*)(P + res[r0 + j].mlp_w_off);
      sg.b[j] = (const float*)(P + res[r0 + j].mlp_b_off);
      sg.yoff[j] = (r0 + j) * C;
    }
    if ((rc = rowdot_segs(w.h2, TE, sg, w.tb, n_res * C, S, C, TE, 0, 0, st))) return rc;
  }
  return 0;
}

VConvArgs Decoder::vargs(const GemmW& g, const char* P, const Work& w, const void* x, int B, int Tl,
                         void* y) const {
  VConvArgs a{};
  a.x = (const bf16*)x;
  a.B = B;
  a.L = Tl;
  a.cin = g.vcin ? g.vcin : g.cin;
  a.w = (const bf16*)(P + g.v_off);
  a.bias = (const float*)(P + g.b_off);
  a.M = a.Mpad = g.cout;
  a.taps = g.k;
  a.dil = g.dil;
  a.pad = g.pad;
  a.y = (bf16*)y;
  a.div = 1.f;
  a.slope = 0.f;
  a.zero = (const bf16*)(P + zero_off);
  a.trash = (bf16*)w.trash;
  a.ln_stats = w.lns;
  a.ln_eps = 1e-5f;
  a.probe = PROBE_VCONV_DEC;
  return a;
}

// ResnetBlock1D (model.py ResnetBlock1D / Block1D): out = block2(block1(x*m) + mlp(t)) * m + res(x*m)
// Generic kernels: K1 conv3 with the input mask in its prologue + GN partials, K2 conv3 with GN/Mish/tb/mask
// in its prologue + GN partials, K3 res 1x1 + mish(GN(y2))*m in its epilogue. On vconv (bf16, x already
// masked by its producer): conv3 + GN partials -> gn_apply -> conv3 + GN partials -> gn_apply -> res 1x1
// with the block output as its residual.
template <class E>
int Decoder::resnet(const char* P, const Work& w, const Res& R, const void* x0, const void* x1, int c0,
                    int cin, bool x_masked, void* out, const float* mask, int B, int Tl, const float* tb,
                    bool* row_stats, hipStream_t st) const {
  int rc, nt1 = 0, nt2 = 0;
  *row_stats = false;
  const float* g1 = (const float*)(P + R.gn1_off);
  const float* g2 = (const float*)(P + R.gn2_off);
  // block 1 -> y1 + gn1
  if (x_masked && vc(R.c1)) {
    VConvArgs a = vargs(R.c1, P, w, x0, B, Tl, w.y1);
    a.x1 = (const bf16*)x1;
    a.c0 = c0;
    a.cin = cin;
    a.gn_out = w.gn1;
    nt1 = a.gn_parts = vconv_gn_parts(B, Tl, C);
    if ((rc = launch_vconv(VE_GNSTATS, a, st))) return rc;
  } else {
    ConvArgs a = gemm_args(R.c1, P, B, Tl);
    a.x0 = x0;
    a.x1 = x1;
    a.c0 = c0;
    a.cin = cin;
    a.y = w.y1;
    a.pmask = mask;
    a.gn_out = w.gn1;
    if ((rc = launch_conv<E, PF_MASK, EF_GNSTATS>(a, st, &nt1))) return rc;
  }
  // block 2 -> y2 + gn2 (generic) or y1 + gn2 (vconv, its input h1 in y2)
  const void* yb2 = w.y2;
  if (vc(R.c2)) {
    if ((rc = gn_apply(w.y1, B, Tl, C, w.gn1, nt1, g1, g1 + C, 1e-5f, tb, w.tb_ld, mask, w.y2, st))) return rc;
    VConvArgs b = vargs(R.c2, P, w, w.y2, B, Tl, w.y1);
    b.gn_out = w.gn2;
    nt2 = b.gn_parts = vconv_gn_parts(B, Tl, C);
    if ((rc = launch_vconv(VE_GNSTATS, b, st))) return rc;
    yb2 = w.y1;
  } else {
    ConvArgs b = gemm_args(R.c2, P, B, Tl);
    b.x0 = w.y1;
    b.y = w.y2;
    b.pmask = mask;
    b.gn_in = w.gn1;
    b.gn_ntiles = nt1;
    b.gn_T = Tl;
    b.gn_g = g1;
    b.gn_b = g1 + C;
    b.tb = tb;
    b.tb_ld = w.tb_ld;
    b.gn_out = w.gn2;
    if ((rc = launch_conv<E, PF_GN | PF_TB | PF_MASK, EF_GNSTATS>(b, st, &nt2))) return rc;
  }
  // residual 1x1 + block output
  if (x_masked && vc(R.res)) {
    VConvArgs c = vargs(R.res, P, w, x0, B, Tl, out);
    c.x1 = (const bf16*)x1;
    c.c0 = c0;
    c.cin = cin;
    c.row_out = w.lnp;  // the LayerNorm partials of the transformer block that reads `out`
    *row_stats = true;
    if (vc(R.c2) && gnres && Tl >= vconv_gnres_min_frames()) {
      // block 2's GroupNorm + Mish + mask applied in this conv's epilogue to the raw conv output (no gn_apply)
      c.resid = (const bf16*)yb2;
      c.gn_in = w.gn2;
      c.gn_in_parts = nt2;
      c.gn_T = Tl;
      c.gn_B = B;
      c.gn_gamma = g2;
      c.gn_beta = g2 + C;
      c.gn_eps = 1e-5f;
      c.emask = mask;
      return launch_vconv(VE_RESID | VE_ROWSTATS | VE_GNRES, c, st);
    }
    if ((rc = gn_apply(yb2, B, Tl, C, w.gn2, nt2, g2, g2 + C, 1e-5f, nullptr, 0, mask, w.y2, st))) return rc;
    c.resid = (const bf16*)w.y2;
    return launch_vconv(VE_RESID | VE_ROWSTATS, c, st);
  }
  ConvArgs c = gemm_args(R.res, P, B, Tl);
  c.x0 = x0;
  c.x1 = x1;
  c.c0 = c0;
  c.cin = cin;
  c.y = out;
  c.pmask = mask;
  c.emask = mask;
  c.gy = yb2;
  c.gn_in = w.gn2;
  c.gn_ntiles = nt2;
  c.gn_T = Tl;
  c.gn_g = g2;
  c.gn_b = g2 + C;
  return launch_conv<E, PF_MASK, EF_GNADD>(c, st);
}

template <class E>
int Decoder::tblock(const char* P, const Work& w, const TB& t, void* x, const float* mask, bool mask_out,
                    bool row_stats, bool uni, int B, int Tl, hipStream_t st) const {
  int rc;
  if constexpr (std::is_same<E, bf16>::value) {
    if (t.qkv.vc && t.out.vc && t.ff1.vc && t.ff2.vc) {
      // bf16: the four GEMMs on mt_vconv's 1x1 pipeline; LayerNorm folded into the QKV / FF1 epilogues
      auto vargs = [&](const GemmW& g, const void* xin, void* y) { return this->vargs(g, P, w, xin, B, Tl, y); };
      // ff(norm3(x)) + x: one fused launch (mt_ffn: the 1024-wide intermediate stays on chip), or FF1 + FF2 on
      // mt_vconv (MT_FFN=0); LayerNorm statistics: the per-slab partials in w.lnp either way
      const bool fused_ff = ffn_on() && B * Tl >= ffn_min_frames() && t.ff1.cin == C && t.ff1.cout == TE && t.ff2.cin == TE && t.ff2.cout == C;
      // ovec: the uniform attention's o_b, added by the fused kernel itself (its x += o_b launch skipped)
      auto feedforward = [&](const float* ovec) -> int {
        if (fused_ff) {
          FfnArgs f{};
          f.ovec = ovec;
          f.T = Tl;
          f.x = (bf16*)x;
          f.frames = B * Tl;
          f.ln_stats = w.lnp;
          f.ln_eps = 1e-5f;
          f.w1 = (const bf16*)(P + t.ff1.v_off);
          f.b1 = (const float*)(P + t.ff1.b_off);
          f.wsum = (const float*)(P + t.wsf_off);
          f.alpha = (const float*)(P + t.snake_off);
          f.ibeta = (const float*)(P + t.snake_off) + TE;
          f.w2 = (const bf16*)(P + t.ff2.v_off);
          f.b2 = (const float*)(P + t.ff2.b_off);
          f.emask = mask_out ? mask : nullptr;
          f.zero = (const bf16*)(P + zero_off);
          f.trash = (bf16*)w.trash;
          return launch_ffn(f, st);
        }
        VConvArgs f1 = vargs(t.ff1, x, w.ff);
        f1.ln_stats = w.lnp;
        f1.wsum = (const float*)(P + t.wsf_off);
        f1.snake_alpha = (const float*)(P + t.snake_off);
        f1.snake_ibeta = (const float*)(P + t.snake_off) + TE;
        int rc1;
        if ((rc1 = launch_vconv(VE_LN | VE_LNP | VE_SNAKE, f1, st))) return rc1;
        VConvArgs f2 = vargs(t.ff2, w.ff, x);
        f2.resid = (const bf16*)x;
        // the chain's last block hands its consumers (convs reading x * mask) a masked copy in place
        f2.emask = mask;
        return launch_vconv(mask_out ? VE_RESID | VE_MASK : VE_RESID, f2, st);
      };
      if (uni && heads == 2 && t.qkv.cout == 384 && t.qkv.cin == C && t.out.cout == C && t.out.cin == 128) {
        // every utterance is padded at this level: attention is query-independent (model.py:697) -> x += o_b
        // with o_b from a masked mean and two GEMVs; no QKV GEMM, no attention, no per-frame out-projection
        if ((rc = launch_uniform_attention(x, mask, B, Tl, P + t.qkv.v_off, t.qkv.cout, (const float*)(P + t.qkv.b_off),
                                           P + t.out.v_off, (const float*)(P + t.out.b_off), w.upart, w.lnp, st,
                                           !fused_ff)))
          return rc;
        return feedforward(fused_ff ? uniform_attention_ovec(w.upart, B) : nullptr);
      }
      // LayerNorm statistics: per-slab partials from the producing conv's epilogue (VE_ROWSTATS) when it
      // wrote them, else a row-statistics pass
      VConvArgs q = vargs(t.qkv, x, w.qkv);
      q.wsum = (const float*)(P + t.wsq_off);
      if (row_stats) {
        q.ln_stats = w.lnp;
        if ((rc = launch_vconv(VE_LN | VE_LNP, q, st))) return rc;
      } else {
        if ((rc = rowstats(dtype, x, B * Tl, C, 1e-5f, w.lns, st))) return rc;
        if ((rc = launch_vconv(VE_LN, q, st))) return rc;
      }
      if ((rc = launch_attention(dtype, w.qkv, mask, w.ob, B, Tl, heads, st, w.apart))) return rc;
      VConvArgs o = vargs(t.out, w.ob, x);
      o.resid = (const bf16*)x;
      o.row_out = w.lnp;
      if ((rc = launch_vconv(VE_RESID | VE_ROWSTATS, o, st))) return rc;
      return feedforward(nullptr);
    }
  }
  if ((rc = rowstats(dtype, x, B * Tl, C, 1e-5f, w.lns, st))) return rc;
  ConvArgs q = gemm_args(t.qkv, P, B, Tl);
  q.x0 = x;
  q.y = w.qkv;
  q.ln_stats = w.lns;
  if ((rc = launch_conv<E, PF_LN, 0>(q, st))) return rc;
  if ((rc = launch_attention(dtype, w.qkv, mask, w.ob, B, Tl, heads, st, w.apart))) return rc;
  ConvArgs o = gemm_args(t.out, P, B, Tl);
  o.x0 = w.ob;
  o.y = x;
  o.resid = x;
  o.ldr = C;
  if ((rc = launch_conv<E, 0, EF_RESID>(o, st))) return rc;
  if ((rc = rowstats(dtype, x, B * Tl, C, 1e-5f, w.lns, st))) return rc;
  ConvArgs f1 = gemm_args(t.ff1, P, B, Tl);
  f1.x0 = x;
  f1.y = w.ff;
  f1.ln_stats = w.lns;
  f1.snake_alpha = (const float*)(P + t.snake_off);
  f1.snake_ibeta = (const float*)(P + t.snake_off) + TE;
  if ((rc = launch_conv<E, PF_LN, EF_SNAKE>(f1, st))) return rc;
  ConvArgs f2 = gemm_args(t.ff2, P, B, Tl);
  f2.x0 = w.ff;
  f2.y = x;
  f2.resid = x;
  f2.ldr = C;
  if ((rc = launch_conv<E, 0, EF_RESID>(f2, st))) return rc;
  return mask_out ? mask_rows(dtype, x, B * Tl, C, mask, st) : 0;
}

int Decoder::tap(const Work& w, int i, const void* src, int B, int Tl, hipStream_t st) const {
  if (!w.taps || !w.taps[i]) return 0;
  return btc_to_bct(dtype, src, C, 0, B, C, Tl, w.taps[i], st);
}

template <class E>
int Decoder::eval(const char* P, const Work& w, int B, int T, int ev, const Euler& eu, hipStream_t st) const {
  int rc;
  const int T1 = T / 2;
  const float* m0 = w.m0;
  const float* m1 = w.m1;
  // time bias of resnet r: one vector per evaluation, or (tb_ld != 0) one per utterance
  auto tbp = [&](int r) { return w.tb_ld ? w.tb + (size_t)r * C : w.tb + ((size_t)ev * n_res + r) * C; };
  // bf16 + vconv: every tensor a conv reads as x * mask is stored masked by its producer (the last
  // transformer block of a chain, the down/up convs), so mt_vconv needs no input prologue
  const bool mio = vconv && std::is_same<E, bf16>::value;
  bool rs = false;  // the last resnet's output conv wrote the LayerNorm partials of its output
  auto tblocks = [&](int r, void* x, const float* m, int Tl) -> int {
    const int nb = (int)tbs[r].size();
    const bool uni = uniform_attn && (Tl == T ? w.uni0 : w.uni1);
    for (int j = 0; j < nb; ++j) {
      int e = tblock<E>(P, w, tbs[r][j], x, m, mio && j == nb - 1, rs && j == 0, uni, B, Tl, st);
      if (e) return e;
    }
    return 0;
  };
  // m: the input mask; mo: the output frames' mask (masked-input mode)
  auto plain = [&](const GemmW& g, const void* x, const float* m, const float* mo, int Tl, void* out) -> int {
    if (mio && vc(g)) {
      VConvArgs a = vargs(g, P, w, x, B, Tl, out);
      a.emask = mo;
      return launch_vconv(VE_MASK, a, st);
    }
    ConvArgs a = gemm_args(g, P, B, Tl);
    a.x0 = x;
    a.y = out;
    if (mio) {
      a.emask = mo;
      return launch_conv<E, 0, EF_MASK>(a, st);
    }
    a.pmask = m;
    return launch_conv<E, PF_MASK, 0>(a, st);
  };
  // down 0 @T
  const int xc = mio ? xld() : c_cond;  // input channels of the first ResnetBlock as stored
  if ((rc = resnet<E>(P, w, res[0], w.xin, nullptr, xc, xc, mio, w.H0, m0, B, T, tbp(0), &rs, st))) return rc;
  if ((rc = tap(w, 0, w.H0, B, T, st))) return rc;
  if ((rc = tblocks(0, w.H0, m0, T))) return rc;
  if ((rc = tap(w, 1, w.H0, B, T, st))) return rc;
  if (mio && vc(down0)) {  // frame pairs: [T][C] rows read as [T/2][2C]
    VConvArgs a = vargs(down0, P, w, w.H0, B, T1, w.XA);
    a.taps = 2;
    a.pad = 1;
    a.emask = m1;
    if ((rc = launch_vconv(VE_MASK, a, st))) return rc;
  } else if ((rc = plain(down0, w.H0, m0, m1, T, w.XA))) {
    return rc;
  }
  // down 1 @T/2
  if ((rc = resnet<E>(P, w, res[1], w.XA, nullptr, C, C, mio, w.H1, m1, B, T1, tbp(1), &rs, st))) return rc;
  if ((rc = tblocks(1, w.H1, m1, T1))) return rc;
  if ((rc = plain(down1, w.H1, m1, m1, T1, w.XB))) return rc;
  char* half[3] = {w.XA, w.XB, w.XC};
  int cur = 1;
  for (int i = 0; i < n_mid; ++i) {
    const int nx = (cur + 1) % 3;
    if ((rc = resnet<E>(P, w, res[2 + i], half[cur], nullptr, C, C, mio, half[nx], m1, B, T1, tbp(2 + i), &rs, st)))
      return rc;
    if ((rc = tblocks(2 + i, half[nx], m1, T1))) return rc;
    if (i == n_mid - 1 && (rc = tap(w, 2, half[nx], B, T1, st))) return rc;
    cur = nx;
  }
  // up 0 @T/2: cat(x, skip=H1)
  {
    const int nx = (cur + 1) % 3;
    const int r = 2 + n_mid;
    if ((rc = resnet<E>(P, w, res[r], half[cur], w.H1, C, 2 * C, mio, half[nx], m1, B, T1, tbp(r), &rs, st)))
      return rc;
    if ((rc = tblocks(r, half[nx], m1, T1))) return rc;
    if (mio && vc(up0)) {  // ConvTranspose1d k4 s2 p1 -> T as a polyphase conv with a placed, masked output
      int Tout = 0, Ncols = 0;
      gemm_geom(up0, T1, &Tout, &Ncols);
      VConvArgs a = vargs(up0, P, w, half[nx], B, T1, w.U);
      a.M = a.Mpad = up0.vrows;
      a.taps = up0.taps;
      a.pad = up0.gpad;
      a.Lout = Ncols;
      a.ldy = up0.M;
      a.yshift = up0.opad * up0.cout;
      a.ylim = Tout * up0.cout;
      a.ystride = (long long)Tout * up0.cout;
      a.mask_div = up0.cout;
      a.emask = m0;
      a.probe = -1;
      if ((rc = launch_vconv(VE_PMASK, a, st))) return rc;
    } else if ((rc = plain(up0, half[nx], m1, m0, T1, w.U))) {  // ConvTranspose1d k4 s2 p1 -> T
      return rc;
    }
    if ((rc = tap(w, 3, w.U, B, T, st))) return rc;
  }
  // up 1 @T: cat(U, skip=H0)
  {
    const int r = 3 + n_mid;
    if ((rc = resnet<E>(P, w, res[r], w.U, w.H0, C, 2 * C, mio, w.XF, m0, B, T, tbp(r), &rs, st))) return rc;
    if ((rc = tblocks(r, w.XF, m0, T))) return rc;
    if ((rc = tap(w, 4, w.XF, B, T, st))) return rc;
    if ((rc = plain(up1, w.XF, m0, m0, T, w.U))) return rc;
  }
  // final block + projection + ODE update
  int ntf = 0;
  if (mio && vc(fconv)) {
    VConvArgs a = vargs(fconv, P, w, w.U, B, T, w.y1);
    a.gn_out = w.gn1;
    ntf = a.gn_parts = vconv_gn_parts(B, T, C);
    if ((rc = launch_vconv(VE_GNSTATS, a, st))) return rc;
  } else {
    ConvArgs a = gemm_args(fconv, P, B, T);
    a.x0 = w.U;
    a.y = w.y1;
    a.pmask = m0;
    a.gn_out = w.gn1;
    if ((rc = launch_conv<E, PF_MASK, EF_GNSTATS>(a, st, &ntf))) return rc;
  }
  ConvArgs f = gemm_args(fproj, P, B, T);
  f.x0 = w.y1;
  f.y = nullptr;
  f.pmask = m0;
  f.emask = m0;
  f.gn_in = w.gn1;
  f.gn_ntiles = ntf;
  f.gn_T = T;
  f.gn_g = (const float*)(P + fgn_off);
  f.gn_b = (const float*)(P + fgn_off) + C;
  f.zmaster = w.zm;
  f.xin_z = w.xin;
  f.ld_xin = xld();
  f.dt = eu.dt;
  f.half_step = eu.half_step;
  f.update_master = eu.update_master;
  if (std::is_same<E, bf16>::value && (dec_kernels() & DECK_PROJ) && proj_euler_supported(f))
    return launch_proj_euler(f, st);
  return launch_conv<E, PF_GN | PF_MASK, EF_MASK | EF_EULER>(f, st);
}

int Decoder::init_inputs(const Work& w, const float* z, float temperature, const float* mu_y,
                         const float* spks, int B, int T, hipStream_t st) const {
  int rc;
  const int ld = xld();
  if (ld != c_cond) MT_CHECK_HIP(hipMemsetAsync(w.xin, 0, (size_t)B * T * ld * esize, st));  // zero pad channels
  if ((rc = bct_to_btc(F32, z, B, NF, T, temperature, w.zm, NF, 0, st))) return rc;
  if ((rc = bct_to_btc(dtype, z, B, NF, T, temperature, w.xin, ld, 0, st))) return rc;
  if ((rc = bct_to_btc(dtype, mu_y, B, NF, T, 1.f, w.xin, ld, NF, st))) return rc;
  if (c_cond > 2 * NF) {
    MT_REQUIRE(spks != nullptr, "decoder: c_cond %d needs speaker embeddings", c_cond);
    if ((rc = spk_fill(dtype, spks, B, c_cond - 2 * NF, T, w.xin, ld, 2 * NF, st))) return rc;
  }
  // the vconv path reads x ‖ mu ‖ spk as x * mask straight from HBM: store it masked (the generic path masks
  // in its prologue, so both read the same values; the Euler epilogue keeps the z slot masked)
  if (vconv && dtype == BF16 && (rc = mask_rows(dtype, w.xin, B * T, ld, w.m0, st))) return rc;
  return mask_half(w.m0, B, T, w.m1, st);
}

static int check_geom(int B, int T) {
  MT_REQUIRE(B > 0 && T > 0, "decoder: empty batch");
  MT_REQUIRE(T % 2 == 0, "decoder: T=%d must be even (synthesize pads to a multiple of 4)", T);
  return 0;
}

// ---- captured evaluation chains (hipGraph) ----
struct Decoder::GraphCache {
  struct Entry {
    const void* P;
    const void* ws;
    int B, T, S, n_steps, solver, uni0, uni1, vconv, gnres, uniform_attn, kpath, deck;
    hipGraphExec_t ex;
  };
  std::vector<Entry> entries;  // most recently used last
  hipStream_t cap = nullptr;   // private capture stream (the legacy null stream cannot be captured)
  ~GraphCache() {
    for (Entry& e : entries) (void)hipGraphExecDestroy(e.ex);
    if (cap) (void)hipStreamDestroy(cap);
  }
};

namespace {
constexpr size_t kMaxGraphs = 8;
}

int Decoder::chain_graph(const char* P, const Work& w, const TimeSched& ts, int S, int B, int T, int n_steps,
                         int solver, const void* ws, hipGraphExec_t* out) const {
  if (!gcache) gcache = std::make_shared<GraphCache>();
  GraphCache& gc = *gcache;
  // kpath: the process-wide kernel selection (compile-time K loops on / off): a graph holds the kernels it captured
  const GraphCache::Entry key{P, ws, B, T, S, n_steps, solver, w.uni0, w.uni1, vconv, gnres, uniform_attn,
                              vconv_path_id() | (ffn_on() << 3) | (std::min(ffn_min_frames(), 1 << 25) << 5),
                              dec_kernels(), nullptr};
  for (size_t i = 0; i < gc.entries.size(); ++i) {
    const GraphCache::Entry& e = gc.entries[i];
    if (e.P == key.P && e.ws == key.ws && e.B == key.B && e.T == key.T && e.S == key.S && e.n_steps == key.n_steps &&
        e.solver == key.solver && e.uni0 == key.uni0 && e.uni1 == key.uni1 && e.vconv == key.vconv &&
        e.gnres == key.gnres && e.uniform_attn == key.uniform_attn && e.kpath == key.kpath && e.deck == key.deck) {
      GraphCache::Entry hit = e;
      gc.entries.erase(gc.entries.begin() + (long)i);
      gc.entries.push_back(hit);
      *out = hit.ex;
      return 0;
    }
  }
  if (!gc.cap) MT_CHECK_HIP(hipStreamCreateWithFlags(&gc.cap, hipStreamNonBlocking));
  MT_CHECK_HIP(hipStreamBeginCapture(gc.cap, hipStreamCaptureModeThreadLocal));
  const int rc = solve_chain(P, w, ts, S, B, T, n_steps, solver, gc.cap);
  hipGraph_t g = nullptr;
  const hipError_t e = hipStreamEndCapture(gc.cap, &g);
  if (rc || e != hipSuccess || !g) {
    if (g) (void)hipGraphDestroy(g);
    if (rc) return rc;
    set_error("decoder: graph capture failed (%s)", hipGetErrorString(e));
    return -1;
  }
  hipGraphExec_t ex = nullptr;
  const hipError_t ie = hipGraphInstantiate(&ex, g, nullptr, nullptr, 0);
  (void)hipGraphDestroy(g);
  MT_CHECK_HIP(ie);
  if (gc.entries.size() >= kMaxGraphs) {
    (void)hipGraphExecDestroy(gc.entries.front().ex);
    gc.entries.erase(gc.entries.begin());
  }
  GraphCache::Entry ent = key;
  ent.ex = ex;
  gc.entries.push_back(ent);
  *out = ex;
  return 0;
}

int Decoder::solve(const void* packed, const float* z_noise, float temperature, const float* mu_y,
                   const float* mask, const float* spks, int B, int T, int n_steps, int solver, float* z_out,
                   void* ws, size_t ws_bytes, hipStream_t st, int max_valid) const {
  int rc;
  if ((rc = check_geom(B, T))) return rc;
  MT_REQUIRE(n_steps >= 1, "cfm: n_timesteps must be >= 1");
  MT_REQUIRE(solver == 0 || solver == 1, "cfm: solver must be 0 (euler) or 1 (midpoint)");
  const int S = solver == 0 ? n_steps : 2 * n_steps;
  MT_REQUIRE(S <= TimeSched::MAX, "cfm: too many evaluations (%d)", S);
  MT_REQUIRE(ws_bytes >= workspace_bytes(B, T, S), "cfm: workspace %zu < %zu", ws_bytes,
             workspace_bytes(B, T, S));
  const char* P = (const char*)packed;
  Work w = carve(ws, B, T, S);
  w.m0 = mask;
  // the caller's bound on valid frames (model.py's y_max): below T every utterance is padded at full resolution,
  // at <= T - 2 also at half resolution (mask[:, ::2] keeps frame T - 2)
  MT_REQUIRE(max_valid >= 0 && max_valid <= T, "cfm: max_valid %d outside [0, T=%d]", max_valid, T);
  w.uni0 = max_valid > 0 && max_valid < T;
  w.uni1 = max_valid > 0 && max_valid <= T - 2;
  // evaluation times exactly as the reference forms them in fp32 (model.py:1086-1104)
  TimeSched ts{};
  const float dt = (float)(1.0 / (double)n_steps);
  for (int i = 0; i < n_steps; ++i) {
    const float t = (float)((double)i / (double)n_steps);
    if (solver == 0) {
      ts.t[i] = t;
    } else {
      ts.t[2 * i] = t;
      ts.t[2 * i + 1] = t + dt * 0.5f;
    }
  }
  // eager only while the decoder's own launches are probed or logged: an armed vocoder probe (bench.py's last timed
  // step) must not take the solve off its graph
  if (!(graphs && !probe_armed(PROBE_VCONV_DEC) && !vclog_armed())) {
    if ((rc = init_inputs(w, z_noise, temperature, mu_y, spks, B, T, st))) return rc;
    if ((rc = solve_chain(P, w, ts, S, B, T, n_steps, solver, st))) return rc;
    return btc_to_bct(F32, w.zm, NF, 0, B, NF, T, z_out, st);
  }
  // graph path: the chain reads only the packed weights and the workspace (inputs and mask staged into it)
  MT_CHECK_HIP(hipMemcpyAsync(w.mst, mask, (size_t)B * T * 4, hipMemcpyDeviceToDevice, st));
  w.m0 = w.mst;
  if ((rc = init_inputs(w, z_noise, temperature, mu_y, spks, B, T, st))) return rc;
  hipGraphExec_t ex = nullptr;
  if ((rc = chain_graph(P, w, ts, S, B, T, n_steps, solver, ws, &ex))) return rc;
  MT_CHECK_HIP(hipGraphLaunch(ex, st));
  return btc_to_bct(F32, w.zm, NF, 0, B, NF, T, z_out, st);
}

int Decoder::solve_chain(const char* P, const Work& w, const TimeSched& ts, int S, int B, int T, int n_steps,
                         int solver, hipStream_t st) const {
  int rc;
  const float dt = (float)(1.0 / (double)n_steps);
  if ((rc = time_embed(P, w, ts, S, st))) return rc;
  for (int i = 0; i < n_steps; ++i) {
    if (solver == 0) {
      Euler eu{dt, 0, 1};
      rc = dtype == BF16 ? eval<bf16>(P, w, B, T, i, eu, st) : eval<float>(P, w, B, T, i, eu, st);
      if (rc) return rc;
    } else {
      Euler e1{dt, 1, 0}, e2{dt, 0, 1};
      rc = dtype == BF16 ? eval<bf16>(P, w, B, T, 2 * i, e1, st) : eval<float>(P, w, B, T, 2 * i, e1, st);
      if (rc) return rc;
      rc = dtype == BF16 ? eval<bf16>(P, w, B, T, 2 * i + 1, e2, st)
                         : eval<float>(P, w, B, T, 2 * i + 1, e2, st);
      if (rc) return rc;
    }
  }
  return 0;
}

int Decoder::step(const void* packed, const float* x, const float* mu_y, const float* mask, const float* spks,
                  float t, int B, int T, float* out, void* ws, size_t ws_bytes, hipStream_t st) const {
  int rc;
  if ((rc = check_geom(B, T))) return rc;
  MT_REQUIRE(ws_bytes >= workspace_bytes(B, T, 1), "decoder: workspace too small");
  const char* P = (const char*)packed;
  Work w = carve(ws, B, T, 1);
  w.m0 = mask;
  w.taps = taps;
  TimeSched ts{};
  ts.t[0] = t;
  if ((rc = time_embed(P, w, ts, 1, st))) return rc;
  if ((rc = init_inputs(w, x, 1.f, mu_y, spks, B, T, st))) return rc;
  MT_CHECK_HIP(hipMemsetAsync(w.zm, 0, (size_t)B * T * NF * 4, st));
  Euler eu{1.f, 0, 1};  // z = 0 + pred * 1  ==  pred exactly
  rc = dtype == BF16 ? eval<bf16>(P, w, B, T, 0, eu, st) : eval<float>(P, w, B, T, 0, eu, st);
  if (rc) return rc;
  return btc_to_bct(F32, w.zm, NF, 0, B, NF, T, out, st);
}

// One estimator evaluation with a time per utterance (CFM.compute_loss draws t ~ U(0,1) per sample,
// model.py:1147-1162): the time MLPs run once per utterance and every ResnetBlock adds its utterance's
// time bias. t: [B] fp32 in device memory.
int Decoder::step_times(const void* packed, const float* x, const float* mu_y, const float* mask,
                        const float* spks, const float* t_dev, int B, int T, float* out, void* ws, size_t ws_bytes,
                        hipStream_t st) const {
  int rc;
  if ((rc = check_geom(B, T))) return rc;
  MT_REQUIRE(t_dev, "decoder: per-utterance times missing");
  MT_REQUIRE(ws_bytes >= workspace_bytes(B, T, B), "decoder: workspace too small");
  const char* P = (const char*)packed;
  Work w = carve(ws, B, T, B);
  w.m0 = mask;
  w.tb_ld = n_res * C;
  TimeSched ts{};
  if ((rc = time_embed(P, w, ts, B, st, t_dev))) return rc;
  if ((rc = init_inputs(w, x, 1.f, mu_y, spks, B, T, st))) return rc;
  MT_CHECK_HIP(hipMemsetAsync(w.zm, 0, (size_t)B * T * NF * 4, st));
  Euler eu{1.f, 0, 1};
  rc = dtype == BF16 ? eval<bf16>(P, w, B, T, 0, eu, st) : eval<float>(P, w, B, T, 0, eu, st);
  if (rc) return rc;
  return btc_to_bct(F32, w.zm, NF, 0, B, NF, T, out, st);
}

}  // namespace mt
