// Decoder self-attention core (model.py:686-701) for gfx950.
//
// qkv [B][T][3*inner] (q | k | v, head h at columns h*64..h*64+63 of each part),
// mask [B][T] (frame mask at this U-Net level), out [B][T][inner].
// Workgroup = 4 waves = 64 queries of one (utterance, head); flash-style online softmax
// over 64-key tiles, S = Q.K^T and O += P.V on MFMA (bf16: 16x16x32, f32: 16x16x4).
//
// Key split (flash-decoding): an unpadded utterance's 64-query tile is the launch's critical path
// (T/64 dependent key-tile iterations), so grid.z carries NS key ranges per utterance; each writes
// its unnormalised (o, m, l) to a workspace slot and attn_merge_kernel combines the slots in split
// order (deterministic). The next key tile's K/V rows are fetched into registers while the current
// tile computes.
//
// Reference mask semantics, kept exactly: masked keys are filled with
// -torch.finfo(fp32).min = +3.4e38 (model.py:697), so for an utterance whose mask has ANY
// zero at this level every query attends uniformly to the masked keys:
//     out = sum_{j masked} (1/n_masked) * v_j          (independent of q and k)
// and for an utterance without padding the ordinary softmax over all keys applies.
#include "mt_common.h"
#include "mt_misc.h"

#include <algorithm>
#include <cstdlib>
#include <type_traits>

namespace mt {

template <class E>
__global__ __launch_bounds__(256) void attn_kernel(const E* __restrict__ qkv,
                                                   const float* __restrict__ mask,
                                                   E* __restrict__ out, int T, int inner, int NS,
                                                   float* __restrict__ part) {
  constexpr int CH = Chunk<E>::CH;          // elements per 64-byte chunk
  constexpr int VN = Vec16<E>::N;           // elements per 16 bytes
  constexpr int NDC = 64 / CH;              // d-chunks per head (bf16 2, f32 4)
  constexpr int ROW = 64 * sizeof(E) + 16;  // LDS row bytes for 64 elements (+16 pad)
  constexpr bool PRECISE = std::is_same<E, float>::value;

  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Ks = smem;              // [64 keys][64 d]
  char* Vt = Ks + 64 * ROW;     // [64 d][64 keys]
  char* Ps = Vt + 64 * ROW;     // [4 waves][16 q][64 keys]
  float* red = reinterpret_cast<float*>(Ps + 64 * ROW);  // [4][64]

  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int b = blockIdx.z / NS, sp = blockIdx.z - b * NS, h = blockIdx.y, q0 = blockIdx.x * 64;
  const int ld = 3 * inner;
  const E* Q = qkv + (size_t)b * T * ld + h * 64;
  const E* K = Q + inner;
  const E* V = Q + 2 * inner;
  const float* mk = mask + (size_t)b * T;
  E* O = out + (size_t)b * T * inner + h * 64;

  // ---- does this utterance have padded frames at this level? ----
  int npad_local = 0;
  for (int j = tid; j < T; j += 256) npad_local += (mk[j] == 0.f) ? 1 : 0;
  if (__syncthreads_or(npad_local)) {
    if (sp != 0) return;  // one block per query tile serves the uniform case
    // exact count of masked keys
    int* cnt = reinterpret_cast<int*>(red);
    if (tid == 0) cnt[0] = 0;
    __syncthreads();
    if (npad_local) atomicAdd(cnt, npad_local);
    __syncthreads();
    const int n = cnt[0];
    __syncthreads();
    const float p = 1.f / (float)n;
    // thread (kg, dc): 16-byte column chunk dc of keys j = kg (mod KG), several rows in flight
    constexpr int NC = 64 / VN, KG = 256 / NC;
    const int kg = tid / NC, dc = tid % NC;
    float s[VN];
#pragma unroll
    for (int e = 0; e < VN; ++e) s[e] = 0.f;
#pragma unroll 4
    for (int j = kg; j < T; j += KG) {
      const Vec16<E> v = load16(V + (size_t)j * ld + dc * VN);
      const float w = mk[j] == 0.f ? p : 0.f;
#pragma unroll
      for (int e = 0; e < VN; ++e) s[e] += w * v.get(e);
    }
    float* part_s = reinterpret_cast<float*>(smem);  // [KG][64] (the K tile region is free here)
#pragma unroll
    for (int e = 0; e < VN; ++e) part_s[kg * 64 + dc * VN + e] = s[e];
    __syncthreads();
    if (tid < 64) {
      float t = 0.f;
      for (int k = 0; k < KG; ++k) t += part_s[k * 64 + tid];
      red[tid] = t;
    }
    __syncthreads();
    for (int i = tid; i < 64 * NC; i += 256) {
      const int q = q0 + i / NC, c = i % NC;
      if (q >= T) continue;
      Vec16<E> o;
#pragma unroll
      for (int e = 0; e < VN; ++e) o.set(e, red[c * VN + e]);
      store16(O + (size_t)q * inner + c * VN, o);
    }
    return;
  }

  // ---- ordinary softmax attention ----
  const int qrow = q0 + wave * 16 + (lane & 15);
  Vec16<E> qf[NDC];
#pragma unroll
  for (int c = 0; c < NDC; ++c)
    qf[c] = (qrow < T) ? load16(Q + (size_t)qrow * ld + c * CH + (lane >> 4) * VN) : zero16<E>();

  f32x4 o[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float m_run[4], l_run[4];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    m_run[r] = -INFINITY;
    l_run[r] = 0.f;
  }

  char* Pw = Ps + wave * 16 * ROW;
  const int nkt_all = (T + 63) / 64;
  const int per = (nkt_all + NS - 1) / NS;
  const int kt0 = sp * per, kt1 = min(nkt_all, kt0 + per);
  constexpr int NI = 64 * (64 / VN) / 256;  // 16-byte K (and V) pieces per thread per key tile
  Vec16<E> kn[NI], vn[NI];
  auto fetch = [&](int kt) {
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int v = tid + i * 256;
      const int r = v / (64 / VN), s = v % (64 / VN);
      const int key = kt * 64 + r;
      kn[i] = zero16<E>();
      vn[i] = zero16<E>();
      if (key < T) {
        kn[i] = load16(K + (size_t)key * ld + s * VN);
        vn[i] = load16(V + (size_t)key * ld + s * VN);
      }
    }
  };
  if (kt0 < kt1) fetch(kt0);
  for (int kt = kt0; kt < kt1; ++kt) {
    const int k0 = kt * 64;
    // stage K rows and V^T from the prefetched registers, then fetch the next tile
#pragma unroll
    for (int i = 0; i < NI; ++i) {
      const int v = tid + i * 256;
      const int r = v / (64 / VN), s = v % (64 / VN);
      store16(reinterpret_cast<E*>(Ks + r * ROW + s * 16), kn[i]);
#pragma unroll
      for (int e = 0; e < VN; ++e)
        reinterpret_cast<E*>(Vt + (s * VN + e) * ROW)[r] = from_f<E>(vn[i].get(e));
    }
    if (kt + 1 < kt1) fetch(kt + 1);
    __syncthreads();

    // S = Q K^T : 16 queries x 64 keys per wave (4 fragments of 16 keys)
    f32x4 sfr[4];
#pragma unroll
    for (int fn = 0; fn < 4; ++fn) {
      f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int c = 0; c < NDC; ++c) {
        const Vec16<E> kb = load16(reinterpret_cast<const E*>(
            Ks + (fn * 16 + (lane & 15)) * ROW + c * 64 + (lane >> 4) * 16));
        acc = mfma16(qf[c].v, kb.v, acc);
      }
      sfr[fn] = acc;
    }
    // scale, invalid keys, row max over the 64 keys of this tile
    float mt[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) mt[r] = -INFINITY;
#pragma unroll
    for (int fn = 0; fn < 4; ++fn) {
      const bool kval = (k0 + fn * 16 + (lane & 15)) < T;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float s = kval ? sfr[fn][r] * 0.125f : -INFINITY;
        sfr[fn][r] = s;
        mt[r] = fmaxf(mt[r], s);
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) mt[r] = fmaxf(mt[r], __shfl_xor(mt[r], off, 64));
    }
    float corr[4], rs[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float mn = fmaxf(m_run[r], mt[r]);
      corr[r] = (m_run[r] == -INFINITY) ? 0.f : (PRECISE ? expf(m_run[r] - mn) : __expf(m_run[r] - mn));
      m_run[r] = mn;
      rs[r] = 0.f;
    }
#pragma unroll
    for (int fn = 0; fn < 4; ++fn) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const float p = PRECISE ? expf(sfr[fn][r] - m_run[r]) : __expf(sfr[fn][r] - m_run[r]);
        sfr[fn][r] = p;
        rs[r] += p;
      }
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) {
#pragma unroll
      for (int off = 1; off < 16; off <<= 1) rs[r] += __shfl_xor(rs[r], off, 64);
      l_run[r] = l_run[r] * corr[r] + rs[r];
    }
#pragma unroll
    for (int df = 0; df < 4; ++df)
#pragma unroll
      for (int r = 0; r < 4; ++r) o[df][r] *= corr[r];

    // P -> LDS (row q, col key) in the element type
#pragma unroll
    for (int fn = 0; fn < 4; ++fn)
#pragma unroll
      for (int r = 0; r < 4; ++r)
        reinterpret_cast<E*>(Pw + (4 * (lane >> 4) + r) * ROW)[fn * 16 + (lane & 15)] =
            from_f<E>(sfr[fn][r]);
    __syncthreads();

    // O += P V : A = P[16 q][64 keys], B = V[64 keys][16 d] via V^T rows
#pragma unroll
    for (int c = 0; c < NDC; ++c) {
      const Vec16<E> pa =
          load16(reinterpret_cast<const E*>(Pw + (lane & 15) * ROW + c * 64 + (lane >> 4) * 16));
#pragma unroll
      for (int df = 0; df < 4; ++df) {
        const Vec16<E> vb = load16(reinterpret_cast<const E*>(
            Vt + (df * 16 + (lane & 15)) * ROW + c * 64 + (lane >> 4) * 16));
        o[df] = mfma16(pa.v, vb.v, o[df]);
      }
    }
    __syncthreads();
  }

  // normalise and store: lane holds rows q = 4(lane>>4)+r, col d = 16 df + (lane&15)
  if (NS == 1) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int q = q0 + wave * 16 + 4 * (lane >> 4) + r;
      if (q >= T) continue;
      const float inv = 1.f / l_run[r];
#pragma unroll
      for (int df = 0; df < 4; ++df) O[(size_t)q * inner + df * 16 + (lane & 15)] = from_f<E>(o[df][r] * inv);
    }
    return;
  }
  // split: slot = [64 q][64 d] o + [64 q] (m, l); an empty key range leaves m = -inf, l = 0
  const int tile = (b * gridDim.y + h) * gridDim.x + blockIdx.x;
  float* slot = part + ((size_t)tile * NS + sp) * (64 * 66);
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int ql = wave * 16 + 4 * (lane >> 4) + r;
#pragma unroll
    for (int df = 0; df < 4; ++df) slot[ql * 64 + df * 16 + (lane & 15)] = o[df][r];
    if ((lane & 15) == 0) {
      slot[64 * 64 + 2 * ql] = m_run[r];
      slot[64 * 64 + 2 * ql + 1] = l_run[r];
    }
  }
}

// combines the NS key-range slots of every query tile of the unpadded utterances, split order fixed
template <class E>
__global__ __launch_bounds__(256) void attn_merge_kernel(const float* __restrict__ part,
                                                         const float* __restrict__ mask, E* __restrict__ out,
                                                         int T, int inner, int NS) {
  constexpr bool PRECISE = std::is_same<E, float>::value;
  const int tid = threadIdx.x, b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * 64;
  const float* mk = mask + (size_t)b * T;
  int npad_local = 0;
  for (int j = tid; j < T; j += 256) npad_local += (mk[j] == 0.f) ? 1 : 0;
  if (__syncthreads_or(npad_local)) return;  // the uniform path wrote this utterance
  const int tile = (b * gridDim.y + h) * gridDim.x + blockIdx.x;
  const float* slot0 = part + (size_t)tile * NS * (64 * 66);
  const int ql = tid >> 2, dq = (tid & 3) * 16;
  const int q = q0 + ql;
  if (q >= T) return;
  float mx = -INFINITY;
  for (int k = 0; k < NS; ++k) mx = fmaxf(mx, slot0[(size_t)k * (64 * 66) + 64 * 64 + 2 * ql]);
  float acc[16], lsum = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) acc[i] = 0.f;
  for (int k = 0; k < NS; ++k) {
    const float* sl = slot0 + (size_t)k * (64 * 66);
    const float mk_ = sl[64 * 64 + 2 * ql];
    if (mk_ == -INFINITY) continue;
    const float wk = PRECISE ? expf(mk_ - mx) : __expf(mk_ - mx);
    lsum += sl[64 * 64 + 2 * ql + 1] * wk;
#pragma unroll
    for (int i = 0; i < 16; ++i) acc[i] += sl[ql * 64 + dq + i] * wk;
  }
  const float inv = 1.f / lsum;
  E* O = out + ((size_t)b * T + q) * inner + h * 64 + dq;
#pragma unroll
  for (int i = 0; i < 16; ++i) O[i] = from_f<E>(acc[i] * inv);
}

static int attn_splits(int T) {
  const int nkt = (T + 63) / 64;
  return std::min(8, (nkt + 2) / 3);
}
size_t attention_part_bytes(int B, int T, int heads) {
  const int NS = attn_splits(T);
  return NS <= 1 ? 0 : (size_t)B * heads * ((T + 63) / 64) * NS * 64 * 66 * sizeof(float);
}

// ------------------------------------------------------------------------------------------------------
// Query-independent attention of utterances WITH padding (bf16 decoder, C = 256, heads x 64 = 128).
// The reference fills masked keys with +3.4e38 (model.py:697), so every query of such an utterance attends
// uniformly to its masked keys: attn1's output is the same row for every frame,
//     o = W_o (mean_{j masked} V_j) + b_o,   V_j = W_v LN1(x_j) + b_v = W'_v xhat_j + b'_v
// (LN1's gamma / beta are folded into the packed QKV image W' / bias b'; xhat_j = (x_j - mu_j) rstd_j). So the
// block needs neither Q, K, V of every frame nor the per-frame out-projection: one masked mean of xhat per
// utterance and two 256-wide GEMVs. BasicTransformerBlock's x + attn1(...) (model.py:733-737) becomes x_j += o.
// part: grid (S, B), slice s of utterance b -> part[b][s][0..255] = sum over masked frames of xhat, [256] = count
// vec: grid B, merges the utterance's S partials (slice order) and runs the two GEMVs -> o_b (one launch per
//   utterance: the round-2 apply that redid them in every slice's workgroup was 1.56 vs 1.25 ms per step)
// apply: grid (S, B), x_j = bf16(x_j + o) for the slice's frames + the (mean, M2) per 64-channel slab of the stored row
//   (the LayerNorm partials LN3 reads, VE_ROWSTATS format). Rounding as the GEMM path: V averaged in fp32,
//   o rounded to bf16 (the attention output was stored bf16), x + (W_o o + b_o) in fp32, stored bf16.
constexpr int UNI_C = 256, UNI_PART = UNI_C + 4;  // UNI_PSMAX (mt_misc.h): part slices per utterance

__global__ __launch_bounds__(256) void attn_uni_part_kernel(const bf16* __restrict__ x, const float* __restrict__ mask,
                                                            int T, float* __restrict__ part, int xr) {
  __shared__ float red[8][UNI_C + 1];
  const int S = gridDim.x, tid = threadIdx.x;
  const int ci = xcd_chunk(blockIdx.x + S * blockIdx.y, S * gridDim.y, xr);  // (slice, utterance), XCD-aligned
  const int s = ci % S, b = ci / S;
  const int fr = tid >> 5, cl = tid & 31, c = cl * 8;
  const int f0 = (int)((long)s * T / S), f1 = (int)((long)(s + 1) * T / S);
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f}, n = 0.f;
  constexpr int FB = 4;  // frames per thread per round: their loads are issued together
  for (int jb = f0 + fr; jb < f1; jb += 8 * FB) {
    u32x4 wv[FB];
    bool use[FB];
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const int j = jb + 8 * i;
      use[i] = j < f1 && mask[(size_t)b * T + min(j, f1 - 1)] == 0.f;  // the 32 lanes of a frame agree
      wv[i] = use[i] ? *reinterpret_cast<const u32x4*>(x + ((size_t)b * T + j) * UNI_C + c) : u32x4{0u, 0u, 0u, 0u};
    }
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      if (!use[i]) continue;
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        v[2 * e] = __uint_as_float(wv[i][e] << 16);
        v[2 * e + 1] = __uint_as_float(wv[i][e] & 0xffff0000u);
      }
      float sm = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) sm += __shfl_xor(sm, o, 64);
      const float mu = sm * (1.f / UNI_C);
      float q = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) q += (v[e] - mu) * (v[e] - mu);
#pragma unroll
      for (int o = 1; o < 32; o <<= 1) q += __shfl_xor(q, o, 64);
      const float rs = rsqrtf(q * (1.f / UNI_C) + 1e-5f);  // nn.LayerNorm eps (BasicTransformerBlock.norm1)
#pragma unroll
      for (int e = 0; e < 8; ++e) acc[e] += (v[e] - mu) * rs;
      n += 1.f;
    }
  }
#pragma unroll
  for (int e = 0; e < 8; ++e) red[fr][c + e] = acc[e];
  if (cl == 0) red[fr][UNI_C] = n;
  __syncthreads();
  for (int i = tid; i <= UNI_C; i += 256) {
    float t = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) t += red[k][i];
    part[((size_t)b * S + s) * UNI_PART + i] = t;
  }
}

// the utterance's attention output vector o_b (grid B): merge of the SP masked-sum slices, then the two GEMVs.
// Every load is issued up front, the weights first (this lane's V-row and out-projection pieces, then the
// partials: none depends on another), so the kernel pays one memory round trip instead of three; the slice counts
// come in as one lane-varying load (lane k: slice k) read back with v_readlane — as 32 wave-uniform loads they went
// through the scalar cache, whose ≤ 15 outstanding loads and lgkmcnt(0) waits split the kernel into several
// round trips (9–10 us per launch at any B). The arithmetic and its order are unchanged.
__global__ __launch_bounds__(256) void attn_uni_vec_kernel(int SP, const float* __restrict__ part,
                                                           const bf16* __restrict__ wqkv, int mq, const float* __restrict__ bqkv,
                                                           const bf16* __restrict__ wout, const float* __restrict__ bout,
                                                           float* __restrict__ ovec) {
  __shared__ float zb[UNI_C], vb[128];
  const int b = blockIdx.x, tid = threadIdx.x;
  // GEMVs: 4 lanes per output row, each a quarter of K, combined by two lane shuffles
  const int q4 = tid & 3, rq = tid >> 2;  // 64 row slots per pass
  // V rows 256 .. 383 of the LN-folded QKV image [4 chunks][mq rows][64]; lane quarter q4 = chunk q4
  u32x4 wv[2][8];
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const bf16* wr = wqkv + ((size_t)q4 * mq + 256 + rq + 64 * pass) * 64;
#pragma unroll
    for (int i = 0; i < 8; ++i) wv[pass][i] = *reinterpret_cast<const u32x4*>(wr + 8 * i);
  }
  // out-projection [2 chunks][256 rows][64]: quarter q4 = chunk q4 / 2, half (q4 & 1) of its 64 elements
  const int ck = q4 >> 1, k0 = (q4 & 1) * 32;
  u32x4 wo[4][4];
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const bf16* wr = wout + ((size_t)ck * UNI_C + rq + 64 * pass) * 64 + k0;
#pragma unroll
    for (int i = 0; i < 4; ++i) wo[pass][i] = *reinterpret_cast<const u32x4*>(wr + 8 * i);
  }
  float bq[2], bo[4];  // the biases this lane's rows add (q4 == 0 lanes use them)
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) bq[pass] = bqkv[256 + rq + 64 * pass];
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) bo[pass] = bout[rq + 64 * pass];
  float zz[UNI_PSMAX];
#pragma unroll
  for (int k = 0; k < UNI_PSMAX; ++k) zz[k] = part[((size_t)b * SP + min(k, SP - 1)) * UNI_PART + tid];
  const float nl = part[((size_t)b * SP + min(tid & (UNI_PSMAX - 1), SP - 1)) * UNI_PART + UNI_C];
  {  // merge the utterance's SP part slices in order
    float z = 0.f, n = 0.f;
#pragma unroll
    for (int k = 0; k < UNI_PSMAX; ++k)
      if (k < SP) {
        z += zz[k];
        n += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(nl), k));
      }
    zb[tid] = z / n;
  }
  __syncthreads();
  auto dot8 = [](u32x4 w, const float* z) {
    float acc = 0.f;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      acc += __uint_as_float(w[e] << 16) * z[2 * e] + __uint_as_float(w[e] & 0xffff0000u) * z[2 * e + 1];
    return acc;
  };
#pragma unroll
  for (int pass = 0; pass < 2; ++pass) {
    const int r = rq + 64 * pass;
    float v = 0.f;
#pragma unroll
    for (int i = 0; i < 8; ++i) v += dot8(wv[pass][i], zb + q4 * 64 + 8 * i);
    v += __shfl_xor(v, 1, 64);
    v += __shfl_xor(v, 2, 64);
    if (q4 == 0) vb[r] = (float)(bf16)(v + bq[pass]);
  }
  __syncthreads();
#pragma unroll
  for (int pass = 0; pass < 4; ++pass) {
    const int r = rq + 64 * pass;
    float o = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) o += dot8(wo[pass][i], vb + ck * 64 + k0 + 8 * i);
    o += __shfl_xor(o, 1, 64);
    o += __shfl_xor(o, 2, 64);
    if (q4 == 0) ovec[(size_t)b * UNI_C + r] = o + bo[pass];
  }
}

// x += o_b on every frame of the slice, + the next LayerNorm's per-slab (mean, M2) (grid slices x B)
__global__ __launch_bounds__(256) void attn_uni_apply_kernel(bf16* __restrict__ x, int T, const float* __restrict__ ovec,
                                                             float* __restrict__ row_out, int xr) {
  __shared__ float ob[UNI_C];
  const int S = gridDim.x, tid = threadIdx.x;
  const int ci = xcd_chunk(blockIdx.x + S * blockIdx.y, S * gridDim.y, xr);  // (slice, utterance), XCD-aligned
  const int s = ci % S, b = ci / S;
  ob[tid] = ovec[(size_t)b * UNI_C + tid];
  __syncthreads();
  const int fr = tid >> 5, cl = tid & 31, c = cl * 8;
  const int f0 = (int)((long)s * T / S), f1 = (int)((long)(s + 1) * T / S);
  constexpr int FB = 4;  // frames per thread per round: loads issued together, then the stores
  for (int jb = f0 + fr; jb < f1; jb += 8 * FB) {
    u32x4 wv[FB];
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const int j = min(jb + 8 * i, f1 - 1);
      wv[i] = *reinterpret_cast<const u32x4*>(x + ((size_t)b * T + j) * UNI_C + c);
    }
#pragma unroll
    for (int i = 0; i < FB; ++i) {
      const int j = jb + 8 * i;
      if (j >= f1) break;
      u32x4 w = wv[i];
      float v[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        const bf16 lo = (bf16)(__uint_as_float(w[e] << 16) + ob[c + 2 * e]);
        const bf16 hi = (bf16)(__uint_as_float(w[e] & 0xffff0000u) + ob[c + 2 * e + 1]);
        v[2 * e] = (float)lo;
        v[2 * e + 1] = (float)hi;
        w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
      }
      *reinterpret_cast<u32x4*>(x + ((size_t)b * T + j) * UNI_C + c) = w;
      // (mean, M2) of the 64-channel slab (8 lanes x 8 channels), two-pass over the stored values
      float sm = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) sm += __shfl_xor(sm, o, 64);
      const float mu = sm * (1.f / 64.f);
      float q = 0.f;  // fused multiply-adds spelled out: mt_ffn's fold of this pass computes the same bits
#pragma unroll
      for (int e = 0; e < 8; ++e) q = __builtin_fmaf(v[e] - mu, v[e] - mu, q);
#pragma unroll
      for (int o = 1; o < 8; o <<= 1) q += __shfl_xor(q, o, 64);
      if ((cl & 7) == 0) *reinterpret_cast<float2*>(row_out + 2 * (((size_t)b * T + j) * 4 + (cl >> 3))) = float2{mu, q};
    }
  }
}

// the masked-sum pass streams x once: finer slices (up to 32 per utterance) for more workgroups in flight
int uniform_part_slices(int T) { return std::max(1, std::min(UNI_PSMAX, T / 24)); }
size_t uniform_attention_floats(int B) { return (size_t)B * (UNI_PSMAX * UNI_PART + UNI_C); }

const float* uniform_attention_ovec(const float* part, int B) { return part + (size_t)B * UNI_PSMAX * UNI_PART; }

int launch_uniform_attention(void* x, const float* mask, int B, int T, const void* wqkv, int mq, const float* bqkv,
                             const void* wout, const float* bout, float* part, float* row_out, hipStream_t st,
                             bool apply) {
  MT_REQUIRE(x && mask && wqkv && bqkv && wout && bout && part && (row_out || !apply) && B > 0 && T > 0 && mq == 384,
             "uniform attention: arguments (C = 256, 2 heads x 64)");
  const int SP = uniform_part_slices(T);
  float* ovec = part + (size_t)B * UNI_PSMAX * UNI_PART;  // [B][256] after the slice sums (uniform_attention_floats)
  const int xr = xcd_remap_for((size_t)B * T * UNI_C * sizeof(bf16));
  hipLaunchKernelGGL(attn_uni_part_kernel, dim3(SP, B), dim3(256), 0, st, (const bf16*)x, mask, T, part, xr);
  hipLaunchKernelGGL(attn_uni_vec_kernel, dim3(B), dim3(256), 0, st, SP, (const float*)part, (const bf16*)wqkv, mq,
                     bqkv, (const bf16*)wout, bout, ovec);
  if (apply)
    hipLaunchKernelGGL(attn_uni_apply_kernel, dim3(SP, B), dim3(256), 0, st, (bf16*)x, T, (const float*)ovec, row_out,
                     xr);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int launch_attention(int dtype, const void* qkv, const float* mask, void* out, int B, int T,
                     int heads, hipStream_t stream, float* part) {
  MT_REQUIRE(B > 0 && T > 0 && heads > 0, "attention: empty geometry");
  const int inner = heads * 64;
  const int esz = dtype == BF16 ? 2 : 4;
  const size_t row = 64 * esz + 16;
  const size_t lds = 3 * 64 * row + 4 * 64 * sizeof(float);
  const int nkt = (T + 63) / 64;
  const int NS = part ? attn_splits(T) : 1;
  dim3 grid((unsigned)nkt, (unsigned)heads, (unsigned)(B * NS));
  if (dtype == BF16)
    hipLaunchKernelGGL(attn_kernel<bf16>, grid, dim3(256), lds, stream, (const bf16*)qkv, mask,
                       (bf16*)out, T, inner, NS, part);
  else
    hipLaunchKernelGGL(attn_kernel<float>, grid, dim3(256), lds, stream, (const float*)qkv, mask,
                       (float*)out, T, inner, NS, part);
  MT_CHECK_HIP(hipGetLastError());
  if (NS > 1) {
    dim3 mg((unsigned)nkt, (unsigned)heads, (unsigned)B);
    if (dtype == BF16)
      hipLaunchKernelGGL(attn_merge_kernel<bf16>, mg, dim3(256), 0, stream, part, mask, (bf16*)out, T, inner, NS);
    else
      hipLaunchKernelGGL(attn_merge_kernel<float>, mg, dim3(256), 0, stream, part, mask, (float*)out, T, inner, NS);
    MT_CHECK_HIP(hipGetLastError());
  }
  return 0;
}

}  // namespace mt
