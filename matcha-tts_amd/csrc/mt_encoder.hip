// Text encoder + duration predictor on the GPU (model.py:148-535).
//
//   ids [B][Tx] -> emb * sqrt(C) -> prenet: 3 x (conv_k5(h*m) -> LN -> ReLU), (x + proj(h)) * m
//   [-> ++ spks]  -> 6 x { x*m; x = LN1(x + conv_o(RoPE-MHA(x))); x = LN2(x + conv_2(relu(conv_1(x*m))*m)*m) } * m
//   mu = proj_m(x) * m                                     -> [B][80][Tx] fp32
//   logw = proj(LN(relu(conv_2(LN(relu(conv_1(x*m)))*m)))*m) * m   -> [B][1][Tx] fp32
// Activations are [B][Tx][C] (channel-contiguous) in the element type; every Conv1d / 1x1 projection
// runs on the implicit-GEMM conv kernel (mt_conv.h) with its mask / ReLU / residual fused, LayerNorms
// run as one-wave-per-frame row kernels, attention as a RoPE-fused online-softmax kernel with the
// reference's mask semantics (scores of masked (query, key) pairs := -1e4, model.py:353-354).
#include <math.h>

#include <algorithm>

#include "mt_model.h"
#include "mt_vconv.h"

namespace mt {

// ---------------------------------------------------------------------------------------
// embedding (model.py:522) and x_mask (sequence_mask, model.py:42-46)
// ---------------------------------------------------------------------------------------
template <class E>
__global__ void embed_kernel(const long long* __restrict__ ids, const long long* __restrict__ xlen, int Tx,
                             const float* __restrict__ emb, int nvocab, int C, float scale, E* __restrict__ out,
                             float* __restrict__ xmask, int* __restrict__ oov) {
  const int row = blockIdx.x;  // b * Tx + t
  const int b = row / Tx, t = row - b * Tx;
  long long id = ids[row];
  // nn.Embedding rejects an id outside [0, n_vocab) anywhere in x, padding included (model.py:522): flag it for the
  // host (the caller raises IndexError at its next sync), and read a valid row so no access leaves the table
  if (id < 0 || id >= nvocab) {
    if (oov && threadIdx.x == 0) oov[0] = 1;
    id = id < 0 ? 0 : nvocab - 1;
  }
  const float* e = emb + (size_t)id * C;
  // stored masked: every consumer reads x * x_mask (the prenet's first conv, model.py:203; its residual x_org is
  // masked again by the prenet's final `* x_mask`, model.py:208), so no conv needs a mask prologue
  const float m = (long long)t < xlen[b] ? 1.f : 0.f;
  for (int c = threadIdx.x; c < C; c += blockDim.x) out[(size_t)row * C + c] = from_f<E>(e[c] * scale * m);
  if (threadIdx.x == 0) xmask[row] = m;
}

// ---------------------------------------------------------------------------------------
// LayerNorm over channels of one frame (model.py:152-161: mean, mean((x-mean)^2), rsqrt(var+eps)),
// one wave per frame; optional ReLU after it (prenet order, model.py:203-205) and frame mask.
// ---------------------------------------------------------------------------------------
template <class E, int VPL>
__global__ __launch_bounds__(256) void rowln_kernel(const E* __restrict__ x, int rows, int C,
                                                    const float* __restrict__ g, const float* __restrict__ bt,
                                                    float eps, const float* __restrict__ mask, int relu,
                                                    E* __restrict__ y, bf16* __restrict__ ys) {
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (row >= rows) return;
  const E* xr = x + (size_t)row * C;
  float v[VPL];
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    v[i] = c < C ? to_f(xr[c]) : 0.f;
    s += v[i];
  }
  const float mean = wave_sum(s) / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    const float d = c < C ? v[i] - mean : 0.f;
    q += d * d;
  }
  const float rstd = 1.f / sqrtf(wave_sum(q) / (float)C + eps);
  const float m = mask ? mask[row] : 1.f;
#pragma unroll
  for (int i = 0; i < VPL; ++i) {
    const int c = lane + 64 * i;
    if (c >= C) continue;
    float o = (v[i] - mean) * rstd * g[c] + bt[c];
    if (relu) o = fmaxf(o, 0.f);
    y[(size_t)row * C + c] = from_f<E>(o * m);
    if (ys) {  // the split-bf16 convs' input (VConvArgs::f32 == 2): planes h1 h1 h1 h2 h2 h3 of the stored value
      bf16 h[3];
      split3_bf16((float)from_f<E>(o * m), h[0], h[1], h[2]);
      bf16* yr = ys + (size_t)row * 6 * C + c;
#pragma unroll
      for (int pl = 0; pl < 6; ++pl) yr[pl * C] = h[pl < 3 ? 0 : pl < 5 ? 1 : 2];
    }
  }
}

// ---------------------------------------------------------------------------------------
// RoPE (RotaryPositionalEmebeddings.forward, model.py:276-290) applied in place to the q and k parts of
// qkv [B][Tx][3W]: for head h, pair (i, i + d/2) of the first d = dk/2 dims, angle t * theta_i
// (the cached cos/sin table, idx_theta2 = [idx_theta, idx_theta]); x_rope*cos + neg_half(x_rope)*sin.
// ---------------------------------------------------------------------------------------
template <class E>
__global__ void rope_kernel(E* __restrict__ qkv, int rows, int Tx, int W, int heads, int dk,
                            const float* __restrict__ theta) {
  const int hr = dk / 4;
  const size_t total = (size_t)rows * 2 * heads * hr;
  for (size_t e = blockIdx.x * (size_t)blockDim.x + threadIdx.x; e < total; e += (size_t)gridDim.x * blockDim.x) {
    const int i = (int)(e % hr);
    size_t r = e / hr;
    const int h = (int)(r % heads);
    r /= heads;
    const int part = (int)(r % 2);
    const size_t row = r / 2;
    const int t = (int)(row % Tx);
    E* x = qkv + row * 3 * W + part * W + h * dk;
    const float ang = (float)t * theta[i];
    const float cs = cosf(ang), sn = sinf(ang);
    const float a = to_f(x[i]), b = to_f(x[i + hr]);
    x[i] = from_f<E>(a * cs - b * sn);
    x[i + hr] = from_f<E>(b * cs + a * sn);
  }
}

// ---------------------------------------------------------------------------------------
// The same attention core for bf16 and dk = 96 on MFMA (v_mfma_f32_16x16x32_bf16). Workgroup = 64 queries
// (4 waves x 16) of one (utterance, head); key tiles of 64 stream through LDS.
//   S^T = K . Q^T per wave: A = K rows (LDS, 224-byte rows), B = this wave's Q rows (registers, loaded once);
//   two 16-key blocks X / Y per 32-key slice take the keys {0-7, 16-23} / {8-15, 24-31}, so that one
//   v_permlane16_swap of their bf16 probabilities leaves lane row g4 holding keys 8 g4 .. 8 g4 + 7 of one
//   query: exactly the B operand of O^T = V^T . P^T, with A = V^T rows (LDS, transposed at staging,
//   160-byte rows). Both LDS strides make every ds_read_b128 lane group conflict-free (exhaustive check).
// Per query the softmax runs online over the key tiles in fp32 (max / sum over the 4 lanes holding its keys);
// P enters the second product as bf16. Masked (query, key) pairs := -1e4 as the reference; key tiles that
// are all padding and query tiles that are all padding are skipped exactly as in enc_attn_kernel.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_attn_mfma96_kernel(const bf16* __restrict__ qkv,
                                                              const float* __restrict__ xmask, float sdiv, int Tx,
                                                              int heads, bf16* __restrict__ out) {
  constexpr int DK = 96, KRS = 224, VRS = 160;
  __shared__ __attribute__((aligned(16))) char Ks[64 * KRS];
  __shared__ __attribute__((aligned(16))) char Vt[DK * VRS];
  __shared__ float km[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = lane >> 4, l16 = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, t0 = blockIdx.x * 64;
  const int W = heads * DK, ld = 3 * W;
  const bf16* base = qkv + (size_t)b * Tx * ld + h * DK;
  const int tq = t0 + 16 * wave + l16;  // this lane's query (column of S^T / O^T)
  bf16x8 qf[3];
#pragma unroll
  for (int ks = 0; ks < 3; ++ks)
    qf[ks] = *reinterpret_cast<const bf16x8*>(base + (size_t)min(tq, Tx - 1) * ld + ks * 32 + 8 * g4);
  const float mq = tq < Tx ? xmask[(size_t)b * Tx + tq] : 0.f;
  f32x4 o[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, lrun = 0.f;
  auto keyX = [](int i) { return i < 8 ? i : i + 8; };
  auto keyY = [](int i) { return i < 8 ? i + 8 : i + 16; };
  const bool any_q = __syncthreads_or(mq != 0.f);
  for (int k0 = 0; any_q && k0 < Tx; k0 += 64) {
    const bool kval = tid < 64 && k0 + tid < Tx && xmask[(size_t)b * Tx + k0 + tid] != 0.f;
    if (!__syncthreads_or(kval)) continue;
    // K rows as they are; V transposed (dim-major) for the A operand of O^T
#pragma unroll
    for (int i = 0; i < 3; ++i) {
      const int e = tid + 256 * i, r = e / 12, c = e - r * 12;
      const int t = k0 + r;
      u32x4 kv = {0u, 0u, 0u, 0u}, vv = {0u, 0u, 0u, 0u};
      if (t < Tx) {
        const bf16* src = base + (size_t)t * ld + c * 8;
        kv = *reinterpret_cast<const u32x4*>(src + W);
        vv = *reinterpret_cast<const u32x4*>(src + 2 * W);
      }
      *reinterpret_cast<u32x4*>(Ks + r * KRS + c * 16) = kv;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        *reinterpret_cast<uint16_t*>(Vt + (c * 8 + 2 * j) * VRS + r * 2) = (uint16_t)(vv[j] & 0xffffu);
        *reinterpret_cast<uint16_t*>(Vt + (c * 8 + 2 * j + 1) * VRS + r * 2) = (uint16_t)(vv[j] >> 16);
      }
    }
    if (tid < 64) km[tid] = k0 + tid < Tx ? xmask[(size_t)b * Tx + k0 + tid] : 0.f;
    __syncthreads();
    // S^T for the tile: blocks (X, Y) of slices 0 and 1
    f32x4 s[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      s[s2][0] = s[s2][1] = f32x4{0.f, 0.f, 0.f, 0.f};
      const char* ax = Ks + (32 * s2 + keyX(l16)) * KRS + g4 * 16;
      const char* ay = Ks + (32 * s2 + keyY(l16)) * KRS + g4 * 16;
#pragma unroll
      for (int ks = 0; ks < 3; ++ks) {
        s[s2][0] = mfma16(*reinterpret_cast<const bf16x8*>(ax + ks * 64), qf[ks], s[s2][0]);
        s[s2][1] = mfma16(*reinterpret_cast<const bf16x8*>(ay + ks * 64), qf[ks], s[s2][1]);
      }
    }
    // scale, mask, online softmax (this lane: 16 keys of query tq; the other 48 keys on lanes l16 + 16 j)
    float cmax = -INFINITY;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2)
#pragma unroll
      for (int xy = 0; xy < 2; ++xy)
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int kk = 32 * s2 + (xy ? keyY(4 * g4 + r) : keyX(4 * g4 + r));
          float sc = s[s2][xy][r] / sdiv;
          if (mq * km[kk] == 0.f) sc = -1e4f;
          if (k0 + kk >= Tx) sc = -INFINITY;
          s[s2][xy][r] = sc;
          cmax = fmaxf(cmax, sc);
        }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
    const float mnew = fmaxf(mrun, cmax);
    const float corr = expf(mrun - mnew);
    lrun *= corr;
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] *= corr;
    mrun = mnew;
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
      uint32_t pk[2][2];
#pragma unroll
      for (int xy = 0; xy < 2; ++xy) {
        float p[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          p[r] = expf(s[s2][xy][r] - mnew);
          lrun += p[r];
        }
        pk[xy][0] = (uint32_t)__builtin_bit_cast(uint16_t, (bf16)p[0]) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, (bf16)p[1]) << 16);
        pk[xy][1] = (uint32_t)__builtin_bit_cast(uint16_t, (bf16)p[2]) |
                    ((uint32_t)__builtin_bit_cast(uint16_t, (bf16)p[3]) << 16);
      }
      const auto r0 = __builtin_amdgcn_permlane16_swap(pk[0][0], pk[1][0], false, false);
      const auto r1 = __builtin_amdgcn_permlane16_swap(pk[0][1], pk[1][1], false, false);
      const u32x4 pb = {r0[0], r1[0], r0[1], r1[1]};  // keys 32 s2 + 8 g4 .. + 7 of query tq
      const bf16x8 bp = __builtin_bit_cast(bf16x8, pb);
#pragma unroll
      for (int db = 0; db < 6; ++db)
        o[db] = mfma16(*reinterpret_cast<const bf16x8*>(Vt + (16 * db + l16) * VRS + (4 * s2 + g4) * 16), bp, o[db]);
    }
    __syncthreads();
  }
  lrun += __shfl_xor(lrun, 16, 64);
  lrun += __shfl_xor(lrun, 32, 64);
  if (tq < Tx) {
    const float inv = lrun > 0.f ? 1.f / lrun : 0.f;
    bf16* dst = out + ((size_t)b * Tx + tq) * W + h * DK + 4 * g4;
#pragma unroll
    for (int db = 0; db < 6; ++db) {
      const uint32_t w0 = (uint32_t)__builtin_bit_cast(uint16_t, (bf16)(o[db][0] * inv)) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (bf16)(o[db][1] * inv)) << 16);
      const uint32_t w1 = (uint32_t)__builtin_bit_cast(uint16_t, (bf16)(o[db][2] * inv)) |
                          ((uint32_t)__builtin_bit_cast(uint16_t, (bf16)(o[db][3] * inv)) << 16);
      *reinterpret_cast<uint2*>(dst + 16 * db) = make_uint2(w0, w1);
    }
  }
}

// ---------------------------------------------------------------------------------------
// The attention core in fp32 and dk = 96 on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32, 4 per mfma16): the text
// encoder runs fp32 in both model precisions (its logw drives the exact index path). Workgroup = 64 queries
// (4 waves x 16) of one (utterance, head); key tiles of 64 through LDS.
//   S^T = K . Q^T: A = K rows (LDS, 416-byte rows), B = this wave's Q rows (registers, loaded once). The f32
//   MFMA's output layout (lane (g, q) holds keys 4g..4g+3 of query q) IS its B-operand layout, so the
//   probabilities feed O^T = V^T . P^T straight from registers, with A = V^T rows (LDS, transposed at staging,
//   288-byte rows). Both strides make every ds_read_b128 lane group conflict-free for any 16-byte offset.
// Softmax online in fp32 over the key tiles; masked (query, key) pairs := -1e4 as the reference
// (model.py:353-354); all-padding key tiles and query tiles skipped exactly as in enc_attn_kernel.
// ---------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void enc_attn_mfma96f_kernel(const float* __restrict__ qkv,
                                                               const float* __restrict__ xmask, float sdiv, int Tx,
                                                               int heads, float* __restrict__ out) {
  constexpr int DK = 96, KRS = 104, VRS = 72;  // row strides in floats
  __shared__ __attribute__((aligned(16))) float Ks[64 * KRS];
  __shared__ __attribute__((aligned(16))) float Vt[DK * VRS];
  __shared__ float km[64];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int g4 = lane >> 4, l16 = lane & 15;
  const int h = blockIdx.y, b = blockIdx.z, t0 = blockIdx.x * 64;
  const int W = heads * DK, ld = 3 * W;
  const float* base = qkv + (size_t)b * Tx * ld + h * DK;
  const int tq = t0 + 16 * wave + l16;  // this lane's query (column of S^T / O^T)
  f32x4 qf[6];
#pragma unroll
  for (int j = 0; j < 6; ++j)
    qf[j] = *reinterpret_cast<const f32x4*>(base + (size_t)min(tq, Tx - 1) * ld + 16 * j + 4 * g4);
  const float mq = tq < Tx ? xmask[(size_t)b * Tx + tq] : 0.f;
  f32x4 o[6];
#pragma unroll
  for (int i = 0; i < 6; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
  float mrun = -INFINITY, lrun = 0.f;
  const bool any_q = __syncthreads_or(mq != 0.f);
  for (int k0 = 0; any_q && k0 < Tx; k0 += 64) {
    const bool kval = tid < 64 && k0 + tid < Tx && xmask[(size_t)b * Tx + k0 + tid] != 0.f;
    if (!__syncthreads_or(kval)) continue;
#pragma unroll
    for (int i = 0; i < 6; ++i) {  // 64 rows x 24 chunks of 4 floats
      const int e = tid + 256 * i, r = e / 24, c = e - r * 24;
      const int t = k0 + r;
      f32x4 kv = {0.f, 0.f, 0.f, 0.f}, vv = {0.f, 0.f, 0.f, 0.f};
      if (t < Tx) {
        const float* src = base + (size_t)t * ld + 4 * c;
        kv = *reinterpret_cast<const f32x4*>(src + W);
        vv = *reinterpret_cast<const f32x4*>(src + 2 * W);
      }
      *reinterpret_cast<f32x4*>(Ks + r * KRS + 4 * c) = kv;
#pragma unroll
      for (int j = 0; j < 4; ++j) Vt[(4 * c + j) * VRS + r] = vv[j];
    }
    if (tid < 64) km[tid] = k0 + tid < Tx ? xmask[(size_t)b * Tx + k0 + tid] : 0.f;
    __syncthreads();
    f32x4 s[4];  // block kb: keys 16 kb + 4 g4 + i of query tq
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      s[kb] = f32x4{0.f, 0.f, 0.f, 0.f};
      const float* ak = Ks + (16 * kb + l16) * KRS + 4 * g4;
#pragma unroll
      for (int j = 0; j < 6; ++j) s[kb] = mfma16(*reinterpret_cast<const f32x4*>(ak + 16 * j), qf[j], s[kb]);
    }
    float cmax = -INFINITY;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb)
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int kk = 16 * kb + 4 * g4 + r;
        float sc = s[kb][r] / sdiv;
        if (mq * km[kk] == 0.f) sc = -1e4f;
        if (k0 + kk >= Tx) sc = -INFINITY;
        s[kb][r] = sc;
        cmax = fmaxf(cmax, sc);
      }
    cmax = fmaxf(cmax, __shfl_xor(cmax, 16, 64));
    cmax = fmaxf(cmax, __shfl_xor(cmax, 32, 64));
    const float mnew = fmaxf(mrun, cmax);
    const float corr = expf(mrun - mnew);
    lrun *= corr;
#pragma unroll
    for (int i = 0; i < 6; ++i) o[i] *= corr;
    mrun = mnew;
#pragma unroll
    for (int kb = 0; kb < 4; ++kb) {
      f32x4 p;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        p[r] = expf(s[kb][r] - mnew);
        lrun += p[r];
      }
#pragma unroll
      for (int db = 0; db < 6; ++db)
        o[db] = mfma16(*reinterpret_cast<const f32x4*>(Vt + (16 * db + l16) * VRS + 16 * kb + 4 * g4), p, o[db]);
    }
    __syncthreads();
  }
  lrun += __shfl_xor(lrun, 16, 64);
  lrun += __shfl_xor(lrun, 32, 64);
  if (tq < Tx) {
    const float inv = lrun > 0.f ? 1.f / lrun : 0.f;
    float* dst = out + ((size_t)b * Tx + tq) * W + h * DK + 4 * g4;
#pragma unroll
    for (int db = 0; db < 6; ++db) *reinterpret_cast<f32x4*>(dst + 16 * db) = o[db] * inv;
  }
}

// ---------------------------------------------------------------------------------------
// Multi-head self-attention core (MultiHeadAttention.attention, model.py:343-364) on RoPE'd qkv.
// Workgroup = 64 queries x 4 lanes of one (utterance, head); lane p of a query owns dk/4 dims of q and
// of its output. Keys stream through LDS 64 at a time; scores = q.k / sqrt(dk), masked (query, key)
// pairs := -1e4 (x_mask_i * x_mask_j == 0), online softmax over all Tx keys, out [B][Tx][W].
// ---------------------------------------------------------------------------------------
template <class E, int DK>
__global__ __launch_bounds__(256) void enc_attn_kernel(const E* __restrict__ qkv, const float* __restrict__ xmask,
                                                       float sdiv, int Tx, int heads, E* __restrict__ out) {
  constexpr int DP = DK / 4;   // dims per lane
  constexpr int KS = DK + 4;   // LDS row (floats): 16-byte aligned, rows offset by 4 banks
  __shared__ __attribute__((aligned(16))) float Ks[64 * KS];
  __shared__ __attribute__((aligned(16))) float Vs[64 * KS];
  __shared__ float km[64];
  const int tid = threadIdx.x;
  const int qi = tid >> 2, p = tid & 3;
  const int h = blockIdx.y, b = blockIdx.z;
  const int t0 = blockIdx.x * 64;
  const int W = heads * DK, ld = 3 * W;
  const E* base = qkv + (size_t)b * Tx * ld + h * DK;

  const int tq = t0 + qi;
  float q[DP], o[DP];
  {
    const E* src = base + (size_t)min(tq, Tx - 1) * ld + p * DP;
#pragma unroll
    for (int i = 0; i < DP; ++i) {
      q[i] = to_f(src[i]);
      o[i] = 0.f;
    }
  }
  const float mq = tq < Tx ? xmask[(size_t)b * Tx + tq] : 0.f;
  // A tile of padded queries only: their rows are zeroed downstream (the FFN and LayerNorm outputs are
  // masked) and never read unmasked, so they are written as 0.
  if (!__syncthreads_or(mq != 0.f)) {
    if (tq < Tx) {
      E* dst = out + ((size_t)b * Tx + tq) * W + h * DK + p * DP;
#pragma unroll
      for (int i = 0; i < DP; ++i) dst[i] = from_f<E>(0.f);
    }
    return;
  }
  float mrun = -INFINITY, lrun = 0.f;
  for (int k0 = 0; k0 < Tx; k0 += 64) {
    // a tile of padded keys only adds exp(-1e4 - m) == 0 for every valid query: skipped (exact)
    const bool kval = tid < 64 && k0 + tid < Tx && xmask[(size_t)b * Tx + k0 + tid] != 0.f;
    if (!__syncthreads_or(kval)) continue;
    // 16-byte loads of K and V rows, widened to fp32 in LDS
    constexpr int VN = Vec16<E>::N, VPR = DK / VN;
    for (int e = tid; e < 64 * VPR; e += 256) {
      const int r = e / VPR, c = e - r * VPR;
      const int t = k0 + r;
      Vec16<E> kv = zero16<E>(), vv = zero16<E>();
      if (t < Tx) {
        const E* src = base + (size_t)t * ld + c * VN;
        kv = load16(src + W);
        vv = load16(src + 2 * W);
      }
#pragma unroll
      for (int i = 0; i < VN; i += 4) {
        *reinterpret_cast<f32x4*>(Ks + r * KS + c * VN + i) = f32x4{kv.get(i), kv.get(i + 1), kv.get(i + 2), kv.get(i + 3)};
        *reinterpret_cast<f32x4*>(Vs + r * KS + c * VN + i) = f32x4{vv.get(i), vv.get(i + 1), vv.get(i + 2), vv.get(i + 3)};
      }
    }
    if (tid < 64) km[tid] = k0 + tid < Tx ? xmask[(size_t)b * Tx + k0 + tid] : 0.f;
    __syncthreads();
    const int nk = min(64, Tx - k0);
    float s[64];
    float cmax = -INFINITY;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const f32x4* kr = reinterpret_cast<const f32x4*>(Ks + j * KS + p * DP);
      float d = 0.f;
#pragma unroll
      for (int i = 0; i < DP / 4; ++i) {
        const f32x4 kk = kr[i];
        d += q[4 * i] * kk[0] + q[4 * i + 1] * kk[1] + q[4 * i + 2] * kk[2] + q[4 * i + 3] * kk[3];
      }
      d += __shfl_xor(d, 1, 64);
      d += __shfl_xor(d, 2, 64);
      float sc = d / sdiv;
      if (mq * km[j] == 0.f) sc = -1e4f;
      s[j] = j < nk ? sc : -INFINITY;
      cmax = fmaxf(cmax, s[j]);
    }
    const float mnew = fmaxf(mrun, cmax);
    const float corr = expf(mrun - mnew);
    lrun *= corr;
#pragma unroll
    for (int i = 0; i < DP; ++i) o[i] *= corr;
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const float pj = expf(s[j] - mnew);
      lrun += pj;
      const f32x4* vr = reinterpret_cast<const f32x4*>(Vs + j * KS + p * DP);
#pragma unroll
      for (int i = 0; i < DP / 4; ++i) {
        const f32x4 vv = vr[i];
        o[4 * i] += pj * vv[0];
        o[4 * i + 1] += pj * vv[1];
        o[4 * i + 2] += pj * vv[2];
        o[4 * i + 3] += pj * vv[3];
      }
    }
    mrun = mnew;
  }
  if (tq < Tx) {
    E* dst = out + ((size_t)b * Tx + tq) * W + h * DK + p * DP;
#pragma unroll
    for (int i = 0; i < DP; ++i) dst[i] = from_f<E>(o[i] / lrun);
  }
}

// ---------------------------------------------------------------------------------------
// host
// ---------------------------------------------------------------------------------------
int Encoder::init(int n_vocab_, int n_ch, int filt, int heads_, int layers_, int ksize, int n_spks_, int spk_dim_,
                  int dp_filt, int dp_k, int prenet_, int dtype_) {
  MT_REQUIRE(n_vocab_ > 0 && n_ch > 0 && filt > 0 && layers_ >= 1 && ksize >= 1 && dp_k >= 1, "encoder: config");
  MT_REQUIRE(dtype_ == F32 || dtype_ == BF16, "encoder: dtype");
  n_vocab = n_vocab_;
  C = n_ch;
  F = filt;
  heads = heads_;
  layers = layers_;
  k = ksize;
  n_spks = n_spks_;
  spk_dim = n_spks > 1 ? spk_dim_ : 0;
  W = C + spk_dim;
  DF = dp_filt;
  dpk = dp_k;
  prenet = prenet_;
  dtype = dtype_;
  esize = dtype == BF16 ? 2 : 4;
  MT_REQUIRE(W % heads == 0, "encoder: width %d not divisible by %d heads", W, heads);
  dk = W / heads;
  MT_REQUIRE(dk == 96 || dk == 128 || dk == 64, "encoder: head dim %d not compiled in (64/96/128)", dk);
  MT_REQUIRE(C <= 1024 && W <= 1024 && F <= 1024 && DF <= 1024, "encoder: width");
  const int align = 64 / esize;
  MT_REQUIRE(C % 16 == 0 && W % 16 == 0 && F % align == 0 && DF % align == 0, "encoder: channels must be 16-aligned");
  Packer pk;
  ParamList& L = params;
  L = ParamList();
  lay.clear();
  pre.clear();
  ezero_off = 0;
  const long long Cl = C, Wl = W;
  emb = L.add("emb.weight", {n_vocab, Cl});
  emb_off = pk.take((size_t)n_vocab * C * 4);
  if (prenet) {
    for (int i = 0; i < 3; ++i) {
      const std::string p = "prenet.";
      int w = L.add(p + "conv_layers." + std::to_string(i) + ".weight", {Cl, Cl, 5});
      int b = L.add(p + "conv_layers." + std::to_string(i) + ".bias", {Cl});
      Pre q;
      q.conv = make_conv(C, C, 5, 1, 2, 1, {w}, b, esize, pk);
      q.g = L.add(p + "norm_layers." + std::to_string(i) + ".gamma", {Cl});
      q.b = L.add(p + "norm_layers." + std::to_string(i) + ".beta", {Cl});
      q.ln_off = pk.take(2 * C * 4);
      pre.push_back(q);
    }
    int w = L.add("prenet.proj.weight", {Cl, Cl, 1});
    int b = L.add("prenet.proj.bias", {Cl});
    pre_proj = make_conv(C, C, 1, 1, 0, 1, {w}, b, esize, pk);
  }
  for (int i = 0; i < layers; ++i) {
    const std::string a = "encoder.attn_layers." + std::to_string(i) + ".";
    const std::string f = "encoder.ffn_layers." + std::to_string(i) + ".";
    Layer l;
    int wq = L.add(a + "conv_q.weight", {Wl, Wl, 1});
    int bq = L.add(a + "conv_q.bias", {Wl});
    int wk = L.add(a + "conv_k.weight", {Wl, Wl, 1});
    int bk = L.add(a + "conv_k.bias", {Wl});
    int wv = L.add(a + "conv_v.weight", {Wl, Wl, 1});
    int bv = L.add(a + "conv_v.bias", {Wl});
    int wo = L.add(a + "conv_o.weight", {Wl, Wl, 1});
    int bo = L.add(a + "conv_o.bias", {Wl});
    l.n1g = L.add("encoder.norm_layers_1." + std::to_string(i) + ".gamma", {Wl});
    l.n1b = L.add("encoder.norm_layers_1." + std::to_string(i) + ".beta", {Wl});
    int w1 = L.add(f + "conv_1.weight", {(long long)F, Wl, k});
    int b1 = L.add(f + "conv_1.bias", {(long long)F});
    int w2 = L.add(f + "conv_2.weight", {Wl, (long long)F, k});
    int b2 = L.add(f + "conv_2.bias", {Wl});
    l.n2g = L.add("encoder.norm_layers_2." + std::to_string(i) + ".gamma", {Wl});
    l.n2b = L.add("encoder.norm_layers_2." + std::to_string(i) + ".beta", {Wl});
    l.qkv = make_conv(3 * W, W, 1, 1, 0, 1, {wq, wk, wv}, -1, esize, pk);
    l.qkv.bsrcs = {bq, bk, bv};
    l.o = make_conv(W, W, 1, 1, 0, 1, {wo}, bo, esize, pk);
    l.f1 = make_conv(F, W, k, 1, k / 2, 1, {w1}, b1, esize, pk);
    l.f2 = make_conv(W, F, k, 1, k / 2, 1, {w2}, b2, esize, pk);
    if (dtype == BF16 && vconv_supported(W, F, k, 1, 1) && vconv_supported(F, W, k, 1, 1)) {
      // the FFN convs on mt_vconv: their inputs are stored masked by their producers (LN1, FFN conv 1)
      for (GemmW* g : {&l.f1, &l.f2}) {
        g->vc = true;
        g->v_off = pk.take(vconv_packed_bytes(g->cin, g->cout, g->k));
      }
      if (!ezero_off) ezero_off = pk.take(256);
    }
    l.n1_off = pk.take(2 * W * 4);
    l.n2_off = pk.take(2 * W * 4);
    lay.push_back(l);
  }
  {
    int w = L.add("proj_m.weight", {80, Wl, 1});
    int b = L.add("proj_m.bias", {80});
    proj_m = make_conv(80, W, 1, 1, 0, 1, {w}, b, esize, pk);
  }
  {
    const long long D = DF;
    int w1 = L.add("proj_w.conv_1.weight", {D, Wl, dpk});
    int b1 = L.add("proj_w.conv_1.bias", {D});
    dn1g = L.add("proj_w.norm_1.gamma", {D});
    dn1b = L.add("proj_w.norm_1.beta", {D});
    int w2 = L.add("proj_w.conv_2.weight", {D, D, dpk});
    int b2 = L.add("proj_w.conv_2.bias", {D});
    dn2g = L.add("proj_w.norm_2.gamma", {D});
    dn2b = L.add("proj_w.norm_2.beta", {D});
    int wp = L.add("proj_w.proj.weight", {1, D, 1});
    int bp = L.add("proj_w.proj.bias", {1});
    dp1 = make_conv(DF, W, dpk, 1, dpk / 2, 1, {w1}, b1, esize, pk);
    dp2 = make_conv(DF, DF, dpk, 1, dpk / 2, 1, {w2}, b2, esize, pk);
    dpp = make_conv(1, DF, 1, 1, 0, 1, {wp}, bp, esize, pk);
    dn1_off = pk.take(2 * DF * 4);
    dn2_off = pk.take(2 * DF * 4);
  }
  if (dtype == F32) {
    // fp32: every conv / projection whose shapes mt_vconv's fp32 mode takes runs there (LDS-DMA operand staging,
    // exact-fp32 MFMA); proj_m (80 rows) and the duration head (1 row) stay on the generic kernel
    auto vc32 = [&](GemmW& g) {
      if (!vconv_supported_f32(g.cin, g.cout, g.k, g.s) || g.kind != 0) return;
      g.vc = true;
      g.v_off = pk.take(vconv_packed_bytes_f32(g.cin, g.cout, g.k));
      if (!ezero_off) ezero_off = pk.take(256);
    };
    for (Pre& q : pre) vc32(q.conv);
    if (prenet) vc32(pre_proj);
    for (Layer& l : lay) {
      for (GemmW* g : {&l.qkv, &l.o, &l.f1, &l.f2}) vc32(*g);
      // the FFN convs' split-bf16 images (encoder precision "fp32x3", Encoder::split): 6 cin input channels
      if (l.f1.vc && l.f2.vc && (6 * l.f1.cin) % 384 == 0 && (6 * l.f2.cin) % 384 == 0 && l.f1.k >= 2 && l.f2.k >= 2) {
        l.s1_off = pk.take(vconv_packed_bytes_split6(l.f1.cin, l.f1.cout, l.f1.k));
        l.s2_off = pk.take(vconv_packed_bytes_split6(l.f2.cin, l.f2.cout, l.f2.k));
      }
    }
    vc32(dp1);
    vc32(dp2);
  }
  theta = L.add("_rope_theta", {dk / 4});  // 1 / 10000^(arange(0, dk/2, 2) / (dk/2)), host-computed
  theta_off = pk.take(dk / 4 * 4);
  packed_bytes = pk.off;
  return 0;
}

int Encoder::pack(const float* const* p, void* packed, hipStream_t st) const {
  char* P = (char*)packed;
  int rc;
#define PK(expr) \
  if ((rc = (expr)) != 0) return rc
  PK(pack_vec(p[emb], n_vocab * C, n_vocab * C, 0, (float*)(P + emb_off), st));
  for (const Pre& q : pre) {
    PK(pack_gemm(q.conv, dtype, p, P, st));
    PK(pack_vec(p[q.g], C, C, 0, (float*)(P + q.ln_off), st));
    PK(pack_vec(p[q.b], C, C, 0, (float*)(P + q.ln_off) + C, st));
  }
  if (prenet) PK(pack_gemm(pre_proj, dtype, p, P, st));
  for (const Layer& l : lay) {
    PK(pack_gemm(l.qkv, dtype, p, P, st));
    PK(pack_gemm(l.o, dtype, p, P, st));
    PK(pack_gemm(l.f1, dtype, p, P, st));
    PK(pack_gemm(l.f2, dtype, p, P, st));
    for (const GemmW* g : {&l.f1, &l.f2})
      if (g->vc) PK(vconv_repack(P + g->w_off, g->Mpad, g->taps, g->cin_pad, g->cin, g->cout, P + g->v_off, st));
    PK(pack_vec(p[l.n1g], W, W, 0, (float*)(P + l.n1_off), st));
    PK(pack_vec(p[l.n1b], W, W, 0, (float*)(P + l.n1_off) + W, st));
    PK(pack_vec(p[l.n2g], W, W, 0, (float*)(P + l.n2_off), st));
    PK(pack_vec(p[l.n2b], W, W, 0, (float*)(P + l.n2_off) + W, st));
  }
  PK(pack_gemm(proj_m, dtype, p, P, st));
  PK(pack_gemm(dp1, dtype, p, P, st));
  PK(pack_gemm(dp2, dtype, p, P, st));
  PK(pack_gemm(dpp, dtype, p, P, st));
  PK(pack_vec(p[dn1g], DF, DF, 0, (float*)(P + dn1_off), st));
  PK(pack_vec(p[dn1b], DF, DF, 0, (float*)(P + dn1_off) + DF, st));
  PK(pack_vec(p[dn2g], DF, DF, 0, (float*)(P + dn2_off), st));
  PK(pack_vec(p[dn2b], DF, DF, 0, (float*)(P + dn2_off) + DF, st));
  PK(pack_vec(p[theta], dk / 4, dk / 4, 0, (float*)(P + theta_off), st));
  if (dtype == F32) {
    auto rp = [&](const GemmW& g) -> int {
      return g.vc ? vconv_repack_f32(P + g.w_off, g.Mpad, g.taps, g.cin_pad, g.cin, g.cout, P + g.v_off, st) : 0;
    };
    for (const Pre& q : pre) PK(rp(q.conv));
    if (prenet) PK(rp(pre_proj));
    for (const Layer& l : lay) {
      for (const GemmW* g : {&l.qkv, &l.o, &l.f1, &l.f2}) PK(rp(*g));
      if (l.s1_off) {
        PK(vconv_repack_split6(P + l.f1.w_off, l.f1.Mpad, l.f1.taps, l.f1.cin_pad, l.f1.cin, l.f1.cout, P + l.s1_off, st));
        PK(vconv_repack_split6(P + l.f2.w_off, l.f2.Mpad, l.f2.taps, l.f2.cin_pad, l.f2.cin, l.f2.cout, P + l.s2_off, st));
      }
    }
    PK(rp(dp1));
    PK(rp(dp2));
  }
  if (ezero_off) PK(pack_vec(nullptr, 1, 64, 0, (float*)(P + ezero_off), st));
#undef PK
  return 0;
}

// the split-bf16 FFN's 6-plane operands (LN1 output, hidden), bf16
static size_t split_ws(bool on, size_t n, int W, int F) { return on ? align256(n * 6 * W * 2) + align256(n * 6 * F * 2) : 0; }

size_t Encoder::workspace_bytes(int B, int Tx) const {
  const size_t n = (size_t)B * Tx;
  const int wmax = std::max(std::max(W, 3 * W), std::max(F, DF));
  return 5 * align256(n * wmax * esize) + align256(n * 80 * esize) + align256(n * 4) + 4096 +  // + vconv trash
         split_ws(split && dtype == F32, n, W, F);
}

template <class E>
static int rowln(const E* x, int rows, int C, const float* gb, float eps, const float* mask, int relu, E* y,
                 hipStream_t st, bf16* ys = nullptr) {
  const dim3 grid((rows + 3) / 4), blk(256);
  if (C <= 256)
    hipLaunchKernelGGL((rowln_kernel<E, 4>), grid, blk, 0, st, x, rows, C, gb, gb + C, eps, mask, relu, y, ys);
  else if (C <= 512)
    hipLaunchKernelGGL((rowln_kernel<E, 8>), grid, blk, 0, st, x, rows, C, gb, gb + C, eps, mask, relu, y, ys);
  else
    hipLaunchKernelGGL((rowln_kernel<E, 16>), grid, blk, 0, st, x, rows, C, gb, gb + C, eps, mask, relu, y, ys);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

constexpr int kNotVc = 0x7fff0001;  // v32(): the layer is not on mt_vconv's fp32 mode (run the generic kernel)

template <class E>
int Encoder::forward_t(const char* P, const long long* ids, const long long* xlen, const float* spks, int B, int Tx,
                       float* mu, float* logw, float* xmask, int* oov, char* ws, hipStream_t st) const {
  int rc;
  const size_t n = (size_t)B * Tx;
  const int wmax = std::max(std::max(W, 3 * W), std::max(F, DF));
  const size_t big = align256(n * wmax * esize);
  char* X = ws;             // encoder state [B][Tx][W]
  char* A = ws + big;       // scratch
  char* Bb = ws + 2 * big;  // scratch
  char* Q = ws + 3 * big;   // qkv / prenet input
  char* Hh = ws + 4 * big;  // FFN hidden
  char* MU = ws + 5 * big;  // [B][Tx][80]
  const float eps = 1e-4f;
  // fp32: a conv on mt_vconv's fp32 mode (its input stored masked where the reference masks it); kNotVc = not there
  char* trash = MU + align256(n * 80 * esize) + align256(n * 4);
  auto v32 = [&](const GemmW& g, const void* x, void* y, int ef, const void* resid) -> int {
    if (!(std::is_same<E, float>::value && g.vc && f32vc)) return kNotVc;
    VConvArgs a{};
    a.f32 = 1;
    a.x = (const bf16*)x;
    a.B = B;
    a.L = Tx;
    a.cin = g.cin;
    a.w = (const bf16*)(P + g.v_off);
    a.bias = (const float*)(P + g.b_off);
    a.M = a.Mpad = g.cout;
    a.taps = g.k;
    a.dil = 1;
    a.pad = g.pad;
    a.y = (bf16*)y;
    a.resid = (const bf16*)resid;
    a.emask = xmask;
    a.div = 1.f;
    a.zero = (const bf16*)(P + ezero_off);
    a.trash = (bf16*)trash;
    a.probe = -1;
    return launch_vconv(ef, a, st);
  };
  // embedding * sqrt(C) and x_mask (+ the out-of-vocabulary flag)
  if (oov) MT_CHECK_HIP(hipMemsetAsync(oov, 0, sizeof(int), st));
  hipLaunchKernelGGL((embed_kernel<E>), dim3((unsigned)n), dim3(256), 0, st, ids, xlen, Tx, (const float*)(P + emb_off),
                     n_vocab, C, sqrtf((float)C), (E*)Q, xmask, oov);
  MT_CHECK_HIP(hipGetLastError());
  // prenet (ConvReluNorm, model.py:196-208): h = relu(LN(conv(h*m))) x3, x = (x + proj(h)) * m
  const char* cur = Q;
  if (prenet) {
    const char* h = Q;
    char* bufs[2] = {A, Bb};
    for (int i = 0; i < 3; ++i) {
      if ((rc = v32(pre[i].conv, h, Hh, 0, nullptr)) != kNotVc && rc) return rc;
      if (rc == kNotVc) {
        ConvArgs a = gemm_args(pre[i].conv, P, B, Tx);
        a.x0 = h;  // h * m as stored (masked embedding / masked LN output)
        a.y = Hh;
        if ((rc = launch_conv<E, 0, 0>(a, st))) return rc;
      }
      if ((rc = rowln<E>((const E*)Hh, (int)n, C, (const float*)(P + pre[i].ln_off), eps, xmask, 1, (E*)bufs[i & 1], st)))
        return rc;
      h = bufs[i & 1];
    }
    if ((rc = v32(pre_proj, h, W == C ? X : Hh, VE_RESID | VE_MASK, Q)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs a = gemm_args(pre_proj, P, B, Tx);
      a.x0 = h;
      a.y = W == C ? X : Hh;
      a.ldy = C;
      a.resid = Q;
      a.ldr = C;
      a.emask = xmask;
      if ((rc = launch_conv<E, 0, EF_RESID | EF_FMASK>(a, st))) return rc;
    }
    cur = W == C ? X : Hh;
  }
  if (W != C) {  // ++ speaker embedding channels (model.py:526-527), x*m
    if ((rc = spk_fill(dtype, spks, B, spk_dim, Tx, X, W, C, st))) return rc;
    if ((rc = copy_rows(dtype, cur, C, (int)n, C, X, W, st))) return rc;
  } else if (cur != X) {
    if ((rc = copy_rows(dtype, cur, C, (int)n, C, X, W, st))) return rc;
  }
  // encoder layers (model.py:428-439); X holds x*m at every layer entry
  if (!prenet || W != C) {  // mask the layer-0 input (the prenet's epilogue already did when it wrote X)
    if ((rc = mask_rows(dtype, X, (int)n, W, xmask, st))) return rc;
  }
  const float sdiv = sqrtf((float)dk);
  for (int i = 0; i < layers; ++i) {
    const Layer& l = lay[i];
    if ((rc = v32(l.qkv, X, Q, 0, nullptr)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs q = gemm_args(l.qkv, P, B, Tx);
      q.x0 = X;
      q.y = Q;
      if ((rc = launch_conv<E, 0, 0>(q, st))) return rc;
    }
    {
      const size_t pairs = n * 2 * heads * (dk / 4);
      const int blocks = (int)std::min<size_t>((pairs + 255) / 256, 65535);
      hipLaunchKernelGGL((rope_kernel<E>), dim3(blocks), dim3(256), 0, st, (E*)Q, (int)n, Tx, W, heads, dk,
                         (const float*)(P + theta_off));
      MT_CHECK_HIP(hipGetLastError());
    }
    const dim3 ga((Tx + 63) / 64, heads, B);
    if (std::is_same<E, bf16>::value && dk == 96 && mfma_attn)
      hipLaunchKernelGGL(enc_attn_mfma96_kernel, ga, dim3(256), 0, st, (const bf16*)Q, xmask, sdiv, Tx, heads,
                         (bf16*)A);
    else if (std::is_same<E, float>::value && dk == 96 && mfma_attn)
      hipLaunchKernelGGL(enc_attn_mfma96f_kernel, ga, dim3(256), 0, st, (const float*)Q, xmask, sdiv, Tx, heads,
                         (float*)A);
    else if (dk == 96)
      hipLaunchKernelGGL((enc_attn_kernel<E, 96>), ga, dim3(256), 0, st, (const E*)Q, xmask, sdiv, Tx, heads, (E*)A);
    else if (dk == 128)
      hipLaunchKernelGGL((enc_attn_kernel<E, 128>), ga, dim3(256), 0, st, (const E*)Q, xmask, sdiv, Tx, heads, (E*)A);
    else
      hipLaunchKernelGGL((enc_attn_kernel<E, 64>), ga, dim3(256), 0, st, (const E*)Q, xmask, sdiv, Tx, heads, (E*)A);
    MT_CHECK_HIP(hipGetLastError());
    if ((rc = v32(l.o, A, Bb, VE_RESID, X)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs o = gemm_args(l.o, P, B, Tx);
      o.x0 = A;
      o.y = Bb;
      o.resid = X;
      o.ldr = W;
      if ((rc = launch_conv<E, 0, EF_RESID>(o, st))) return rc;
    }
    if constexpr (std::is_same<E, bf16>::value) {
      if (l.f1.vc && l.f2.vc) {
        // FFN on vconv (model.py:119-130): LN1 stores A masked, conv 1 stores relu(.) masked, conv 2 adds the
        // residual and masks (its padded frames differ from the generic order v*m + A, and LN2 masks them)
        if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n1_off), eps, xmask, 0, (E*)A, st)))
          return rc;
        auto vargs = [&](const GemmW& g, const void* x, void* y) {
          VConvArgs a{};
          a.x = (const bf16*)x;
          a.B = B;
          a.L = Tx;
          a.cin = g.cin;
          a.w = (const bf16*)(P + g.v_off);
          a.bias = (const float*)(P + g.b_off);
          a.M = a.Mpad = g.cout;
          a.taps = g.k;
          a.dil = 1;
          a.pad = g.pad;
          a.y = (bf16*)y;
          a.div = 1.f;
          a.zero = (const bf16*)(P + ezero_off);
          a.trash = (bf16*)trash;
          a.emask = xmask;
          a.probe = -1;
          return a;
        };
        if ((rc = launch_vconv(VE_RELU | VE_MASK, vargs(l.f1, A, Hh), st))) return rc;
        VConvArgs f2 = vargs(l.f2, Hh, Bb);
        f2.resid = (const bf16*)A;
        if ((rc = launch_vconv(VE_RESID | VE_MASK, f2, st))) return rc;
        if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n2_off), eps, xmask, 0, (E*)X, st)))
          return rc;
        continue;
      }
    }
    // FFN (model.py:375-393) on masked operands: LN1 stores x*m, conv 1 stores relu(.)*m, conv 2 adds the
    // (masked) residual and masks; valid frames are unchanged (the reference's unmasked residual only reaches
    // padded frames, which LN2's mask zeroes), and no conv needs a mask prologue
    if (std::is_same<E, float>::value && split && f32vc && l.s1_off) {
      // split-bf16 ("fp32x3"): LN1 stores A (fp32, conv 2's residual) and its 6-plane split A6; conv 1 stores the
      // hidden as its 6-plane split H6; conv 2 sums its six bf16 products per fp32 product in fp32 (mt_vconv.h f32 2)
      bf16* A6 = (bf16*)(trash + 4096);
      bf16* H6 = (bf16*)((char*)A6 + align256(n * 6 * W * 2));
      if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n1_off), eps, xmask, 0, (E*)A, st, A6))) return rc;
      auto sargs = [&](const GemmW& g, size_t s_off, const void* x, void* y) {
        VConvArgs a{};
        a.f32 = 2;
        a.x = (const bf16*)x;
        a.B = B;
        a.L = Tx;
        a.cin = 6 * g.cin;
        a.w = (const bf16*)(P + s_off);
        a.bias = (const float*)(P + g.b_off);
        a.M = a.Mpad = g.cout;
        a.taps = g.k;
        a.dil = 1;
        a.pad = g.pad;
        a.y = (bf16*)y;
        a.emask = xmask;
        a.div = 1.f;
        a.zero = (const bf16*)(P + ezero_off);
        a.trash = (bf16*)trash;
        a.probe = -1;
        return a;
      };
      if ((rc = launch_vconv(VE_RELU | VE_MASK | VE_SPLIT6, sargs(l.f1, l.s1_off, A6, H6), st))) return rc;
      VConvArgs f2 = sargs(l.f2, l.s2_off, H6, Bb);
      f2.resid = (const bf16*)A;
      if ((rc = launch_vconv(VE_RESID | VE_MASK, f2, st))) return rc;
      if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n2_off), eps, xmask, 0, (E*)X, st))) return rc;
      continue;
    }
    if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n1_off), eps, xmask, 0, (E*)A, st))) return rc;
    if ((rc = v32(l.f1, A, Hh, VE_RELU | VE_MASK, nullptr)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs f1 = gemm_args(l.f1, P, B, Tx);
      f1.x0 = A;
      f1.y = Hh;
      f1.emask = xmask;
      if ((rc = launch_conv<E, 0, EF_RELU | EF_MASK>(f1, st))) return rc;
    }
    // (v + A) * m on vconv, v * m + A generic: equal, A being masked
    if ((rc = v32(l.f2, Hh, Bb, VE_RESID | VE_MASK, A)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs f2 = gemm_args(l.f2, P, B, Tx);
      f2.x0 = Hh;
      f2.y = Bb;
      f2.emask = xmask;
      f2.resid = A;
      f2.ldr = W;
      if ((rc = launch_conv<E, 0, EF_MASK | EF_RESID>(f2, st))) return rc;
    }
    // LN2, then the next layer's (or the final) x * x_mask
    if ((rc = rowln<E>((const E*)Bb, (int)n, W, (const float*)(P + l.n2_off), eps, xmask, 0, (E*)X, st))) return rc;
  }
  // mu = proj_m(x) * m -> [B][80][Tx] fp32
  {
    ConvArgs a = gemm_args(proj_m, P, B, Tx);
    a.x0 = X;
    a.y = MU;
    a.emask = xmask;
    if ((rc = launch_conv<E, 0, EF_MASK>(a, st))) return rc;
    if ((rc = btc_to_bct(dtype, MU, 80, 0, B, 80, Tx, mu, st))) return rc;
  }
  // duration predictor on x (model.py:217-229: conv -> relu -> LN, twice, then proj(h*m)*m)
  {
    // every conv input stored masked (X is x*m; the LayerNorms store LN(.)*m), so no mask prologue
    if ((rc = v32(dp1, X, Hh, VE_RELU, nullptr)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs a = gemm_args(dp1, P, B, Tx);
      a.x0 = X;
      a.y = Hh;
      if ((rc = launch_conv<E, 0, EF_RELU>(a, st))) return rc;
    }
    if ((rc = rowln<E>((const E*)Hh, (int)n, DF, (const float*)(P + dn1_off), eps, xmask, 0, (E*)A, st))) return rc;
    if ((rc = v32(dp2, A, Hh, VE_RELU, nullptr)) != kNotVc && rc) return rc;
    if (rc == kNotVc) {
      ConvArgs b = gemm_args(dp2, P, B, Tx);
      b.x0 = A;
      b.y = Hh;
      if ((rc = launch_conv<E, 0, EF_RELU>(b, st))) return rc;
    }
    if ((rc = rowln<E>((const E*)Hh, (int)n, DF, (const float*)(P + dn2_off), eps, xmask, 0, (E*)A, st))) return rc;
    ConvArgs c = gemm_args(dpp, P, B, Tx);
    c.x0 = A;
    c.y = logw;
    c.ldy = 1;
    c.emask = xmask;
    if ((rc = launch_conv<E, 0, EF_MASK | EF_OUTF32>(c, st))) return rc;
  }
  return 0;
}

int Encoder::forward(const void* packed, const long long* ids, const long long* xlen, const float* spks, int B, int Tx,
                     float* mu, float* logw, float* xmask, int* oov, void* ws, size_t ws_bytes, hipStream_t st) const {
  MT_REQUIRE(B > 0 && Tx > 0 && ids && xlen && mu && logw && xmask, "encoder: empty input");
  MT_REQUIRE(W == C || spks, "encoder: multi-speaker model needs spks [B][%d]", spk_dim);
  MT_REQUIRE(ws_bytes >= workspace_bytes(B, Tx), "encoder: workspace %zu < %zu", ws_bytes, workspace_bytes(B, Tx));
  if (dtype == BF16)
    return forward_t<bf16>((const char*)packed, ids, xlen, spks, B, Tx, mu, logw, xmask, oov, (char*)ws, st);
  return forward_t<float>((const char*)packed, ids, xlen, spks, B, Tx, mu, logw, xmask, oov, (char*)ws, st);
}

}  // namespace mt
