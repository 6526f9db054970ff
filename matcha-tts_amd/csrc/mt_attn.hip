// Decoder self-attention core (model.py:686-701) for gfx950.
//
// qkv [B][T][3*inner] (q | k | v, head h at columns h*64..h*64+63 of each part),
// mask [B][T] (frame mask at this U-Net level), out [B][T][inner].
// Workgroup = 4 waves = 64 queries of one (utterance, head); flash-style online softmax
// over 64-key tiles, S = Q.K^T and O += P.V on MFMA (bf16: 16x16x32, f32: 16x16x4).
//
// Reference mask semantics, kept exactly: masked keys are filled with
// -torch.finfo(fp32).min = +3.4e38 (model.py:697), so for an utterance whose mask has ANY
// zero at this level every query attends uniformly to the masked keys:
//     out = sum_{j masked} (1/n_masked) * v_j          (independent of q and k)
// and for an utterance without padding the ordinary softmax over all keys applies.
#include "mt_common.h"

#include <type_traits>

namespace mt {

template <class E>
__global__ __launch_bounds__(256) void attn_kernel(const E* __restrict__ qkv,
                                                   const float* __restrict__ mask,
                                                   E* __restrict__ out, int T, int inner) {
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
  const int b = blockIdx.z, h = blockIdx.y, q0 = blockIdx.x * 64;
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
    // exact count of masked keys
    int* cnt = reinterpret_cast<int*>(red);
    if (tid == 0) cnt[0] = 0;
    __syncthreads();
    if (npad_local) atomicAdd(cnt, npad_local);
    __syncthreads();
    const int n = cnt[0];
    __syncthreads();
    const float p = 1.f / (float)n;
    // thread (kg, d): partial sum over keys j = kg (mod 4)
    const int kg = tid >> 6, d = tid & 63;
    float s = 0.f;
    for (int j = kg; j < T; j += 4)
      if (mk[j] == 0.f) s += p * to_f(V[(size_t)j * ld + d]);
    red[kg * 64 + d] = s;
    __syncthreads();
    if (tid < 64) red[tid] = ((red[tid] + red[64 + tid]) + red[128 + tid]) + red[192 + tid];
    __syncthreads();
    for (int i = tid; i < 64 * 64; i += 256) {
      const int q = q0 + (i >> 6), dd = i & 63;
      if (q < T) O[(size_t)q * inner + dd] = from_f<E>(red[dd]);
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
  const int nkt = (T + 63) / 64;
  for (int kt = 0; kt < nkt; ++kt) {
    const int k0 = kt * 64;
    // stage K rows and V^T
    for (int v = tid; v < 64 * (64 / VN); v += 256) {
      const int r = v / (64 / VN), s = v % (64 / VN);
      const int key = k0 + r;
      Vec16<E> kv = zero16<E>(), vv = zero16<E>();
      if (key < T) {
        kv = load16(K + (size_t)key * ld + s * VN);
        vv = load16(V + (size_t)key * ld + s * VN);
      }
      store16(reinterpret_cast<E*>(Ks + r * ROW + s * 16), kv);
#pragma unroll
      for (int i = 0; i < VN; ++i)
        reinterpret_cast<E*>(Vt + (s * VN + i) * ROW)[r] = from_f<E>(vv.get(i));
    }
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
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int q = q0 + wave * 16 + 4 * (lane >> 4) + r;
    if (q >= T) continue;
    const float inv = 1.f / l_run[r];
#pragma unroll
    for (int df = 0; df < 4; ++df) O[(size_t)q * inner + df * 16 + (lane & 15)] = from_f<E>(o[df][r] * inv);
  }
}

int launch_attention(int dtype, const void* qkv, const float* mask, void* out, int B, int T,
                     int heads, hipStream_t stream) {
  MT_REQUIRE(B > 0 && T > 0 && heads > 0, "attention: empty geometry");
  const int inner = heads * 64;
  const int esz = dtype == BF16 ? 2 : 4;
  const size_t row = 64 * esz + 16;
  const size_t lds = 3 * 64 * row + 4 * 64 * sizeof(float);
  dim3 grid((unsigned)((T + 63) / 64), (unsigned)heads, (unsigned)B);
  if (dtype == BF16)
    hipLaunchKernelGGL(attn_kernel<bf16>, grid, dim3(256), lds, stream, (const bf16*)qkv, mask,
                       (bf16*)out, T, inner);
  else
    hipLaunchKernelGGL(attn_kernel<float>, grid, dim3(256), lds, stream, (const float*)qkv, mask,
                       (float*)out, T, inner);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
