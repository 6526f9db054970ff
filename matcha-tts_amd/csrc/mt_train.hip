// Training-step kernels (§8f rank 3): the CFM training step of train_standalone.py:623-707 (encoder +
// duration predictor, MAS, duration / prior / flow-matching losses, estimator forward AND backward,
// Adam) in fp32 on gfx950. Activations are [rows][C] (frame-major, channel-contiguous, as everywhere in
// this library); every op of the model is expressed with the primitives below, forward and backward:
//
//   gemm        batched strided C = alpha op(A) op(B) + beta C on exact-fp32 MFMA (v_mfma_f32_16x16x4_f32),
//               64 x 64 tiles, K staged through LDS in chunks of 16: Linear / 1x1 conv forward, dgrad, wgrad;
//               conv1d = im2col + gemm (wgrad: gemm over the columns; dgrad: gemm then col2im);
//               attention S = QK^T, O = PV and their gradients; the MAS log-prior
//   im2col / col2im   [B][T][C] <-> [B*Tout][k*C] columns with stride, padding, dilation (col2im gathers, so
//               the gradient sum is deterministic)
//   ew          elementwise with broadcasting (add / mul / masks / biases / activations and their gradients)
//   colsum      segmented column sums (bias / gamma / beta / time-bias / SnakeBeta parameter gradients)
//   groupnorm, layernorm  forward (saving mean / rstd) and backward
//   softmax     row softmax with the reference's mask modes (decoder: masked keys := +3.4e38, model.py:697;
//               encoder: masked scores := -1e4, model.py:353) and its backward
//   rope        rotary embedding and its inverse (model.py:244-292)
//   embed       embedding gather and its deterministic per-row gradient
//   adam        torch.optim.Adam (defaults) with the global-norm clip factor folded in (Lightning
//               gradient_clip_val = 5.0, train_standalone.py:869)
// No reduction here uses atomics: every sum runs in a fixed order, so a step is bitwise reproducible.
#include <math.h>

#include <algorithm>

#include "mt_train.h"

namespace mt {

// ------------------------------------------------------------------------------------------------ gemm
// 128 x 128 block tile, K staged through LDS 32 at a time (k-major: As[k][m], Bs[k][n]), 4 waves of 64 x 64,
// each 2 x 2 v_mfma_f32_32x32x2_f32 accumulators (exact fp32: a k-ordered fma chain per output). The next
// K chunk's global loads (16-byte along the operand's contiguous dimension when aligned) are issued before
// the current chunk's MFMAs. Split-K (small M x N, long K: the weight gradients, K = frames) writes per-slice
// partials that a second kernel sums in slice order — deterministic, no atomics.
namespace {
constexpr int GBM = 128, GBK = 32, GLD = GBM + 4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

// v[j] = src[row][col + j] for the 4-wide group (0 outside [0, nrow) x [0, ncol))
__device__ __forceinline__ f32x4 ld4(const float* __restrict__ base, int ld, int row, int col, int nrow, int ncol,
                                     bool vec) {
  f32x4 v = {0.f, 0.f, 0.f, 0.f};
  if (row >= nrow) return v;
  const float* p = base + (size_t)row * ld + col;
  if (vec && col + 3 < ncol) return *reinterpret_cast<const f32x4*>(p);
#pragma unroll
  for (int j = 0; j < 4; ++j)
    if (col + j < ncol) v[j] = p[j];
  return v;
}
}  // namespace

// op(A) tile (128 m x 32 k) / op(B) tile (32 k x 128 n): 1024 groups of 4, 4 per thread
template <int TA>
__device__ __forceinline__ void gemm_load_a(const GemmF32& g, const float* A, int m0, int kb, int kend, bool vec,
                                            f32x4 (&r)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (TA) r[i] = ld4(A, g.lda, kb + (e >> 5), m0 + (e & 31) * 4, kend, g.M, vec);  // stored [K][M]
    else r[i] = ld4(A, g.lda, m0 + (e >> 3), kb + (e & 7) * 4, g.M, kend, vec);      // stored [M][K]
  }
}
template <int TA>
__device__ __forceinline__ void gemm_store_a(float (*As)[GLD], const f32x4 (&r)[4]) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int e = threadIdx.x + 256 * i;
    if (TA) {
      *reinterpret_cast<f32x4*>(&As[e >> 5][(e & 31) * 4]) = r[i];
    } else {
#pragma unroll
      for (int j = 0; j < 4; ++j) As[(e & 7) * 4 + j][e >> 3] = r[i][j];
    }
  }
}

template <int TA, int TB>
__global__ __launch_bounds__(256) void gemm_f32_kernel(GemmF32 g, int kchunk, int split, bool va, bool vb) {
  __shared__ float As[GBK][GLD], Bs[GBK][GLD];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBM, z = blockIdx.z;
  const float* A = g.A + (split ? 0 : (size_t)z * g.sA);
  const float* B = g.B + (split ? 0 : (size_t)z * g.sB);
  float* Cm = g.C + (size_t)z * g.sC;
  const int kbeg = split ? z * kchunk : 0, kend = split ? min(g.K, kbeg + kchunk) : g.K;
  // B is loaded as op(B)^T's A-shaped case: TB == 1 means stored [N][K] (contiguous k) like TA == 0
  GemmF32 gb = g;
  gb.M = g.N;
  gb.lda = g.ldb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f32x4 ra[4], rb[4];
  gemm_load_a<TA>(g, A, m0, kbeg, kend, va, ra);
  gemm_load_a<1 - TB>(gb, B, n0, kbeg, kend, vb, rb);
  for (int kb = kbeg; kb < kend; kb += GBK) {
    gemm_store_a<TA>(As, ra);
    gemm_store_a<1 - TB>(Bs, rb);
    __syncthreads();
    if (kb + GBK < kend) {
      gemm_load_a<TA>(g, A, m0, kb + GBK, kend, va, ra);
      gemm_load_a<1 - TB>(gb, B, n0, kb + GBK, kend, vb, rb);
    }
#pragma unroll
    for (int kk = 0; kk < GBK; kk += 2) {
      const int kr = kk + (lane >> 5);
      float a[2], b[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        a[f] = As[kr][wm * 64 + f * 32 + (lane & 31)];
        b[f] = Bs[kr][wn * 64 + f * 32 + (lane & 31)];
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
          acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
    }
    __syncthreads();
  }
  // D of a 32 x 32 fragment: column lane & 31, row (r & 3) + 8 (r >> 2) + 4 (lane >> 5)
  const float alpha = split ? 1.f : g.alpha, beta = split ? 0.f : g.beta;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 64 + fm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int gn = n0 + wn * 64 + fn * 32 + (lane & 31);
        if (gm >= g.M || gn >= g.N) continue;
        float* c = Cm + (size_t)gm * (split ? g.N : g.ldc) + gn;
        float v = alpha * acc[fm][fn][r];
        if (beta != 0.f) v += beta * *c;
        if (!split && g.bias) v += g.bias[gn];
        if (!split && g.rmask) v *= g.rmask[(size_t)z * g.M + gm];
        *c = v;
      }
}

// Mixed-precision GEMM (the "16-mixed" / "bf16-mixed" training modes): the same 128 x 128 tile, register-staged
// fp32 loads and epilogue as gemm_f32_kernel, but the operands are rounded (RNE) to fp16 (FMT 1) or bf16 (FMT 2)
// when they are written to LDS, and the K loop runs v_mfma_f32_32x32x16_{f16,bf16} with fp32 accumulation —
// autocast's matmul arithmetic (16-bit operands, fp32 sums). LDS holds op(A) as [m][k] and op(B) as [n][k] with
// k contiguous (40-element rows: 80 B, so the 8 lanes of a ds_read_b128 phase hit distinct banks), which is
// each lane's operand fragment (row l & 31, k = 8 (l >> 5) + j) as one 16-byte read.
namespace {
constexpr int GKH = GBK + 8;
template <int FMT> struct Half;
template <> struct Half<1> { typedef _Float16 T; };
template <> struct Half<2> { typedef __bf16 T; };

// op(A) tile (128 rows x 32 k) for the 16-bit kernel. Stored [M][K]: gemm_load_a's groups. Stored [K][M] (TA): thread
// t loads k rows 4 (t >> 5) .. + 3 of row group t & 31 (each k row's 128 floats still one contiguous 512-byte run per
// 32 lanes), so every one of its 4 rows gets 4 consecutive k — one 8-byte LDS store per row instead of four 2-byte ones
template <int TA>
__device__ __forceinline__ void gemm_load_h(const GemmF32& g, const float* A, int m0, int kb, int kend, bool vec,
                                            f32x4 (&r)[4]) {
  if constexpr (TA) {
    const int q = threadIdx.x >> 5, mg = threadIdx.x & 31;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = ld4(A, g.lda, kb + 4 * q + i, m0 + mg * 4, kend, g.M, vec);
  } else {
    gemm_load_a<0>(g, A, m0, kb, kend, vec, r);
  }
}

// the tile of gemm_load_h into LDS as [row][k] in 16-bit
template <int TA, typename H>
__device__ __forceinline__ void gemm_store_h(H (*As)[GKH], const f32x4 (&r)[4]) {
  typedef H h4 __attribute__((ext_vector_type(4)));
  if constexpr (TA) {  // r[i][j]: k = 4q + i of row 4 mg + j
    const int q = threadIdx.x >> 5, mg = threadIdx.x & 31;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      h4 v;
#pragma unroll
      for (int i = 0; i < 4; ++i) v[i] = (H)r[i][j];
      *reinterpret_cast<h4*>(&As[mg * 4 + j][4 * q]) = v;
    }
  } else {  // 4 consecutive k of one row
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int e = threadIdx.x + 256 * i;
      h4 v;
#pragma unroll
      for (int j = 0; j < 4; ++j) v[j] = (H)r[i][j];
      *reinterpret_cast<h4*>(&As[e >> 3][(e & 7) * 4]) = v;
    }
  }
}
}  // namespace

template <int TA, int TB, int FMT>
__global__ __launch_bounds__(256) void gemm_h_kernel(GemmF32 g, int kchunk, int split, bool va, bool vb) {
  typedef typename Half<FMT>::T H;
  typedef H h8 __attribute__((ext_vector_type(8)));
  __shared__ __attribute__((aligned(16))) H As[GBM][GKH];
  __shared__ __attribute__((aligned(16))) H Bs[GBM][GKH];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.y * GBM, n0 = blockIdx.x * GBM, z = blockIdx.z;
  const float* A = g.A + (split ? 0 : (size_t)z * g.sA);
  const float* B = g.B + (split ? 0 : (size_t)z * g.sB);
  float* Cm = g.C + (size_t)z * g.sC;
  const int kbeg = split ? z * kchunk : 0, kend = split ? min(g.K, kbeg + kchunk) : g.K;
  GemmF32 gb = g;
  gb.M = g.N;
  gb.lda = g.ldb;
  f32x16 acc[2][2];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;
  f32x4 ra[4], rb[4];
  gemm_load_h<TA>(g, A, m0, kbeg, kend, va, ra);
  gemm_load_h<1 - TB>(gb, B, n0, kbeg, kend, vb, rb);
  const int fr = lane & 31, fk = 8 * (lane >> 5);
  for (int kb = kbeg; kb < kend; kb += GBK) {
    gemm_store_h<TA>(As, ra);
    gemm_store_h<1 - TB>(Bs, rb);
    __syncthreads();
    if (kb + GBK < kend) {
      gemm_load_h<TA>(g, A, m0, kb + GBK, kend, va, ra);
      gemm_load_h<1 - TB>(gb, B, n0, kb + GBK, kend, vb, rb);
    }
#pragma unroll
    for (int s = 0; s < GBK; s += 16) {
      h8 a[2], b[2];
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        a[f] = *reinterpret_cast<const h8*>(&As[wm * 64 + f * 32 + fr][s + fk]);
        b[f] = *reinterpret_cast<const h8*>(&Bs[wn * 64 + f * 32 + fr][s + fk]);
      }
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) {
          if constexpr (FMT == 1)
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_f16(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
          else
            acc[fm][fn] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a[fm], b[fn], acc[fm][fn], 0, 0, 0);
        }
    }
    __syncthreads();
  }
  const float alpha = split ? 1.f : g.alpha, beta = split ? 0.f : g.beta;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int gm = m0 + wm * 64 + fm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        const int gn = n0 + wn * 64 + fn * 32 + (lane & 31);
        if (gm >= g.M || gn >= g.N) continue;
        float* c = Cm + (size_t)gm * (split ? g.N : g.ldc) + gn;
        float v = alpha * acc[fm][fn][r];
        if (beta != 0.f) v += beta * *c;
        if (!split && g.bias) v += g.bias[gn];
        if (!split && g.rmask) v *= g.rmask[(size_t)z * g.M + gm];
        *c = v;
      }
}

// C = alpha * sum_z P[z] + beta * C, slices in order
__global__ void splitk_reduce_kernel(const float* __restrict__ P, int S, int M, int N, float alpha, float beta,
                                     const float* __restrict__ bias, const float* __restrict__ rmask,
                                     float* __restrict__ C, int ldc) {
  const size_t mn = (size_t)M * N;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < mn; i += (size_t)gridDim.x * blockDim.x) {
    float s = 0.f;
    for (int z = 0; z < S; ++z) s += P[z * mn + i];
    float* c = C + (i / N) * ldc + i % N;
    float v = alpha * s;
    if (beta != 0.f) v += beta * *c;
    if (bias) v += bias[i % N];
    if (rmask) v *= rmask[i / N];
    *c = v;
  }
}

namespace {
bool vec_ok(const float* p, int ld, long long stride, int batch) {
  return ((uintptr_t)p & 15) == 0 && ld % 4 == 0 && (batch == 1 || stride % 4 == 0);
}
// split-K plan: slices of kchunk (a multiple of GBK) when a single GEMM has few output tiles and a long K
int splitk_plan(int M, int N, int K, int batch, int* kchunk) {
  const int tiles = ((N + GBM - 1) / GBM) * ((M + GBM - 1) / GBM);
  *kchunk = K;
  if (batch != 1 || tiles >= 128 || K < 2048) return 1;
  const int want = std::min((K + 511) / 512, (256 + tiles - 1) / tiles);
  *kchunk = ((K + want - 1) / want + GBK - 1) / GBK * GBK;
  const int S = (K + *kchunk - 1) / *kchunk;
  if (S <= 1) *kchunk = K;
  return S;
}
}  // namespace

size_t gemm_f32_workspace_floats(int M, int N, int K, int batch) {
  int kc;
  const int S = splitk_plan(M, N, K, batch, &kc);
  return S > 1 ? (size_t)S * M * N : 0;
}

static dim3 ew_grid(size_t n);

int gemm_f32(const GemmF32& g, hipStream_t st) {
  MT_REQUIRE(g.M > 0 && g.N > 0 && g.K > 0 && g.batch > 0 && g.A && g.B && g.C, "gemm: shape / null");
  const int gx = (g.N + GBM - 1) / GBM, gy = (g.M + GBM - 1) / GBM;
  MT_REQUIRE(gy <= 65535 && g.batch <= 65535, "gemm: grid too large");
  const bool va = vec_ok(g.A, g.lda, g.sA, g.batch), vb = vec_ok(g.B, g.ldb, g.sB, g.batch);
  int split = 0, kchunk = g.K, S = g.batch;
  GemmF32 k = g;
  if (g.batch == 1) {
    const int s = splitk_plan(g.M, g.N, g.K, 1, &kchunk);
    if (s > 1 && g.ws && g.ws_floats >= (size_t)s * g.M * g.N) {  // without the workspace: one unsplit pass
      split = 1;
      S = s;
      k.C = g.ws;
      k.sC = (long long)g.M * g.N;
    } else {
      kchunk = g.K;
    }
  }
  dim3 grid(gx, gy, S);
  MT_REQUIRE(g.opfmt >= 0 && g.opfmt <= 2, "gemm: operand format (0 fp32, 1 fp16, 2 bf16)");
  auto kern = g.transA ? (g.transB ? gemm_f32_kernel<1, 1> : gemm_f32_kernel<1, 0>)
                       : (g.transB ? gemm_f32_kernel<0, 1> : gemm_f32_kernel<0, 0>);
  if (g.opfmt == 1)
    kern = g.transA ? (g.transB ? gemm_h_kernel<1, 1, 1> : gemm_h_kernel<1, 0, 1>)
                    : (g.transB ? gemm_h_kernel<0, 1, 1> : gemm_h_kernel<0, 0, 1>);
  else if (g.opfmt == 2)
    kern = g.transA ? (g.transB ? gemm_h_kernel<1, 1, 2> : gemm_h_kernel<1, 0, 2>)
                    : (g.transB ? gemm_h_kernel<0, 1, 2> : gemm_h_kernel<0, 0, 2>);
  hipLaunchKernelGGL(kern, grid, dim3(256), 0, st, k, kchunk, split, va, vb);
  if (split)
    hipLaunchKernelGGL(splitk_reduce_kernel, ew_grid((size_t)g.M * g.N), dim3(256), 0, st, (const float*)g.ws,
                       S, g.M, g.N, g.alpha, g.beta, g.bias, g.rmask, g.C, g.ldc);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// -------------------------------------------------------------------------------------- im2col / col2im
// cols[(b*Tout + o)][c*k + tap] = x[b][o*stride - pad + tap*dil][c] (0 outside [0, T)): channel-major, tap
// fastest, so a torch Conv1d weight [Cout][Cin][k] is the GEMM operand [Cout][Cin*k] as it lies in memory
// (and a ConvTranspose1d weight [Cin][Cout][k] that of its adjoint conv)
__global__ void im2col_kernel(const float* __restrict__ x, const float* __restrict__ mask, int B, int T, int C, int k,
                              int stride, int pad, int dil, int Tout, float* __restrict__ cols) {
  const size_t total = (size_t)B * Tout * C * k;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int tap = (int)(i % k);
    size_t r = i / k;
    const int c = (int)(r % C);
    r /= C;
    const int o = (int)(r % Tout);
    const int b = (int)(r / Tout);
    const int t = o * stride - pad + tap * dil;
    float v = 0.f;
    if (t >= 0 && t < T) {
      v = x[((size_t)b * T + t) * C + c];
      if (mask) v *= mask[(size_t)b * T + t];
    }
    cols[i] = v;
  }
}

// dx[b][t][c] (+)= mask[b][t] * sum over (o, tap) with o*stride - pad + tap*dil == t of dcols[(b*Tout + o)][c*k + tap]
__global__ void col2im_kernel(const float* __restrict__ dcols, const float* __restrict__ mask, int B, int T, int C,
                              int k, int stride, int pad, int dil, int Tout, float* __restrict__ dx, int accumulate) {
  const size_t total = (size_t)B * T * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const int t = (int)((i / C) % T);
    const int b = (int)(i / ((size_t)C * T));
    float s = 0.f;
    for (int tap = 0; tap < k; ++tap) {
      const int num = t + pad - tap * dil;
      if (num < 0 || num % stride) continue;
      const int o = num / stride;
      if (o >= Tout) continue;
      s += dcols[((size_t)b * Tout + o) * C * k + (size_t)c * k + tap];
    }
    if (mask) s *= mask[(size_t)b * T + t];
    dx[i] = accumulate ? dx[i] + s : s;
  }
}

static dim3 ew_grid(size_t n) { return dim3((unsigned)std::min<size_t>((n + 255) / 256, 65535u * 4)); }

int im2col(const float* x, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
           float* cols, hipStream_t st) {
  MT_REQUIRE(x && cols && B > 0 && T > 0 && C > 0 && k > 0 && stride > 0 && dil > 0 && Tout > 0, "im2col: args");
  hipLaunchKernelGGL(im2col_kernel, ew_grid((size_t)B * Tout * k * C), dim3(256), 0, st, x, mask, B, T, C, k, stride,
                     pad, dil, Tout, cols);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int col2im(const float* dcols, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
           float* dx, int accumulate, hipStream_t st) {
  MT_REQUIRE(dcols && dx && B > 0 && T > 0 && C > 0 && k > 0 && stride > 0 && dil > 0 && Tout > 0, "col2im: args");
  hipLaunchKernelGGL(col2im_kernel, ew_grid((size_t)B * T * C), dim3(256), 0, st, dcols, mask, B, T, C, k, stride, pad,
                     dil, Tout, dx, accumulate);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------ elementwise
__device__ __forceinline__ size_t bidx(size_t i, const EwArgs& e) {
  return ((i / e.d0) % e.m0) * e.s0 + ((i / e.d1) % e.m1) * e.s1;
}
__device__ __forceinline__ float softplus_f(float x) { return x > 20.f ? x : log1pf(expf(x)); }

__global__ void ew_kernel(EwArgs e) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < e.n; i += (size_t)gridDim.x * blockDim.x) {
    const float a = e.a ? e.a[i] : 0.f;
    const float b = e.b ? e.b[bidx(i, e)] : 0.f;
    float o;
    switch (e.op) {
      case EW_AXPBY: o = e.alpha * a + e.beta * b; break;
      case EW_MUL: o = e.alpha * a * b; break;
      case EW_MISH: {
        const float sp = softplus_f(a);
        o = a * tanhf(sp);
        break;
      }
      case EW_MISH_BWD: {  // a = x, b = dy (same index space, s0 = 1)
        const float sp = softplus_f(a), th = tanhf(sp);
        const float sg = 1.f / (1.f + expf(-a));
        o = e.c[i] * (th + a * (1.f - th * th) * sg);
        break;
      }
      case EW_SILU: o = a / (1.f + expf(-a)); break;
      case EW_SILU_BWD: {
        const float sg = 1.f / (1.f + expf(-a));
        o = e.c[i] * (sg * (1.f + a * (1.f - sg)));
        break;
      }
      case EW_RELU: o = a > 0.f ? a : 0.f; break;
      case EW_RELU_BWD: o = a > 0.f ? e.c[i] : 0.f; break;
      case EW_EXP: o = expf(a); break;
      case EW_SQDIFF: o = (a - b) * (a - b); break;
      case EW_SIN: o = sinf(a); break;
      case EW_COS: o = cosf(a); break;
      case EW_LOG: o = logf(e.alpha + a); break;
      case EW_RECIP: o = e.alpha / a; break;
      default: o = 0.f;
    }
    if (e.accumulate) o += e.out[i];
    e.out[i] = o;
  }
}

int ew(const EwArgs& e, hipStream_t st) {
  MT_REQUIRE(e.out && e.n > 0 && e.d0 > 0 && e.d1 > 0 && e.m0 > 0 && e.m1 > 0, "ew: args");
  MT_REQUIRE(!(e.op == EW_MISH_BWD || e.op == EW_SILU_BWD || e.op == EW_RELU_BWD) || e.c, "ew: grad input");
  hipLaunchKernelGGL(ew_kernel, ew_grid(e.n), dim3(256), 0, st, e);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// dst[r][doff + j] (+)= src[r][soff + j] for r < rows, j < n: channel concat / split of [rows][C] activations
__global__ void copy_cols_kernel(const float* __restrict__ src, int lds, int soff, float* __restrict__ dst, int ldd,
                                 int doff, int rows, int n, int accumulate) {
  const size_t total = (size_t)rows * n;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / n;
    const int j = (int)(i % n);
    const float v = src[r * lds + soff + j];
    float* o = dst + r * ldd + doff + j;
    *o = accumulate ? *o + v : v;
  }
}

int copy_cols(const float* src, int lds, int soff, float* dst, int ldd, int doff, int rows, int n, int accumulate,
              hipStream_t st) {
  MT_REQUIRE(src && dst && rows > 0 && n > 0 && soff + n <= lds && doff + n <= ldd, "copy_cols: args");
  hipLaunchKernelGGL(copy_cols_kernel, ew_grid((size_t)rows * n), dim3(256), 0, st, src, lds, soff, dst, ldd, doff,
                     rows, n, accumulate);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// sequence_mask (model.py:42-46): out[b][t] = t < lengths[b]
__global__ void seq_mask_kernel(const long long* __restrict__ len, int B, int T, float* __restrict__ out) {
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < B * T; i += gridDim.x * blockDim.x)
    out[i] = (long long)(i % T) < len[i / T] ? 1.f : 0.f;
}

int seq_mask(const long long* lengths, int B, int T, float* out, hipStream_t st) {
  MT_REQUIRE(lengths && out && B > 0 && T > 0, "seq_mask: args");
  hipLaunchKernelGGL(seq_mask_kernel, ew_grid((size_t)B * T), dim3(256), 0, st, lengths, B, T, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------- column sums
// out[s][c] (+)= sum_{r in segment s} a[r][c] * (b ? b[r][c] : 1), segments of `seg` rows. Two fixed-order levels,
// no atomics: partials over blocks of CS_ROWS rows (a 256-thread block = 64 columns x 4 row lanes, lanes combined
// in lane order), then each segment's partials (4 threads per column over interleaved partials, combined in order).
constexpr int CS_ROWS = 512;
__global__ __launch_bounds__(256) void colsum_part_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                          int rows, int C, int seg, int nsub, float* __restrict__ part) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, lr = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, sb = blockIdx.y;
  const int s = sb / nsub, k = sb % nsub;
  const int r0 = s * seg + k * CS_ROWS, r1 = min(min(rows, (s + 1) * seg), r0 + CS_ROWS);
  float acc = 0.f;
  if (c < C)
    for (int r = r0 + lr; r < r1; r += 4) {
      const size_t o = (size_t)r * C + c;
      acc += b ? a[o] * b[o] : a[o];
    }
  red[lr][cl] = acc;
  __syncthreads();
  if (lr == 0 && c < C) part[(size_t)sb * C + c] = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
}

__global__ __launch_bounds__(256) void colsum_merge_kernel(const float* __restrict__ part, int C, int nsub,
                                                           float* __restrict__ out, int accumulate) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, lr = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, s = blockIdx.y;
  float acc = 0.f;
  if (c < C)
    for (int k = lr; k < nsub; k += 4) acc += part[((size_t)s * nsub + k) * C + c];
  red[lr][cl] = acc;
  __syncthreads();
  if (lr == 0 && c < C) {
    float* o = out + (size_t)s * C + c;
    const float v = ((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl];
    *o = accumulate ? *o + v : v;
  }
}

size_t colsum_scratch_floats(int rows, int C, int seg) {
  const int nseg = (rows + seg - 1) / seg, nsub = (seg + CS_ROWS - 1) / CS_ROWS;
  return (size_t)nseg * nsub * C;
}

int colsum(const float* a, const float* b, int rows, int C, int seg, float* out, int accumulate, float* scratch,
           hipStream_t st) {
  MT_REQUIRE(a && out && scratch && rows > 0 && C > 0 && seg > 0, "colsum: args");
  const int nseg = (rows + seg - 1) / seg, nsub = (seg + CS_ROWS - 1) / CS_ROWS;
  MT_REQUIRE((size_t)nseg * nsub <= 65535u * 64, "colsum: too many partial blocks");
  hipLaunchKernelGGL(colsum_part_kernel, dim3((C + 63) / 64, nseg * nsub), dim3(256), 0, st, a, b, rows, C, seg,
                     nsub, scratch);
  hipLaunchKernelGGL(colsum_merge_kernel, dim3((C + 63) / 64, nseg), dim3(256), 0, st, (const float*)scratch, C,
                     nsub, out, accumulate);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// full sum of a (or of a*b) -> out[0], two levels in a fixed order
__global__ __launch_bounds__(256) void sum_kernel(const float* __restrict__ a, const float* __restrict__ b, size_t n,
                                                  float* __restrict__ partial) {
  __shared__ float red[256];
  float s = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) s += b ? a[i] * b[i] : a[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

int sum_all(const float* a, const float* b, size_t n, float* out, float* scratch, hipStream_t st) {
  MT_REQUIRE(a && out && scratch && n > 0, "sum: args");
  const int nb = (int)std::min<size_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(sum_kernel, dim3(nb), dim3(256), 0, st, a, b, n, scratch);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, (const float*)scratch, (const float*)nullptr, (size_t)nb,
                     out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// GradScaler.unscale_ (torch._amp_foreach_non_finite_check_and_unscale_): g *= inv_scale in place with a
// per-element found-inf check on the unscaled value; partial[block] = the block's count of non-finite elements
__global__ __launch_bounds__(256) void unscale_kernel(float* __restrict__ g, size_t n, float inv_scale,
                                                      float* __restrict__ partial) {
  __shared__ float red[256];
  float bad = 0.f;
  for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) {
    const float x = g[i];  // checked as stored, before the multiply (torch._amp_foreach_non_finite_check_and_unscale_)
    bad += isfinite(x) ? 0.f : 1.f;
    g[i] = x * inv_scale;
  }
  red[threadIdx.x] = bad;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

int unscale_found_inf(float* g, size_t n, float inv_scale, float* found, float* scratch, hipStream_t st) {
  MT_REQUIRE(g && found && scratch && n > 0, "unscale: args");
  const int nb = (int)std::min<size_t>(1024, (n + 255) / 256);
  hipLaunchKernelGGL(unscale_kernel, dim3(nb), dim3(256), 0, st, g, n, inv_scale, scratch);
  hipLaunchKernelGGL(sum_kernel, dim3(1), dim3(256), 0, st, (const float*)scratch, (const float*)nullptr, (size_t)nb,
                     found);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------------- dropout
// out = a * keep / (1 - p), keep = hash(seed, i) >= p (counter-based, so a step's masks are a function of its
// seed: reproducible, and the backward re-derives the same mask instead of storing it)
__device__ __forceinline__ float uhash(uint32_t seed, size_t i) {
  uint32_t h = seed * 0x9E3779B9u ^ (uint32_t)i ^ ((uint32_t)(i >> 32) * 0x85EBCA6Bu);
  h ^= h >> 16;
  h *= 0x7FEB352Du;
  h ^= h >> 15;
  h *= 0x846CA68Bu;
  h ^= h >> 16;
  return (h >> 8) * (1.f / 16777216.f);
}
__global__ void dropout_kernel(const float* __restrict__ a, size_t n, float p, uint32_t seed, float* __restrict__ out) {
  const float sc = 1.f / (1.f - p);
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
    out[i] = uhash(seed, i) >= p ? a[i] * sc : 0.f;
}

int dropout(const float* a, size_t n, float p, unsigned seed, float* out, hipStream_t st) {
  MT_REQUIRE(a && out && n > 0 && p >= 0.f && p < 1.f, "dropout: args");
  hipLaunchKernelGGL(dropout_kernel, ew_grid(n), dim3(256), 0, st, a, n, p, (uint32_t)seed, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------- group norm
// x [B][T][C], G groups of C/G channels, statistics over (T, C/G) per (b, g) (torch.nn.GroupNorm)
__global__ __launch_bounds__(256) void gn_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                     const float* __restrict__ beta, int T, int C, int G, float eps,
                                                     float* __restrict__ y, float* __restrict__ mean,
                                                     float* __restrict__ rstd) {
  __shared__ double red[2][256];
  const int b = blockIdx.y, g = blockIdx.x, cg = C / G, n = T * cg;
  const float* xb = x + (size_t)b * T * C + g * cg;
  double s = 0.0, q = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) {
    const double v = xb[(size_t)(i / cg) * C + i % cg];
    s += v;
    q += v * v;
  }
  red[0][threadIdx.x] = s;
  red[1][threadIdx.x] = q;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  const double mu = red[0][0] / n;
  const float var = (float)fmax(red[1][0] / n - mu * mu, 0.0);
  const float m = (float)mu, r = 1.f / sqrtf(var + eps);
  if (threadIdx.x == 0) {
    mean[b * G + g] = m;
    rstd[b * G + g] = r;
  }
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = g * cg + i % cg;
    const size_t o = ((size_t)b * T + i / cg) * C + c;
    y[o] = (x[o] - m) * r * gamma[c] + beta[c];
  }
}

// dx = rstd * (g*dy - mean(g*dy) - xhat * mean(g*dy*xhat)) over the group; dgamma/dbeta per (b, c) partials
// (summed over b by the caller with colsum)
__global__ __launch_bounds__(256) void gn_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                     const float* __restrict__ gamma, const float* __restrict__ mean,
                                                     const float* __restrict__ rstd, int T, int C, int G,
                                                     float* __restrict__ dx, float* __restrict__ dgp,
                                                     float* __restrict__ dbp) {
  __shared__ float red[2][256];
  const int b = blockIdx.y, g = blockIdx.x, cg = C / G, n = T * cg;
  const float m = mean[b * G + g], r = rstd[b * G + g];
  float s1 = 0.f, s2 = 0.f;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = g * cg + i % cg;
    const size_t o = ((size_t)b * T + i / cg) * C + c;
    const float gd = gamma[c] * dy[o], xh = (x[o] - m) * r;
    s1 += gd;
    s2 += gd * xh;
  }
  red[0][threadIdx.x] = s1;
  red[1][threadIdx.x] = s2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (threadIdx.x < o) {
      red[0][threadIdx.x] += red[0][threadIdx.x + o];
      red[1][threadIdx.x] += red[1][threadIdx.x + o];
    }
    __syncthreads();
  }
  const float a1 = red[0][0] / n, a2 = red[1][0] / n;
  for (int i = threadIdx.x; i < n; i += 256) {
    const int c = g * cg + i % cg;
    const size_t o = ((size_t)b * T + i / cg) * C + c;
    const float xh = (x[o] - m) * r;
    dx[o] = r * (gamma[c] * dy[o] - a1 - xh * a2);
  }
  // per-(b, c) parameter-gradient partials: 256 / cg frame lanes per channel, lanes combined in lane order
  __syncthreads();
  const int nl = 256 / cg, cc = threadIdx.x % cg, tl = threadIdx.x / cg;
  float pg = 0.f, pb = 0.f;
  if (tl < nl)
    for (int t = tl; t < T; t += nl) {
      const size_t o = ((size_t)b * T + t) * C + g * cg + cc;
      pg += dy[o] * (x[o] - m) * r;
      pb += dy[o];
    }
  red[0][threadIdx.x] = pg;
  red[1][threadIdx.x] = pb;
  __syncthreads();
  if (threadIdx.x < cg) {
    float sg = 0.f, sbb = 0.f;
    for (int l = 0; l < nl; ++l) {
      sg += red[0][l * cg + threadIdx.x];
      sbb += red[1][l * cg + threadIdx.x];
    }
    dgp[(size_t)b * C + g * cg + threadIdx.x] = sg;
    dbp[(size_t)b * C + g * cg + threadIdx.x] = sbb;
  }
}

int groupnorm_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, int G, float eps,
                  float* y, float* mean, float* rstd, hipStream_t st) {
  MT_REQUIRE(x && gamma && beta && y && mean && rstd && C % G == 0, "groupnorm: args");
  hipLaunchKernelGGL(gn_fwd_kernel, dim3(G, B), dim3(256), 0, st, x, gamma, beta, T, C, G, eps, y, mean, rstd);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int B,
                  int T, int C, int G, float* dx, float* dgp, float* dbp, hipStream_t st) {
  MT_REQUIRE(dy && x && gamma && mean && rstd && dx && dgp && dbp && C % G == 0 && C / G <= 256,
             "groupnorm_bwd: args");
  hipLaunchKernelGGL(gn_bwd_kernel, dim3(G, B), dim3(256), 0, st, dy, x, gamma, mean, rstd, T, C, G, dx, dgp, dbp);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------- layer norm
// per row of C (decoder nn.LayerNorm eps 1e-5; encoder channel LayerNorm eps 1e-4, model.py:148-166)
__global__ __launch_bounds__(64) void ln_fwd_kernel(const float* __restrict__ x, const float* __restrict__ gamma,
                                                    const float* __restrict__ beta, int C, float eps,
                                                    float* __restrict__ y, float* __restrict__ mean,
                                                    float* __restrict__ rstd) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float* xr = x + (size_t)row * C;
  float s = 0.f;
  for (int c = lane; c < C; c += 64) s += xr[c];
  s = wave_sum(s);
  const float m = s / C;
  float q = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float d = xr[c] - m;
    q += d * d;
  }
  q = wave_sum(q);
  const float r = 1.f / sqrtf(q / C + eps);
  if (lane == 0) {
    mean[row] = m;
    rstd[row] = r;
  }
  for (int c = lane; c < C; c += 64) y[(size_t)row * C + c] = (xr[c] - m) * r * gamma[c] + beta[c];
}

__global__ __launch_bounds__(64) void ln_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ x,
                                                    const float* __restrict__ gamma, const float* __restrict__ mean,
                                                    const float* __restrict__ rstd, int C, float* __restrict__ dx) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const float m = mean[row], r = rstd[row];
  const float* xr = x + (size_t)row * C;
  const float* dr = dy + (size_t)row * C;
  float s1 = 0.f, s2 = 0.f;
  for (int c = lane; c < C; c += 64) {
    const float gd = gamma[c] * dr[c];
    s1 += gd;
    s2 += gd * (xr[c] - m) * r;
  }
  s1 = wave_sum(s1) / C;
  s2 = wave_sum(s2) / C;
  for (int c = lane; c < C; c += 64) dx[(size_t)row * C + c] = r * (gamma[c] * dr[c] - s1 - (xr[c] - m) * r * s2);
}

int layernorm_fwd(const float* x, const float* gamma, const float* beta, int rows, int C, float eps, float* y,
                  float* mean, float* rstd, hipStream_t st) {
  MT_REQUIRE(x && gamma && beta && y && mean && rstd && rows > 0 && C > 0, "layernorm: args");
  hipLaunchKernelGGL(ln_fwd_kernel, dim3(rows), dim3(64), 0, st, x, gamma, beta, C, eps, y, mean, rstd);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int rows,
                  int C, float* dx, hipStream_t st) {
  MT_REQUIRE(dy && x && gamma && mean && rstd && dx && rows > 0, "layernorm_bwd: args");
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(rows), dim3(64), 0, st, dy, x, gamma, mean, rstd, C, dx);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------ SnakeBeta
// y = x + 1/(exp(beta)+1e-9) * sin(x exp(alpha))^2 per channel (model.py:580-609, log-scale parameters)
__global__ void snake_fwd_kernel(const float* __restrict__ x, const float* __restrict__ la,
                                 const float* __restrict__ lb, size_t n, int C, float* __restrict__ y) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float al = expf(la[c]), ib = 1.f / (expf(lb[c]) + 1e-9f);
    const float s = sinf(x[i] * al);
    y[i] = x[i] + ib * (s * s);
  }
}

// dx = dy (1 + ib sin(2 x al) al); per-element parameter-gradient terms (reduced by colsum):
// ga = dy ib sin(2 x al) x al (d/d log-alpha), gb = -dy sin^2(x al) ib^2 exp(beta) (d/d log-beta)
__global__ void snake_bwd_kernel(const float* __restrict__ x, const float* __restrict__ la,
                                 const float* __restrict__ lb, const float* __restrict__ dy, size_t n, int C,
                                 float* __restrict__ dx, float* __restrict__ ga, float* __restrict__ gb) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const int c = (int)(i % C);
    const float al = expf(la[c]), eb = expf(lb[c]), ib = 1.f / (eb + 1e-9f);
    const float xa = x[i] * al, s = sinf(xa), s2 = sinf(2.f * xa);
    dx[i] = dy[i] * (1.f + ib * s2 * al);
    ga[i] = dy[i] * ib * s2 * xa;
    gb[i] = -dy[i] * s * s * ib * ib * eb;
  }
}

int snake_fwd(const float* x, const float* la, const float* lb, size_t n, int C, float* y, hipStream_t st) {
  MT_REQUIRE(x && la && lb && y && n > 0, "snake: args");
  hipLaunchKernelGGL(snake_fwd_kernel, ew_grid(n), dim3(256), 0, st, x, la, lb, n, C, y);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int snake_bwd(const float* x, const float* la, const float* lb, const float* dy, size_t n, int C, float* dx, float* ga,
              float* gb, hipStream_t st) {
  MT_REQUIRE(x && la && lb && dy && dx && ga && gb && n > 0, "snake_bwd: args");
  hipLaunchKernelGGL(snake_bwd_kernel, ew_grid(n), dim3(256), 0, st, x, la, lb, dy, n, C, dx, ga, gb);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// -------------------------------------------------------------------------------------------- softmax
// s [BH][Tq][Tk] scores (unscaled); kmask [B][Tk]; row softmax of scale * s with
//   mode 0: masked keys := +3.4e38 (decoder, model.py:697: -finfo.min), mode 1: masked := -1e4 (encoder,
//   model.py:353; its mask is x_mask(q) * x_mask(k), so a masked query row is all -1e4: uniform)
__global__ __launch_bounds__(64) void softmax_fwd_kernel(const float* __restrict__ s, const float* __restrict__ kmask,
                                                         const float* __restrict__ qmask, int H, int Tq, int Tk,
                                                         float scale, int mode, float* __restrict__ p) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const int bh = row / Tq, b = bh / H, q = row % Tq;
  const float* sr = s + (size_t)row * Tk;
  float* pr = p + (size_t)row * Tk;
  const float* km = kmask + (size_t)b * Tk;
  const bool qok = !qmask || qmask[(size_t)b * Tq + q] != 0.f;
  float mx = -INFINITY;
  for (int j = lane; j < Tk; j += 64) {
    float v = sr[j] * scale;
    if (km[j] == 0.f || !qok) v = mode == 0 ? 3.4028234663852886e38f : -1e4f;
    mx = fmaxf(mx, v);
  }
  mx = wave_max(mx);
  float sum = 0.f;
  for (int j = lane; j < Tk; j += 64) {
    float v = sr[j] * scale;
    if (km[j] == 0.f || !qok) v = mode == 0 ? 3.4028234663852886e38f : -1e4f;
    const float e = expf(v - mx);
    pr[j] = e;
    sum += e;
  }
  sum = wave_sum(sum);
  const float inv = 1.f / sum;
  for (int j = lane; j < Tk; j += 64) pr[j] *= inv;
}

// ds = scale * p * (dp - sum_j p dp) (masked entries carry p = 0 or a constant: their score gradient is
// zero because masked_fill replaced the score — handled by zeroing ds where the fill applied)
__global__ __launch_bounds__(64) void softmax_bwd_kernel(const float* __restrict__ p, const float* __restrict__ dp,
                                                         const float* __restrict__ kmask,
                                                         const float* __restrict__ qmask, int H, int Tq, int Tk,
                                                         float scale, float* __restrict__ ds) {
  const int row = blockIdx.x, lane = threadIdx.x;
  const int bh = row / Tq, b = bh / H, q = row % Tq;
  const float* pr = p + (size_t)row * Tk;
  const float* dr = dp + (size_t)row * Tk;
  const float* km = kmask + (size_t)b * Tk;
  const bool qok = !qmask || qmask[(size_t)b * Tq + q] != 0.f;
  float dot = 0.f;
  for (int j = lane; j < Tk; j += 64) dot += pr[j] * dr[j];
  dot = wave_sum(dot);
  for (int j = lane; j < Tk; j += 64) {
    const bool filled = km[j] == 0.f || !qok;
    ds[(size_t)row * Tk + j] = filled ? 0.f : scale * pr[j] * (dr[j] - dot);
  }
}

int softmax_fwd(const float* s, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk, float scale,
                int mode, float* p, hipStream_t st) {
  MT_REQUIRE(s && kmask && p && BH > 0 && H > 0 && Tq > 0 && Tk > 0 && (mode == 0 || mode == 1), "softmax: args");
  hipLaunchKernelGGL(softmax_fwd_kernel, dim3(BH * Tq), dim3(64), 0, st, s, kmask, qmask, H, Tq, Tk, scale, mode, p);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int softmax_bwd(const float* p, const float* dp, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk,
                float scale, float* ds, hipStream_t st) {
  MT_REQUIRE(p && dp && kmask && ds, "softmax_bwd: args");
  hipLaunchKernelGGL(softmax_bwd_kernel, dim3(BH * Tq), dim3(64), 0, st, p, dp, kmask, qmask, H, Tq, Tk, scale, ds);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ----------------------------------------------------------------------------------------------- RoPE
// x [B][T][H*dh] (head h at columns h*dh..), rotary on the first d features of each head with theta[d/2]
// (model.py:244-292: x' = x cos + rot(x) sin, rot = [-x[h:], x[:h]]); inverse = rotation by -angle
__global__ void rope_kernel(float* __restrict__ x, int B, int T, int H, int dh, int d, const float* __restrict__ theta,
                            int inverse) {
  const int hd = d / 2;
  const size_t total = (size_t)B * T * H * hd;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int j = (int)(i % hd);
    size_t r = i / hd;
    const int h = (int)(r % H);
    r /= H;
    const int t = (int)(r % T);
    const int b = (int)(r / T);
    float* p = x + ((size_t)b * T + t) * H * dh + h * dh;
    const float ang = (float)t * theta[j];
    float sn, cs;
    sincosf(ang, &sn, &cs);
    if (inverse) sn = -sn;
    const float x0 = p[j], x1 = p[j + hd];
    p[j] = x0 * cs - x1 * sn;
    p[j + hd] = x1 * cs + x0 * sn;
  }
}

int rope(float* x, int B, int T, int H, int dh, int d, const float* theta, int inverse, hipStream_t st) {
  MT_REQUIRE(x && theta && d % 2 == 0 && d <= dh, "rope: args");
  hipLaunchKernelGGL(rope_kernel, ew_grid((size_t)B * T * H * (d / 2)), dim3(256), 0, st, x, B, T, H, dh, d, theta,
                     inverse);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------------ embedding
__global__ void embed_fwd_kernel(const long long* __restrict__ ids, size_t ntok, const float* __restrict__ table,
                                 int C, float scale, float* __restrict__ out) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < ntok * C; i += (size_t)gridDim.x * blockDim.x)
    out[i] = table[(size_t)ids[i / C] * C + i % C] * scale;
}

// dtable[v][c] = scale * sum over tokens with id v of dout[tok][c]: a 256-thread block per (v, 64 columns), 4 token
// lanes per column, lanes combined in order (deterministic)
__global__ __launch_bounds__(256) void embed_bwd_kernel(const long long* __restrict__ ids, size_t ntok,
                                                        const float* __restrict__ dout, int V, int C, float scale,
                                                        float* __restrict__ dtable) {
  __shared__ float red[4][64];
  const int cl = threadIdx.x & 63, lr = threadIdx.x >> 6, c = blockIdx.x * 64 + cl, v = blockIdx.y;
  float s = 0.f;
  if (c < C)
    for (size_t t = lr; t < ntok; t += 4)
      if (ids[t] == v) s += dout[t * C + c];
  red[lr][cl] = s;
  __syncthreads();
  if (lr == 0 && c < C) dtable[(size_t)v * C + c] = (((red[0][cl] + red[1][cl]) + red[2][cl]) + red[3][cl]) * scale;
}

int embed_fwd(const long long* ids, size_t ntok, const float* table, int C, float scale, float* out, hipStream_t st) {
  MT_REQUIRE(ids && table && out && ntok > 0, "embed: args");
  hipLaunchKernelGGL(embed_fwd_kernel, ew_grid(ntok * C), dim3(256), 0, st, ids, ntok, table, C, scale, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int embed_bwd(const long long* ids, size_t ntok, const float* dout, int V, int C, float scale, float* dtable,
              hipStream_t st) {
  MT_REQUIRE(ids && dout && dtable && V > 0, "embed_bwd: args");
  hipLaunchKernelGGL(embed_bwd_kernel, dim3((C + 63) / 64, V), dim3(256), 0, st, ids, ntok, dout, V, C, scale, dtable);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ---------------------------------------------------------------------------------------------- Adam
// torch.optim.Adam (lr, betas (0.9, 0.999), eps 1e-8, no weight decay) with grad := grad * gscale[0]
// (gscale = clip factor / world size, computed on the device): exp_avg.lerp_(g, 1-b1);
// exp_avg_sq.mul_(b2).addcmul_(g, g, 1-b2); denom = sqrt(exp_avg_sq) / sqrt(bc2) + eps;
// p -= lr / bc1 * exp_avg / denom
__global__ void adam_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                            float* __restrict__ v, size_t n, const float* __restrict__ gscale, float step_size,
                            float b1, float b2, float eps, float bc2_sqrt) {
  const float sc = gscale ? gscale[0] : 1.f;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
    const float gi = g[i] * sc;
    const float mi = m[i] + (1.f - b1) * (gi - m[i]);
    const float vi = v[i] * b2 + (1.f - b2) * gi * gi;
    m[i] = mi;
    v[i] = vi;
    const float denom = sqrtf(vi) / bc2_sqrt + eps;
    p[i] = p[i] + (-step_size) * (mi / denom);
  }
}

// clip factor of the global norm of the world-averaged gradient (the flat buffer holds the SUM over ranks):
// norm = sqrt(sumsq) / world, out = min(1, max_norm / (norm + 1e-6)) / world (torch.nn.utils.clip_grad_norm_ on
// DDP-averaged gradients)
__global__ void clip_factor_kernel(const float* __restrict__ sumsq, float max_norm, float inv_world,
                                   float* __restrict__ out, float* __restrict__ norm_out) {
  const float nrm = sqrtf(sumsq[0]) * inv_world;
  const float c = max_norm / (nrm + 1e-6f);
  out[0] = (c < 1.f ? c : 1.f) * inv_world;
  if (norm_out) norm_out[0] = nrm;
}

int adam_step(float* p, const float* g, float* m, float* v, size_t n, const float* gscale, float lr, float b1,
              float b2, float eps, int step, hipStream_t st) {
  MT_REQUIRE(p && g && m && v && n > 0 && step >= 1, "adam: args");
  // bias corrections in double on the host, as torch's single-tensor Adam computes them from Python floats
  const double bc1 = 1.0 - pow((double)b1, step), bc2 = 1.0 - pow((double)b2, step);
  hipLaunchKernelGGL(adam_kernel, ew_grid(n), dim3(256), 0, st, p, g, m, v, n, gscale, (float)(lr / bc1), b1, b2, eps,
                     (float)sqrt(bc2));
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int clip_factor(const float* sumsq, float max_norm, float inv_world, float* out, float* norm_out, hipStream_t st) {
  MT_REQUIRE(sumsq && out, "clip_factor: args");
  hipLaunchKernelGGL(clip_factor_kernel, dim3(1), dim3(1), 0, st, sumsq, max_norm, inv_world, out, norm_out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
