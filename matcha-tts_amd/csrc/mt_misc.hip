// Support kernels: weight packing, layout transposes, time-embedding MLP, the
// duration -> alignment index path, denormalize/crop.
#include "mt_misc.h"

#include <algorithm>

namespace mt {

// ------------------------------------------------------------------------------------
// weight packing: reference fp32 layouts -> [Mpad][taps][cin_pad] element type
//   kind 0: Conv1d  W[cout][cin][k]       -> taps = k,   row m = co
//   kind 1: ConvT   W[cin][cout][k], s    -> taps = k/s, row m = phase*cout + co,
//                                            tap t <-> kernel index phase + (taps-1-t)*s
// rows >= M and channels >= cin are zero.
// ------------------------------------------------------------------------------------
template <class E>
__global__ void pack_conv_kernel(const float* __restrict__ W, int kind, int cout, int cin, int k,
                                 int s, int row0, int Mpad, int taps, int cin_pad, int Mrows,
                                 const float* __restrict__ colscale, E* __restrict__ out) {
  const size_t total = (size_t)Mrows * taps * cin_pad;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total;
       i += (size_t)gridDim.x * blockDim.x) {
    const int ci = (int)(i % cin_pad);
    const int t = (int)((i / cin_pad) % taps);
    const int m = (int)(i / ((size_t)cin_pad * taps));
    float v = 0.f;
    if (ci < cin) {
      if (kind == 0) {
        if (m < cout) v = W[((size_t)m * cin + ci) * k + t] * (colscale ? colscale[ci] : 1.f);
      } else {
        const int ph = m / cout, co = m % cout;
        if (ph < s) {
          const int kk = ph + (taps - 1 - t) * s;
          v = W[((size_t)ci * cout + co) * k + kk];
        }
      }
    }
    out[((size_t)(row0 + m) * taps + t) * cin_pad + ci] = from_f<E>(v);
  }
  (void)Mpad;
}

int pack_conv(int dtype, const float* W, int kind, int cout, int cin, int k, int s, int row0,
              int Mrows, int Mpad, int taps, int cin_pad, void* out, hipStream_t st, const float* colscale) {
  const size_t total = (size_t)Mrows * taps * cin_pad;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  if (dtype == BF16)
    hipLaunchKernelGGL(pack_conv_kernel<bf16>, dim3(blocks), dim3(256), 0, st, W, kind, cout, cin, k, s,
                       row0, Mpad, taps, cin_pad, Mrows, colscale, (bf16*)out);
  else
    hipLaunchKernelGGL(pack_conv_kernel<float>, dim3(blocks), dim3(256), 0, st, W, kind, cout, cin, k,
                       s, row0, Mpad, taps, cin_pad, Mrows, colscale, (float*)out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// out[m] = src ? src[m % period] : 0, m < n ; op 1: exp(src); op 2: 1/(exp(src)+1e-9)
__global__ void vec_kernel(const float* __restrict__ src, int period, int n, int op,
                           float* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  float v = src ? src[i % period] : 0.f;
  if (op == 1) v = expf(v);
  if (op == 2) v = 1.0f / (expf(v) + 1e-9f);
  out[i] = v;
}

int pack_vec(const float* src, int period, int n, int op, float* out, hipStream_t st) {
  hipLaunchKernelGGL(vec_kernel, dim3((n + 255) / 256), dim3(256), 0, st, src, period, n, op, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// LayerNorm folding (pack time): out[row0 + m] += sum_i W[m][i] * beta[i]  (W [M][K] fp32, Linear)
__global__ void fold_bias_kernel(const float* __restrict__ W, const float* __restrict__ beta, int M, int K,
                                 float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int m = blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= M) return;
  double acc = 0.0;
  for (int i = lane; i < K; i += 64) acc += (double)W[(size_t)m * K + i] * (double)beta[i];
  acc = wave_sum_d(acc);
  if (lane == 0) out[m] = (float)((double)out[m] + acc);
}

int fold_bias(const float* W, const float* beta, int M, int K, float* out, hipStream_t st) {
  hipLaunchKernelGGL(fold_bias_kernel, dim3((M + 3) / 4), dim3(256), 0, st, W, beta, M, K, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------
// LayerNorm row statistics (nn.LayerNorm over the channel axis of [rows][C], C = 256):
// 16 lanes per row, two-pass in registers (mean, then mean of squared deviations).
// ------------------------------------------------------------------------------------
template <class E, int C>
__global__ __launch_bounds__(256) void rowstats_kernel(const E* __restrict__ x, int rows, float eps,
                                                       float* __restrict__ stats) {
  constexpr int VN = Vec16<E>::N;
  constexpr int NV = C / 16 / VN;  // 16-byte vectors per lane
  const int lane = threadIdx.x & 63;
  const int row = (blockIdx.x * blockDim.x + threadIdx.x) >> 4;
  const int sub = lane & 15;
  const bool ok = row < rows;
  const E* p = x + (size_t)(ok ? row : 0) * C;
  Vec16<E> v[NV];
#pragma unroll
  for (int i = 0; i < NV; ++i) v[i] = load16(p + (i * 16 + sub) * VN);
  float s = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < VN; ++k) s += v[i].get(k);
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) s += __shfl_xor(s, o, 64);
  const float mean = s / (float)C;
  float q = 0.f;
#pragma unroll
  for (int i = 0; i < NV; ++i)
#pragma unroll
    for (int k = 0; k < VN; ++k) {
      const float d = v[i].get(k) - mean;
      q += d * d;
    }
#pragma unroll
  for (int o = 1; o < 16; o <<= 1) q += __shfl_xor(q, o, 64);
  if (ok && sub == 0) {
    stats[(size_t)row * 2] = mean;
    stats[(size_t)row * 2 + 1] = 1.f / sqrtf(q / (float)C + eps);
  }
}

int rowstats(int dtype, const void* x, int rows, int C, float eps, float* stats, hipStream_t st) {
  MT_REQUIRE(C == 256, "rowstats: C=%d (built for 256)", C);
  dim3 grid((rows * 16 + 255) / 256);
  if (dtype == BF16)
    hipLaunchKernelGGL((rowstats_kernel<bf16, 256>), grid, dim3(256), 0, st, (const bf16*)x, rows, eps, stats);
  else
    hipLaunchKernelGGL((rowstats_kernel<float, 256>), grid, dim3(256), 0, st, (const float*)x, rows, eps, stats);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------
// layout transposes  [B][C][T] fp32  <->  [B][T][ld] (column offset coff)
// ------------------------------------------------------------------------------------
template <class E>
__global__ void bct_to_btc_kernel(const float* __restrict__ src, int C, int T, float scale,
                                  E* __restrict__ dst, int ld, int coff) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    tile[i][tx] = (c < C && t < T) ? src[((size_t)b * C + c) * T + t] : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    if (c < C && t < T) dst[((size_t)b * T + t) * ld + coff + c] = from_f<E>(tile[tx][i] * scale);
  }
}

template <class E>
__global__ void btc_to_bct_kernel(const E* __restrict__ src, int ld, int coff, int C, int T,
                                  float* __restrict__ dst) {
  __shared__ float tile[32][33];
  const int b = blockIdx.z, c0 = blockIdx.y * 32, t0 = blockIdx.x * 32;
  const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;
  for (int i = ty; i < 32; i += 8) {
    const int t = t0 + i, c = c0 + tx;
    tile[i][tx] = (c < C && t < T) ? to_f(src[((size_t)b * T + t) * ld + coff + c]) : 0.f;
  }
  __syncthreads();
  for (int i = ty; i < 32; i += 8) {
    const int c = c0 + i, t = t0 + tx;
    if (c < C && t < T) dst[((size_t)b * C + c) * T + t] = tile[tx][i];
  }
}

int bct_to_btc(int dtype, const float* src, int B, int C, int T, float scale, void* dst, int ld,
               int coff, hipStream_t st) {
  dim3 grid((T + 31) / 32, (C + 31) / 32, B);
  if (dtype == BF16)
    hipLaunchKernelGGL(bct_to_btc_kernel<bf16>, grid, dim3(256), 0, st, src, C, T, scale, (bf16*)dst, ld,
                       coff);
  else
    hipLaunchKernelGGL(bct_to_btc_kernel<float>, grid, dim3(256), 0, st, src, C, T, scale, (float*)dst,
                       ld, coff);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int btc_to_bct(int dtype, const void* src, int ld, int coff, int B, int C, int T, float* dst,
               hipStream_t st) {
  dim3 grid((T + 31) / 32, (C + 31) / 32, B);
  if (dtype == BF16)
    hipLaunchKernelGGL(btc_to_bct_kernel<bf16>, grid, dim3(256), 0, st, (const bf16*)src, ld, coff, C, T,
                       dst);
  else
    hipLaunchKernelGGL(btc_to_bct_kernel<float>, grid, dim3(256), 0, st, (const float*)src, ld, coff, C,
                       T, dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// speaker embedding broadcast into the estimator input: dst[b][t][coff + c] = spks[b][c]
template <class E>
__global__ void spk_fill_kernel(const float* __restrict__ spks, int C, int T, E* __restrict__ dst,
                                int ld, int coff) {
  const int b = blockIdx.y;
  for (int i = blockIdx.x * blockDim.x + threadIdx.x; i < T * C; i += gridDim.x * blockDim.x) {
    const int t = i / C, c = i % C;
    dst[((size_t)b * T + t) * ld + coff + c] = from_f<E>(spks[(size_t)b * C + c]);
  }
}

int spk_fill(int dtype, const float* spks, int B, int C, int T, void* dst, int ld, int coff,
             hipStream_t st) {
  dim3 grid(std::min((T * C + 255) / 256, 4096), B);
  if (dtype == BF16)
    hipLaunchKernelGGL(spk_fill_kernel<bf16>, grid, dim3(256), 0, st, spks, C, T, (bf16*)dst, ld, coff);
  else
    hipLaunchKernelGGL(spk_fill_kernel<float>, grid, dim3(256), 0, st, spks, C, T, (float*)dst, ld, coff);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// mask at half resolution: m1[b][t] = m0[b][2t]  (model.py:1003 mask[:, :, ::2])
__global__ void mask_half_kernel(const float* __restrict__ m0, int T0, int T1, int B,
                                 float* __restrict__ m1) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= B * T1) return;
  const int b = i / T1, t = i % T1;
  m1[i] = m0[(size_t)b * T0 + 2 * t];
}

int mask_half(const float* m0, int B, int T0, float* m1, hipStream_t st) {
  const int T1 = (T0 + 1) / 2;
  hipLaunchKernelGGL(mask_half_kernel, dim3((B * T1 + 255) / 256), dim3(256), 0, st, m0, T0, T1, B, m1);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------
// time embedding (model.py:747-762, 819-832, 780): per solver evaluation s
//   emb[s] = [sin(1000 t_s f_k), cos(1000 t_s f_k)]  (f_k = exp(-k ln(1e4)/(half-1)), host table)
// ------------------------------------------------------------------------------------
__global__ void sinus_kernel(TimeSched ts, const float* __restrict__ t_dev, const float* __restrict__ freq,
                             int half, float* __restrict__ emb) {
  const int s = blockIdx.x;
  const float st = 1000.f * (t_dev ? t_dev[s] : ts.t[s]);
  for (int k = threadIdx.x; k < 2 * half; k += blockDim.x) {
    const float a = st * freq[k % half];
    emb[(size_t)s * 2 * half + k] = k < half ? sinf(a) : cosf(a);
  }
}

int sinus_embed(const TimeSched& ts, int S, const float* freq, int half, float* emb, hipStream_t st,
                const float* t_dev) {
  MT_REQUIRE(S > 0 && (t_dev || S <= TimeSched::MAX), "time schedule length %d", S);
  hipLaunchKernelGGL(sinus_kernel, dim3(S), dim3(256), 0, st, ts, t_dev, freq, half, emb);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// y[s][yoff + o] = post( sum_i W[o][i] * pre(x[s][i]) + bias[o] ); one wave per output o.
// pre: 0 none, 1 mish ; post: 0 none, 1 silu, 2 mish
// The time-embedding MLPs (model.py TimestepEmbedding, ResnetBlock1D.mlp): S <= 128 rows, I <= 1024.
// pre(x) of RD_S rows is staged once per block in LDS, each wave keeps its output's weight row in
// registers across all rows; per (s, o) the lane-strided sum + wave reduction order is fixed.
constexpr int RD_S = 8, RD_NO = 2, RD_IMAX = 1024;
__global__ __launch_bounds__(256) void rowdot_kernel(const float* __restrict__ x, int ldx,
                                                     const float* __restrict__ W,
                                                     const float* __restrict__ bias, float* __restrict__ y,
                                                     int ldy, int yoff, int S, int O, int I, int pre, int post) {
  __shared__ float xs[RD_S][RD_IMAX];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int KW = RD_IMAX / 64;
  float wv[RD_NO][KW];
  const int obase = (blockIdx.x * 4 + wave) * RD_NO;
#pragma unroll
  for (int j = 0; j < RD_NO; ++j)
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int o = obase + j, i = lane + 64 * k;
      wv[j][k] = (o < O && i < I) ? W[(size_t)o * I + i] : 0.f;
    }
  for (int s0 = 0; s0 < S; s0 += RD_S) {
    const int ns = min(RD_S, S - s0);
    __syncthreads();
    for (int e = threadIdx.x; e < ns * I; e += 256) {
      const int r = e / I, i = e - r * I;
      float xv = x[(size_t)(s0 + r) * ldx + i];
      if (pre == 1) xv = xv * tanhf(log1pf(expf(xv)));
      xs[r][i] = xv;
    }
    __syncthreads();
    for (int r = 0; r < ns; ++r) {
#pragma unroll
      for (int j = 0; j < RD_NO; ++j) {
        const int o = obase + j;
        float acc = 0.f;
#pragma unroll
        for (int k = 0; k < KW; ++k)
          if (lane + 64 * k < I) acc += wv[j][k] * xs[r][lane + 64 * k];
        acc = wave_sum(acc);
        if (lane == 0 && o < O) {
          float v = acc + (bias ? bias[o] : 0.f);
          if (post == 1) v = v / (1.f + expf(-v));
          if (post == 2) v = v * tanhf(log1pf(expf(v)));
          y[(size_t)(s0 + r) * ldy + yoff + o] = v;
        }
      }
    }
  }
}

// The same product with one output per wave and 16-byte weight / row loads (I % 4 == 0): O / 4 workgroups per
// segment, several weight matrices of one shape in one launch. Per (s, o) the sum order is fixed: lane-strided
// float4 partial dot products, then the wave reduction.
__global__ __launch_bounds__(256) void rowdot4_kernel(const float* __restrict__ x, int ldx, RowdotSegs sg,
                                                      float* __restrict__ y, int ldy, int S, int O, int I, int pre,
                                                      int post) {
  __shared__ f32x4 xs[RD_S][RD_IMAX / 4];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int bps = (O + 3) / 4, seg = blockIdx.x / bps;
  const int o = (blockIdx.x - seg * bps) * 4 + wave, I4 = I / 4;
  const f32x4* W4 = reinterpret_cast<const f32x4*>(sg.W[seg]);
  constexpr int KW = RD_IMAX / 256;
  f32x4 wv[KW];
#pragma unroll
  for (int k = 0; k < KW; ++k) {
    const int i4 = lane + 64 * k;
    wv[k] = (o < O && i4 < I4) ? W4[(size_t)o * I4 + i4] : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  for (int s0 = 0; s0 < S; s0 += RD_S) {
    const int ns = min(RD_S, S - s0);
    __syncthreads();
    for (int e = threadIdx.x; e < ns * I4; e += 256) {
      const int r = e / I4, i4 = e - r * I4;
      f32x4 xv = *reinterpret_cast<const f32x4*>(x + (size_t)(s0 + r) * ldx + 4 * i4);
      if (pre == 1)
#pragma unroll
        for (int c = 0; c < 4; ++c) xv[c] = xv[c] * tanhf(log1pf(expf(xv[c])));
      xs[r][i4] = xv;
    }
    __syncthreads();
    for (int r = 0; r < ns; ++r) {
      float acc = 0.f;
#pragma unroll
      for (int k = 0; k < KW; ++k)
        if (lane + 64 * k < I4) {
          const f32x4 xv = xs[r][lane + 64 * k];
          acc += wv[k][0] * xv[0] + wv[k][1] * xv[1] + wv[k][2] * xv[2] + wv[k][3] * xv[3];
        }
      acc = wave_sum(acc);
      if (lane == 0 && o < O) {
        float v = acc + (sg.b[seg] ? sg.b[seg][o] : 0.f);
        if (post == 1) v = v / (1.f + expf(-v));
        if (post == 2) v = v * tanhf(log1pf(expf(v)));
        y[(size_t)(s0 + r) * ldy + sg.yoff[seg] + o] = v;
      }
    }
  }
}

int rowdot_segs(const float* x, int ldx, const RowdotSegs& sg, float* y, int ldy, int S, int O, int I, int pre,
                int post, hipStream_t st) {
  MT_REQUIRE(I > 0 && I <= RD_IMAX && I % 4 == 0 && ldx % 4 == 0 && S > 0 && O > 0 && sg.n >= 1 &&
                 sg.n <= ROWDOT_MAXSEG,
             "rowdot_segs: I %d (max %d, multiple of 4), ldx %d, S %d, O %d, %d segments", I, RD_IMAX, ldx, S, O,
             sg.n);
  hipLaunchKernelGGL(rowdot4_kernel, dim3(sg.n * ((O + 3) / 4)), dim3(256), 0, st, x, ldx, sg, y, ldy, S, O, I, pre,
                     post);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int rowdot(const float* x, int ldx, const float* W, const float* bias, float* y, int ldy, int yoff,
           int S, int O, int I, int pre, int post, hipStream_t st) {
  MT_REQUIRE(I > 0 && I <= RD_IMAX && S > 0 && O > 0, "rowdot: I %d (max %d), S %d, O %d", I, RD_IMAX, S, O);
  if (I % 4 == 0 && ldx % 4 == 0) {
    RowdotSegs sg{};
    sg.W[0] = W;
    sg.b[0] = bias;
    sg.yoff[0] = yoff;
    sg.n = 1;
    return rowdot_segs(x, ldx, sg, y, ldy, S, O, I, pre, post, st);
  }
  const int per = 4 * RD_NO;
  hipLaunchKernelGGL(rowdot_kernel, dim3((O + per - 1) / per), dim3(256), 0, st, x, ldx, W, bias, y, ldy, yoff,
                     S, O, I, pre, post);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------
// duration -> alignment index path (model.py:1273-1289, 42-76). Bit-exact: every value is
// an integer-valued fp32 (< 2^24), so sums and prefix sums are exact in any order.
// ------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void durations_kernel(const float* __restrict__ logw, const float* __restrict__ xmask,
                                                        float ls, int Tx, float* __restrict__ w_ceil,
                                                        float* __restrict__ cum, long long* __restrict__ ylen) {
  // chunks of 256 * DUR_PER tokens; in a chunk thread t owns the `per` consecutive tokens [t * per, (t + 1) * per):
  // ceil(exp(logw) * mask * ls), then an inclusive block scan of the per-thread sums (wave shuffles + one LDS pass)
  // on top of the previous chunks' total. Every value is an integer-valued fp32 below 2^24, so this order gives the
  // serial cumsum's bits exactly.
  constexpr int DUR_PER = 32;
  __shared__ float wsum[4];
  const int b = blockIdx.x, tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  float base = 0.f;
  for (int c0 = 0; c0 < Tx; c0 += 256 * DUR_PER) {
    const int n = min(Tx - c0, 256 * DUR_PER);
    const int per = (n + 255) / 256, x0 = c0 + tid * per;
    float w[DUR_PER];
    float s = 0.f;
#pragma unroll
    for (int k = 0; k < DUR_PER; ++k) {
      const int x = x0 + k;
      w[k] = 0.f;
      if (k < per && x < c0 + n) {
        const size_t i = (size_t)b * Tx + x;
        w[k] = ceilf((expf(logw[i]) * xmask[i]) * ls);
        w_ceil[i] = w[k];
        s += w[k];
      }
    }
    float inc = s;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const float v = __shfl_up(inc, o, 64);
      if (lane >= o) inc += v;
    }
    __syncthreads();  // the previous chunk's wsum reads are done
    if (lane == 63) wsum[wv] = inc;
    __syncthreads();
    float run = base + (inc - s);
    for (int u = 0; u < wv; ++u) run += wsum[u];
#pragma unroll
    for (int k = 0; k < DUR_PER; ++k) {
      const int x = x0 + k;
      if (k < per && x < c0 + n) {
        run += w[k];
        cum[(size_t)b * Tx + x] = run;
      }
    }
    base += wsum[0] + wsum[1] + wsum[2] + wsum[3];
  }
  if (tid == 255) ylen[b] = (long long)(base < 1.f ? 1.f : base);
}

int durations(const float* logw, const float* xmask, float ls, int B, int Tx, float* w_ceil, float* cum,
              long long* ylen, hipStream_t st) {
  MT_REQUIRE(B > 0 && Tx > 0, "durations: B %d, Tx %d", B, Tx);
  hipLaunchKernelGGL(durations_kernel, dim3(B), dim3(256), 0, st, logw, xmask, ls, Tx, w_ceil, cum, ylen);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// frame j of utterance b belongs to the first token x with cum[x] > j (if j < cum[Tx-1]).
// attn[b][x][j] one-hot (optional), mu_y[b][c][j] = mu[b][c][x] (an exact gather).
__global__ void alignment_kernel(const float* __restrict__ cum, const long long* __restrict__ ylen, int Tx,
                                 int T, const float* __restrict__ mu, int C, float* __restrict__ attn,
                                 float* __restrict__ mu_y, float* __restrict__ y_mask) {
  const int b = blockIdx.y, z = blockIdx.z, Z = gridDim.z;  // z: this block's share of the token rows / channels
  const int j = blockIdx.x * blockDim.x + threadIdx.x;
  if (j >= T) return;
  const float* cb = cum + (size_t)b * Tx;
  const float jf = (float)j;
  int tok = -1;
  if (jf < cb[Tx - 1]) {
    int lo = 0, hi = Tx - 1;  // first index with cb[x] > j
    while (lo < hi) {
      const int mid = (lo + hi) >> 1;
      if (cb[mid] > jf) hi = mid; else lo = mid + 1;
    }
    tok = lo;
  }
  if (attn) {
    float* ab = attn + (size_t)b * Tx * T + j;
    for (int x = z * Tx / Z; x < (z + 1) * Tx / Z; ++x) ab[(size_t)x * T] = (x == tok) ? 1.f : 0.f;
  }
  if (y_mask && z == 0) y_mask[(size_t)b * T + j] = (long long)j < ylen[b] ? 1.f : 0.f;
  if (mu_y) {
    for (int c = z * C / Z; c < (z + 1) * C / Z; ++c)
      mu_y[((size_t)b * C + c) * T + j] = tok >= 0 ? mu[((size_t)b * C + c) * Tx + tok] : 0.f;
  }
}

int alignment(const float* cum, const long long* ylen, int B, int Tx, int T, const float* mu, int C, float* attn,
              float* mu_y, float* y_mask, hipStream_t st) {
  MT_REQUIRE(B > 0 && Tx > 0 && T > 0, "alignment: empty input");
  // the writes (the one-hot attn [B][Tx][T] dominates: 23 MB at B = 32) split over 8 blocks per frame range
  dim3 grid((T + 255) / 256, B, std::max(1, std::min(8, std::min(Tx, std::max(C, 1)))));
  hipLaunchKernelGGL(alignment_kernel, grid, dim3(256), 0, st, cum, ylen, Tx, T, mu, C, attn, mu_y, y_mask);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// mel[b][c][t] = z[b][c][t] * std[c] + mean[c], t < Ty   (model.py:106-125, 1295-1298)
__global__ void denorm_crop_kernel(const float* __restrict__ z, const float* __restrict__ mean,
                                   const float* __restrict__ stdv, int C, int T, int Ty,
                                   float* __restrict__ mel) {
  const int bc = blockIdx.y;
  const int c = bc % C;
  for (int t = blockIdx.x * blockDim.x + threadIdx.x; t < Ty; t += gridDim.x * blockDim.x) {
    const float v = z[(size_t)bc * T + t] * stdv[c];
    mel[(size_t)bc * Ty + t] = v + mean[c];
  }
}

int denorm_crop(const float* z, const float* mean, const float* stdv, int B, int C, int T, int Ty,
                float* mel, hipStream_t st) {
  MT_REQUIRE(Ty <= T && Ty > 0, "denorm_crop: Ty %d > T %d", Ty, T);
  dim3 grid(std::min((Ty + 255) / 256, 64), B * C);
  hipLaunchKernelGGL(denorm_crop_kernel, grid, dim3(256), 0, st, z, mean, stdv, C, T, Ty, mel);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// ------------------------------------------------------------------------------------
// row copy / row mask (text encoder: speaker-channel concat model.py:526-527, x * x_mask)
// ------------------------------------------------------------------------------------
template <class E>
__global__ void copy_rows_kernel(const E* __restrict__ src, int lds, int rows, int C, E* __restrict__ dst, int ldd) {
  const size_t total = (size_t)rows * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / C, c = i - r * C;
    dst[r * ldd + c] = src[r * lds + c];
  }
}
template <class E>
__global__ void mask_rows_kernel(E* __restrict__ x, int rows, int C, const float* __restrict__ m) {
  const size_t total = (size_t)rows * C;
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const size_t r = i / C;
    x[i] = from_f<E>(to_f(x[i]) * m[r]);
  }
}
int copy_rows(int dtype, const void* src, int ld_src, int rows, int C, void* dst, int ld_dst, hipStream_t st) {
  const size_t total = (size_t)rows * C;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  if (dtype == BF16)
    hipLaunchKernelGGL(copy_rows_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (const bf16*)src, ld_src, rows, C,
                       (bf16*)dst, ld_dst);
  else
    hipLaunchKernelGGL(copy_rows_kernel<float>, dim3(blocks), dim3(256), 0, st, (const float*)src, ld_src, rows, C,
                       (float*)dst, ld_dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}
int mask_rows(int dtype, void* x, int rows, int C, const float* mask, hipStream_t st) {
  const size_t total = (size_t)rows * C;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  if (dtype == BF16)
    hipLaunchKernelGGL(mask_rows_kernel<bf16>, dim3(blocks), dim3(256), 0, st, (bf16*)x, rows, C, mask);
  else
    hipLaunchKernelGGL(mask_rows_kernel<float>, dim3(blocks), dim3(256), 0, st, (float*)x, rows, C, mask);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// one block = GN_FR frames of one utterance; C/8 threads x 8 channels (16 B) per frame row
constexpr int GN_FR = 32;
__global__ __launch_bounds__(256) void gn_apply_kernel(const bf16* __restrict__ y, int T, int C,
                                                       const double* __restrict__ part, int nparts,
                                                       const float* __restrict__ gamma, const float* __restrict__ beta,
                                                       float eps, const float* __restrict__ tb, int tb_ld,
                                                       const float* __restrict__ mask, bf16* __restrict__ h, int xr) {
  __shared__ float ga[256], gs[256], gm[8], gr[8];
  const int tid = threadIdx.x;
  // (frame block, utterance), XCD-aligned (mt_common.h xcd_chunk)
  const int ci = xcd_chunk(blockIdx.x + gridDim.x * blockIdx.y, gridDim.x * gridDim.y, xr);
  const int b = ci / gridDim.x, bx = ci % gridDim.x;
  const int G = C >> 5;
  const int cpr = C >> 3;  // 16-byte groups per row
  const int rows_per = 256 / cpr;
  const int q = tid % cpr, c = 8 * q;
  // this thread's rows are loaded first (independent of the GroupNorm coefficients), so their latency
  // overlaps the partial-sum merge below
  constexpr int NR = GN_FR / 8;  // rows per thread at C = 256 (fewer used at smaller C)
  u32x4 v[NR];
  float mk[NR];
  const int t0 = bx * GN_FR + tid / cpr;
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int t = min(t0 + j * rows_per, T - 1);
    const size_t row = (size_t)b * T + t;
    v[j] = *reinterpret_cast<const u32x4*>(y + row * C + c);
    mk[j] = mask[row];
  }
  float tbv[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) tbv[k] = tb ? tb[(size_t)b * tb_ld + c + k] : 0.f;
  if (tid < 64) {
    // first wave: 64 / G lanes per group each sum a strided subset of the group's partials (all loads in
    // flight at once), then a butterfly inside the lane segment
    const int lpg = 64 / G, g = tid / lpg, sub = tid % lpg;
    const double* p = part + (size_t)(b * G + g) * nparts * 2;
    double s1 = 0.0, s2 = 0.0;
    for (int i = sub; i < nparts; i += lpg) {
      s1 += p[2 * i];
      s2 += p[2 * i + 1];
    }
    for (int o = lpg >> 1; o > 0; o >>= 1) {
      s1 += __shfl_xor(s1, o, 64);
      s2 += __shfl_xor(s2, o, 64);
    }
    if (sub == 0) {
      const double n = 32.0 * (double)T;
      const double mean = s1 / n;
      double var = s2 / n - mean * mean;
      var = var < 0.0 ? 0.0 : var;
      gm[g] = (float)mean;
      gr[g] = (float)(1.0 / sqrt(var + (double)eps));
    }
  }
  __syncthreads();
  for (int cc = tid; cc < C; cc += 256) {
    const float sc = gr[cc >> 5] * gamma[cc];
    ga[cc] = sc;
    gs[cc] = -sc * gm[cc >> 5] + beta[cc];
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NR; ++j) {
    const int t = t0 + j * rows_per;
    if (t >= T || t >= (bx + 1) * GN_FR) break;
    const size_t row = (size_t)b * T + t;
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const uint32_t w = v[j][e];
      const float x0 = __uint_as_float(w << 16), x1 = __uint_as_float(w & 0xffff0000u);
      const float r0 = (mish_f(x0 * ga[c + 2 * e] + gs[c + 2 * e]) + tbv[2 * e]) * mk[j];
      const float r1 = (mish_f(x1 * ga[c + 2 * e + 1] + gs[c + 2 * e + 1]) + tbv[2 * e + 1]) * mk[j];
      const bf16 h0 = (bf16)r0, h1 = (bf16)r1;
      o[e] = (uint32_t)__builtin_bit_cast(uint16_t, h0) | ((uint32_t)__builtin_bit_cast(uint16_t, h1) << 16);
    }
    *reinterpret_cast<u32x4*>(h + row * C + c) = o;
  }
}

int gn_apply(const void* y, int B, int T, int C, const double* part, int nparts, const float* gamma,
             const float* beta, float eps, const float* tb, int tb_ld, const float* mask, void* h, hipStream_t st) {
  MT_REQUIRE(C % 32 == 0 && C <= 256 && C >= 64 && 256 % (C / 8) == 0 && nparts > 0, "gn_apply: C %d", C);
  hipLaunchKernelGGL(gn_apply_kernel, dim3((T + GN_FR - 1) / GN_FR, B), dim3(256), 0, st, (const bf16*)y, T, C, part, nparts,
                     gamma, beta, eps, tb, tb_ld, mask, (bf16*)h, xcd_remap_for((size_t)B * T * C * sizeof(bf16)));
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
