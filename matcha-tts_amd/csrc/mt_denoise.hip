// Denoiser (hifigan/denoiser.py:62-68) on gfx950.
//
//   S = stft(audio, n_fft=1024, hop=256, win=1024 Hann(periodic), center=True, reflect pad)
//   |S'| = clamp(|S| - strength * bias_spec, 0);  S' = |S'| * (cos angle(S), sin angle(S))
//   out = istft(S')  (window-squared envelope normalisation, center trimmed) -> [B, 256*(L/256)]
// Kernel 1 (stft_denoise2_kernel): one workgroup per (utterance, PAIR of frames). The two reflect-padded windowed
// real frames are the real and imaginary parts of one complex sequence, so one 1024-point FFT gives both spectra
// (X_a[k] = (Z[k] + conj Z[N-k]) / 2, X_b[k] = (Z[k] - conj Z[N-k]) / 2i); each one-sided spectrum is denoised,
// Hermitian-completed and packed back as Y_a + i Y_b, so one inverse FFT returns both frames (real and imaginary
// part). The FFTs are radix-4 Stockham in LDS (5 passes of one radix-4 butterfly per thread, natural order in
// and out, twiddles from an LDS table). The denoise keeps the phase by scaling: S' = S * max(|S| - b s, 0) / |S|
// (= |S'| (cos angle S, sin angle S) of denoiser.py:64-67 without atan2 / cos / sin).
// Kernel 2: overlap-add of the <= 4 frames covering each output sample / window envelope.
// stft_denoise_kernel (one frame per workgroup, radix-2) remains for the bias spectrum (stft_magnitude).
#include <math.h>

#include "mt_fft.h"

namespace mt {

static constexpr int NFFT = 1024, HOP = 256, NBIN = NFFT / 2 + 1;

__global__ __launch_bounds__(256) void stft_denoise_kernel(const float* __restrict__ audio, int L, int nfr,
                                                           const float* __restrict__ bias, float strength,
                                                           float* __restrict__ frames,
                                                           float* __restrict__ mag_out) {
  __shared__ float re[NFFT], im[NFFT], twc[NFFT / 2], tws[NFFT / 2];
  const int f = blockIdx.x, b = blockIdx.y;
  const float* x = audio + (size_t)b * L;
  for (int k = threadIdx.x; k < NFFT / 2; k += blockDim.x) {
    float s, c;
    sincospif(2.f * (float)k / (float)NFFT, &s, &c);
    twc[k] = c;
    tws[k] = s;
  }
  for (int n = threadIdx.x; n < NFFT; n += blockDim.x) {
    int i = f * HOP + n - NFFT / 2;  // reflect padding by n_fft/2 on both sides
    if (i < 0) i = -i;
    if (i >= L) i = 2 * (L - 1) - i;
    const int r = __brev((unsigned)n) >> (32 - 10);
    re[r] = x[i] * hann(n);
    im[r] = 0.f;
  }
  fft1024(re, im, twc, tws, -1.f);
  if (mag_out) {  // |STFT| of this frame only (Denoiser bias spectrum, denoiser.py:57-60)
    for (int k = threadIdx.x; k < NBIN; k += blockDim.x)
      mag_out[((size_t)b * nfr + f) * NBIN + k] = sqrtf(re[k] * re[k] + im[k] * im[k]);
    return;
  }
  // denoise one-sided bins; keep them in registers, then rebuild the Hermitian spectrum
  float nr[3], ni[3];
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int k = threadIdx.x + q * 256;
    nr[q] = ni[q] = 0.f;
    if (k < NBIN) {
      const float a = re[k], c = im[k];
      const float mag = sqrtf(a * a + c * c);
      const float ang = atan2f(c, a);
      const float m2 = fmaxf(mag - bias[k] * strength, 0.f);
      nr[q] = m2 * cosf(ang);
      ni[q] = m2 * sinf(ang);
    }
  }
  __syncthreads();
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int k = threadIdx.x + q * 256;
    if (k >= NBIN) continue;
    // irfft ignores the imaginary part of the DC and Nyquist bins
    const float i0 = (k == 0 || k == NFFT / 2) ? 0.f : ni[q];
    const int r = __brev((unsigned)k) >> (32 - 10);
    re[r] = nr[q];
    im[r] = i0;
    if (k > 0 && k < NFFT / 2) {
      const int r2 = __brev((unsigned)(NFFT - k)) >> (32 - 10);
      re[r2] = nr[q];
      im[r2] = -i0;
    }
  }
  fft1024(re, im, twc, tws, 1.f);
  float* out = frames + ((size_t)b * nfr + f) * NFFT;
  for (int n = threadIdx.x; n < NFFT; n += blockDim.x) out[n] = re[n] * (1.f / NFFT) * hann(n);
}

__device__ __forceinline__ float2 cmulf(float2 a, float2 b) { return float2{a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x}; }

// Stockham radix-4 FFT of 1024 complex points (src, scratch: LDS float2[1024]); tw[t] = (cos, sin)(2 pi t / 1024),
// t < 768; sign -1 forward, +1 inverse (unscaled). 256 threads, all of them call it. Returns the buffer holding
// the result (src or scratch).
__device__ __forceinline__ float2* fft1024_r4(float2* src, float2* scr, const float2* tw, float sign) {
  const int j = threadIdx.x;
#pragma unroll
  for (int Ns = 1; Ns < NFFT; Ns <<= 2) {
    __syncthreads();
    const int k = j & (Ns - 1), step = (NFFT / 4) / Ns;
    float2 v[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) v[r] = src[j + r * (NFFT / 4)];
#pragma unroll
    for (int r = 1; r < 4; ++r) {
      const float2 w = tw[k * step * r];
      v[r] = cmulf(v[r], float2{w.x, sign * w.y});
    }
    // radix-4 DFT, exp(sign i 2 pi r q / 4): q = 1 multiplies v1 by (sign i), v3 by (-sign i)
    const float2 a0 = float2{v[0].x + v[2].x, v[0].y + v[2].y}, a1 = float2{v[0].x - v[2].x, v[0].y - v[2].y};
    const float2 b0 = float2{v[1].x + v[3].x, v[1].y + v[3].y}, b1 = float2{v[1].x - v[3].x, v[1].y - v[3].y};
    const float2 jb1 = float2{-sign * b1.y, sign * b1.x};  // (sign i) * b1
    const int d = (j / Ns) * Ns * 4 + k;
    scr[d] = float2{a0.x + b0.x, a0.y + b0.y};
    scr[d + Ns] = float2{a1.x + jb1.x, a1.y + jb1.y};
    scr[d + 2 * Ns] = float2{a0.x - b0.x, a0.y - b0.y};
    scr[d + 3 * Ns] = float2{a1.x - jb1.x, a1.y - jb1.y};
    float2* t = src;
    src = scr;
    scr = t;
  }
  __syncthreads();
  return src;
}

// ragged batch (lens != null): row b is an utterance of Lb = lens[b] * lmul samples (its own reflect padding and
// 1 + Lb / 256 frames; the rest of the row is not read), as the reference denoises one utterance per call
__global__ __launch_bounds__(256) void stft_denoise2_kernel(const float* __restrict__ audio, int L, int nfr,
                                                            const float* __restrict__ bias, float strength,
                                                            float* __restrict__ frames, const int* lens, int lmul) {
  __shared__ float2 bufA[NFFT], bufB[NFFT], tw[3 * NFFT / 4];
  const int f0 = 2 * blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const float* x = audio + (size_t)b * L;
  const int Lb = lens ? min(max(lens[b] * lmul, 0), L) : L;
  const int nfb = lens ? (Lb > 0 ? 1 + Lb / HOP : 0) : nfr;
  if (f0 >= nfb) return;
  const bool two = f0 + 1 < nfb;
  for (int t = tid; t < 3 * NFFT / 4; t += 256) {
    float sn, cs;
    sincospif(2.f * (float)t / (float)NFFT, &sn, &cs);
    tw[t] = float2{cs, sn};
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = tid + 256 * q;
    const float w = hann(n);
    float v[2];
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      int i = (f0 + u) * HOP + n - NFFT / 2;  // reflect padding by n_fft/2 on both sides
      if (i < 0) i = -i;
      if (i >= Lb) i = 2 * (Lb - 1) - i;
      i = min(max(i, 0), Lb - 1);  // an utterance shorter than n_fft / 2 (torch's reflect pad raises there)
      v[u] = (u == 0 || two) ? x[i] * w : 0.f;
    }
    bufA[n] = float2{v[0], v[1]};
  }
  float2* Z = fft1024_r4(bufA, bufB, tw, -1.f);
  float2* W = Z == bufA ? bufB : bufA;
  // both one-sided spectra, denoised, Hermitian-completed and packed as Y_a + i Y_b
#pragma unroll
  for (int q = 0; q < 3; ++q) {
    const int k = tid + 256 * q;
    if (k > NFFT / 2) continue;
    const float2 zk = Z[k], zn = Z[(NFFT - k) & (NFFT - 1)];
    float2 xa = float2{0.5f * (zk.x + zn.x), 0.5f * (zk.y - zn.y)};
    float2 xb = float2{0.5f * (zk.y + zn.y), -0.5f * (zk.x - zn.x)};
    const float bs = bias[k] * strength;
    auto den = [&](float2& s) {
      const float mag = sqrtf(s.x * s.x + s.y * s.y);
      const float g = mag > 0.f ? fmaxf(mag - bs, 0.f) / mag : 0.f;
      s = float2{s.x * g, s.y * g};
    };
    den(xa);
    den(xb);
    if (k == 0 || k == NFFT / 2) {  // irfft ignores the imaginary part of the DC and Nyquist bins
      xa.y = 0.f;
      xb.y = 0.f;
    }
    W[k] = float2{xa.x - xb.y, xa.y + xb.x};  // Y_a[k] + i Y_b[k]
    if (k > 0 && k < NFFT / 2) W[NFFT - k] = float2{xa.x + xb.y, -xa.y + xb.x};  // conj(Y_a[k]) + i conj(Y_b[k])
  }
  float2* y = fft1024_r4(W, Z, tw, 1.f);
  float* outa = frames + ((size_t)b * nfr + f0) * NFFT;
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int n = tid + 256 * q;
    const float w = hann(n) * (1.f / NFFT);
    const float2 v = y[n];
    outa[n] = v.x * w;
    if (two) outa[NFFT + n] = v.y * w;
  }
}

__global__ void overlap_add_kernel(const float* __restrict__ frames, int nfr, int Lout,
                                   float* __restrict__ out, const int* lens, int lmul, int L) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Lout) return;
  int nfb = nfr;
  if (lens) {  // ragged: this utterance's frames; its output ends at 256 (frames - 1) samples, zeros after
    const int Lb = min(max(lens[b] * lmul, 0), L);
    nfb = Lb > 0 ? 1 + Lb / HOP : 0;
    if (i >= HOP * (nfb - 1)) {
      out[(size_t)b * Lout + i] = 0.f;
      return;
    }
  }
  const int p = i + NFFT / 2;
  int f0 = (p - NFFT + HOP) / HOP;
  if (f0 < 0) f0 = 0;
  int f1 = p / HOP;
  if (f1 > nfb - 1) f1 = nfb - 1;
  float s = 0.f, env = 0.f;
  for (int f = f0; f <= f1; ++f) {
    const int n = p - f * HOP;
    if (n < 0 || n >= NFFT) continue;
    s += frames[((size_t)b * nfr + f) * NFFT + n];
    const float w = hann(n);
    env += w * w;
  }
  out[(size_t)b * Lout + i] = s / env;
}

size_t denoise_workspace_bytes(int B, int L) {
  const int nfr = 1 + L / HOP;
  return (size_t)B * nfr * NFFT * sizeof(float);
}

int denoise(const float* audio, int B, int L, const float* bias_spec, float strength, float* out, void* ws,
            size_t ws_bytes, hipStream_t st, const int* lens, int lmul) {
  MT_REQUIRE(B > 0 && L > NFFT / 2, "denoise: need L > %d samples (reflect padding)", NFFT / 2);
  MT_REQUIRE(ws && ws_bytes >= denoise_workspace_bytes(B, L), "denoise: workspace too small");
  const int nfr = 1 + L / HOP;
  const int Lout = HOP * (nfr - 1);
  MT_REQUIRE(!lens || lmul > 0, "denoise: length multiplier %d", lmul);
  hipLaunchKernelGGL(stft_denoise2_kernel, dim3((nfr + 1) / 2, B), dim3(256), 0, st, audio, L, nfr, bias_spec,
                     strength, (float*)ws, lens, lmul);
  MT_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(overlap_add_kernel, dim3((Lout + 255) / 256, B), dim3(256), 0, st, (const float*)ws, nfr,
                     Lout, out, lens, lmul, L);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

int stft_magnitude(const float* audio, int B, int L, float* mag, hipStream_t st) {
  MT_REQUIRE(B > 0 && L > NFFT / 2, "stft: need L > %d samples (reflect padding)", NFFT / 2);
  const int nfr = 1 + L / HOP;
  hipLaunchKernelGGL(stft_denoise_kernel, dim3(nfr, B), dim3(256), 0, st, audio, L, nfr, (const float*)nullptr,
                     0.f, (float*)nullptr, mag);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
