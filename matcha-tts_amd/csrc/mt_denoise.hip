// Denoiser (hifigan/denoiser.py:62-68) on gfx950.
//
//   S = stft(audio, n_fft=1024, hop=256, win=1024 Hann(periodic), center=True, reflect pad)
//   |S'| = clamp(|S| - strength * bias_spec, 0);  S' = |S'| * (cos angle(S), sin angle(S))
//   out = istft(S')  (window-squared envelope normalisation, center trimmed) -> [B, 256*(L/256)]
// Kernel 1: one workgroup per (utterance, frame): reflect-padded windowed frame -> 1024-point
// complex FFT in LDS (radix-2, twiddles from sincospif) -> denoise the 513 one-sided bins ->
// Hermitian-completed inverse FFT -> windowed frame written to the workspace.
// Kernel 2: overlap-add of the <= 4 frames covering each output sample / window envelope.
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

__global__ void overlap_add_kernel(const float* __restrict__ frames, int nfr, int Lout,
                                   float* __restrict__ out) {
  const int b = blockIdx.y;
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= Lout) return;
  const int p = i + NFFT / 2;
  int f0 = (p - NFFT + HOP) / HOP;
  if (f0 < 0) f0 = 0;
  int f1 = p / HOP;
  if (f1 > nfr - 1) f1 = nfr - 1;
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
            size_t ws_bytes, hipStream_t st) {
  MT_REQUIRE(B > 0 && L > NFFT / 2, "denoise: need L > %d samples (reflect padding)", NFFT / 2);
  MT_REQUIRE(ws && ws_bytes >= denoise_workspace_bytes(B, L), "denoise: workspace too small");
  const int nfr = 1 + L / HOP;
  const int Lout = HOP * (nfr - 1);
  hipLaunchKernelGGL(stft_denoise_kernel, dim3(nfr, B), dim3(256), 0, st, audio, L, nfr, bias_spec, strength,
                     (float*)ws, (float*)nullptr);
  MT_CHECK_HIP(hipGetLastError());
  hipLaunchKernelGGL(overlap_add_kernel, dim3((Lout + 255) / 256, B), dim3(256), 0, st, (const float*)ws, nfr,
                     Lout, out);
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
