// Log-mel featurizer of the training data path (§8f rank 4): train_standalone.py:164-201
// `mel_spectrogram` (same as hifigan/meldataset.py:52-89) followed by `normalize` (:204-210), on gfx950.
//
//   y   = reflect_pad(audio, (n_fft - hop) / 2 = 384 each side)
//   S   = stft(y, n_fft 1024, hop 256, win 1024 Hann (periodic), center=False, onesided)
//   mag = sqrt(re^2 + im^2 + 1e-9)
//   mel = log(clamp(mel_basis[80][513] . mag, 1e-5)),   out = (mel - mean) / std
//
// One 256-thread workgroup per (utterance, frame): the windowed reflect-padded frame goes bit-reversed
// into LDS, a radix-2 1024-point complex FFT runs in place (twiddles from sincospif, the denoiser's
// fft1024), the 513 one-sided magnitudes stay in LDS and each of the 80 filters is a 513-long dot product
// split over 3 lanes. Output [B][80][F] fp32, F = (L - 256) / 256 + 1 frames (torch's framing).
#include <math.h>

#include "mt_fft.h"

namespace mt {

namespace {
constexpr int NFFT = 1024, HOP = 256, NBIN = NFFT / 2 + 1, PAD = (NFFT - HOP) / 2, NMEL = 80;
}

__global__ __launch_bounds__(256) void logmel_kernel(const float* __restrict__ audio, int L, int nfr,
                                                     const float* __restrict__ basis, float mean, float stdv,
                                                     float* __restrict__ out) {
  __shared__ float re[NFFT], im[NFFT], twc[NFFT / 2], tws[NFFT / 2], mag[NBIN], part[3][NMEL];
  const int f = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
  const float* x = audio + (size_t)b * L;
  for (int k = tid; k < NFFT / 2; k += 256) {
    float s, c;
    sincospif(2.f * (float)k / (float)NFFT, &s, &c);
    twc[k] = c;
    tws[k] = s;
  }
  for (int n = tid; n < NFFT; n += 256) {
    int i = f * HOP + n - PAD;  // index into the unpadded audio, reflected at both ends
    if (i < 0) i = -i;
    if (i >= L) i = 2 * (L - 1) - i;
    const int r = __brev((unsigned)n) >> (32 - 10);
    re[r] = x[i] * hann(n);
    im[r] = 0.f;
  }
  fft1024(re, im, twc, tws, -1.f);
  for (int k = tid; k < NBIN; k += 256) mag[k] = sqrtf(re[k] * re[k] + im[k] * im[k] + 1e-9f);
  __syncthreads();
  if (tid < 3 * NMEL) {  // filter m = tid % 80, bins of third tid / 80
    const int m = tid % NMEL, third = tid / NMEL;
    const int k0 = third * 171, k1 = min(NBIN, k0 + 171);
    const float* w = basis + (size_t)m * NBIN;
    float s = 0.f;
    for (int k = k0; k < k1; ++k) s = fmaf(w[k], mag[k], s);
    part[third][m] = s;
  }
  __syncthreads();
  if (tid < NMEL) {
    const float s = (part[0][tid] + part[1][tid]) + part[2][tid];
    out[((size_t)b * NMEL + tid) * nfr + f] = (logf(fmaxf(s, 1e-5f)) - mean) / stdv;
  }
}

int log_mel(const float* audio, int B, int L, const float* basis, float mean, float stdv, float* mel, hipStream_t st) {
  MT_REQUIRE(B > 0 && L >= NFFT - 2 * PAD && L > PAD, "log_mel: need at least %d samples (reflect padding %d)",
             NFFT - 2 * PAD, PAD);
  MT_REQUIRE(stdv != 0.f, "log_mel: std must be non-zero");
  const int nfr = (L + 2 * PAD - NFFT) / HOP + 1;
  hipLaunchKernelGGL(logmel_kernel, dim3(nfr, B), dim3(256), 0, st, audio, L, nfr, basis, mean, stdv, mel);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
