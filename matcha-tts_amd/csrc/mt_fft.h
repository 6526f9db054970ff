// 1024-point radix-2 FFT in LDS and the periodic Hann window (torch.hann_window(1024)), shared by the
// denoiser (hifigan/denoiser.py) and the log-mel featurizer (train_standalone.py:164-201).
#pragma once
#include "mt_common.h"

namespace mt {

__device__ __forceinline__ float hann(int n) {
  const float s = sinpif((float)n / 1024.f);
  return s * s;
}

// in-place iterative radix-2 on bit-reversed input (re, im: 1024 floats in LDS); twiddles
// twc/tws[k] = cos/sin(2 pi k / 1024); sign -1 forward, +1 inverse (unscaled). Every thread of the
// workgroup must call it.
__device__ __forceinline__ void fft1024(float* re, float* im, const float* twc, const float* tws, float sign) {
  constexpr int N = 1024;
  for (int h = 1; h < N; h <<= 1) {
    __syncthreads();
    for (int bfly = threadIdx.x; bfly < N / 2; bfly += blockDim.x) {
      const int j = bfly % h;
      const int base = (bfly / h) * 2 * h + j;
      const int tw = j * (N / (2 * h));
      const float c = twc[tw], s = sign * tws[tw];
      const float ar = re[base], ai = im[base];
      const float br = re[base + h], bi = im[base + h];
      const float tr = br * c - bi * s, ti = br * s + bi * c;
      re[base] = ar + tr;
      im[base] = ai + ti;
      re[base + h] = ar - tr;
      im[base + h] = ai - ti;
    }
  }
  __syncthreads();
}

}  // namespace mt
