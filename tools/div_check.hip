// Exhaustive check of mt_common.h div_rn (v * rd with one FMA correction, rd = RN(1 / d)) against the IEEE quotient
// v / d the compiler emits, for every fp32 v (all 2^32 bit patterns: finite values bit for bit, +-inf bit for bit, NaN
// must stay a NaN) and d = 1..8, on the GPU itself. Prints the mismatch count per divisor; 0 everywhere means the
// ResBlock average's division can use it with bit-identical results. Build: hipcc --offload-arch=gfx950 -O3 -Imatcha-tts_amd/csrc tools/div_check.hip
//   -o tools/div_check  (the vocoder kernels' flags: add -mno-amdgpu-ieee -fno-honor-nans)
#include <hip/hip_runtime.h>
#include <stdio.h>

#include "mt_common.h"

__global__ void div_check_kernel(float d, float rd, unsigned long long* bad, unsigned int* first) {
  unsigned long long nbad = 0;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < (1ull << 32); i += stride) {
    const float v = __uint_as_float((unsigned int)i);
    const float a = v / d;
    const float b = mt::div_rn(v, d, rd);
    const bool same = __builtin_isnan(v) ? __builtin_isnan(b) : __float_as_uint(a) == __float_as_uint(b);
    if (!same) {
      ++nbad;
      atomicMin(first, (unsigned int)i);
    }
  }
  if (nbad) atomicAdd(bad, nbad);
}

int main() {
  unsigned long long* bad;
  unsigned int* first;
  if (hipMalloc(&bad, 8) != hipSuccess || hipMalloc(&first, 4) != hipSuccess) return 2;
  int total = 0;
  for (int di = 1; di <= 8; ++di) {
    const float d = (float)di;
    volatile float one = 1.f;
    const float rd = one / d;
    unsigned long long h = 0;
    unsigned int f = 0xffffffffu;
    hipMemcpy(bad, &h, 8, hipMemcpyHostToDevice);
    hipMemcpy(first, &f, 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(div_check_kernel, dim3(4096), dim3(256), 0, 0, d, rd, bad, first);
    if (hipDeviceSynchronize() != hipSuccess) return 3;
    hipMemcpy(&h, bad, 8, hipMemcpyDeviceToHost);
    hipMemcpy(&f, first, 4, hipMemcpyDeviceToHost);
    printf("d = %d: %llu mismatches over all fp32 v (NaN: stays NaN)%s", di, h, h ? "" : "\n");
    if (h) printf(" (first bit pattern 0x%08x)\n", f);
    total += h != 0;
  }
  hipFree(bad);
  hipFree(first);
  return total ? 1 : 0;
}
