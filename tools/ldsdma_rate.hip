// LDS-DMA fill-rate microbenchmark (no compute): per-CU bytes/s of global_load_lds_dwordx4 versus the number of
// issuing waves per workgroup (one workgroup per CU) and the DMA instructions each wave keeps in flight, from an
// L2-resident window and from an HBM-streamed one. Question it answers: is mt_vconv's ≈ 40 GB/s per CU
// fill in the decoder's K loops a per-CU ceiling of the DMA path, or an issue-parallelism limit of its loader waves?
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ldsdma_rate tools/ldsdma_rate.hip
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

constexpr int LDS_BYTES = 128 * 1024;  // one workgroup per CU

template <int D>
__device__ __forceinline__ void wait_le() {
  // s_waitcnt vmcnt(D), expcnt / lgkmcnt left at their maxima (gfx9 encoding: vmcnt[3:0] | vmcnt[5:4] << 14)
  __builtin_amdgcn_s_waitcnt((D & 15) | ((D >> 4) << 14) | (7 << 4) | (15 << 8));
}

// every wave issues `iters` 1 KiB pieces: piece i of wave w of workgroup g reads window offset
// ((g * W + w) * iters + i) * 1 KiB mod window (a power of two), into LDS slot (w * 8 + i % 8) mod 128 (1 KiB slots)
template <int D>
__global__ void __launch_bounds__(1024) fill_kernel(const char* src, size_t window, int iters, int W) {
  extern __shared__ __attribute__((aligned(16))) char lds[];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  if (wave >= W) return;
  size_t base = ((size_t)blockIdx.x * W + wave) * (size_t)iters * 1024;
  for (int i = 0; i < iters; ++i) {
    const size_t off = (base + (size_t)i * 1024) & (window - 1);  // window: a power of two
    char* slot = lds + (((wave * 8 + (i & 7)) & 127) << 10);
    __builtin_amdgcn_global_load_lds(src + off + lane * 16,
                                     (__attribute__((address_space(3))) void*)slot, 16, 0, 0);
    wait_le<D>();
  }
  wait_le<0>();
}

template <int D>
float run(const char* src, size_t window, int grid, int W, int iters) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  hipLaunchKernelGGL(fill_kernel<D>, dim3(grid), dim3(64 * W), LDS_BYTES, 0, src, window, iters, W);  // warm
  CK(hipEventRecord(a));
  hipLaunchKernelGGL(fill_kernel<D>, dim3(grid), dim3(64 * W), LDS_BYTES, 0, src, window, iters, W);
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  CK(hipGetLastError());
  CK(hipEventDestroy(a)); CK(hipEventDestroy(b));
  return ms;
}

int main() {
  int cus = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));
  CK(hipFuncSetAttribute((const void*)fill_kernel<2>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)fill_kernel<4>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)fill_kernel<8>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)fill_kernel<16>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  CK(hipFuncSetAttribute((const void*)fill_kernel<32>, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
  const size_t big = (size_t)2 << 30;
  char* src; CK(hipMalloc(&src, big + 4096));
  CK(hipMemset(src, 1, big + 4096));
  const int grid = cus;
  printf("CUs %d, grid %d (1 WG/CU), 1 KiB per DMA wave-instruction\n", cus, grid);
  printf("%-8s %3s %3s %10s %12s %12s\n", "window", "W", "D", "ms", "GB/s/CU", "TB/s chip");
  const size_t wins[2] = {(size_t)2 << 20, big};
  const char* wname[2] = {"2MiB", "2GiB"};
  for (int wi = 0; wi < 2; ++wi) {
    for (int W : {1, 2, 4, 8, 16}) {
      // 512 MiB per launch from the L2 window, the whole 2 GiB (once) for the HBM one
      const size_t tot = wi == 0 ? ((size_t)512 << 20) : big;
      const int iters = (int)(tot / 1024 / grid / W);
      for (int D : {2, 4, 8, 16, 32}) {
        float ms = 0;
        switch (D) {
          case 2: ms = run<2>(src, wins[wi], grid, W, iters); break;
          case 4: ms = run<4>(src, wins[wi], grid, W, iters); break;
          case 8: ms = run<8>(src, wins[wi], grid, W, iters); break;
          case 16: ms = run<16>(src, wins[wi], grid, W, iters); break;
          default: ms = run<32>(src, wins[wi], grid, W, iters); break;
        }
        const double bytes = (double)iters * 1024 * W * grid;
        printf("%-8s %3d %3d %10.3f %12.1f %12.2f\n", wname[wi], W, D, ms, bytes / grid / (ms * 1e6),
               bytes / (ms * 1e9));
      }
    }
  }
  CK(hipFree(src));
  return 0;
}
