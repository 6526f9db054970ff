// Monotonic Alignment Search for CFM training (§8f rank 3): the reference's `maximum_path`
// (train_standalone.py:241-325, run there as a CPU numba / Python loop after a device->host copy).
//
// Reference recurrence (NOT the textbook diagonal-predecessor MAS), per utterance with t_x tokens and
// t_y frames, cells (x, y) with max(0, t_x + y - t_y) <= x < min(t_x, y + 1) visited column by
// column, x ascending; unvisited cells hold 0:
//   path[x, y] = v_prev + value[x, y],
//   v_prev = x == 0 ? (y == 0 ? 0 : path[0, y-1])
//                   : (y == 0 ? path[x-1, 0] : max(path[x-1, y], path[x, y-1]))
// so path[x, y] depends on (x-1, y) and (x, y-1): both on anti-diagonal d-1 (d = x + y). One workgroup
// per utterance walks the t_x + t_y - 1 anti-diagonals, one thread per token x, the two live
// diagonals in LDS; every cell's value is the same float32 max-then-add as the reference, so the
// table is bit-identical. The table is kept diagonal-major in HBM for the backtrack:
//   index = t_x - 1; for y = t_y-1 .. 0: out[index, y] = 1; if index > 0 and
//   path[index-1, y-1] > path[index, y-1]: index -= 1
// (at y = 0 the reference compares the already-rewritten last column; the decrement is then unused).
#include "mt_common.h"

namespace mt {

constexpr int MAS_MAXX = 1024;  // tokens per utterance served (threads x per-thread tokens)

__global__ __launch_bounds__(256) void mas_kernel(const float* __restrict__ value, const int* __restrict__ t_xs,
                                                  const int* __restrict__ t_ys, int Tx, int Ty,
                                                  float* __restrict__ diag, float* __restrict__ out) {
  __shared__ float D[2][MAS_MAXX];
  constexpr int XPT = MAS_MAXX / 256;  // tokens per thread
  const int b = blockIdx.x, tid = threadIdx.x;
  // lengths come from mask sums: clamp to the table so a non-binary / oversized mask cannot write
  // outside this utterance's path, diagonal and output rows
  const int tx = min(t_xs[b], Tx), ty = min(t_ys[b], Ty);
  const float* v = value + (size_t)b * Tx * Ty;
  float* dg = diag + (size_t)b * (Tx + Ty) * Tx;  // [d][x]
  float* o = out + (size_t)b * Tx * Ty;
  if (tx <= 0 || ty <= 0) return;
  for (int i = tid; i < MAS_MAXX; i += 256) D[1][i] = 0.f;  // diagonal -1: nothing visited
  __syncthreads();
  const int nd = tx + ty - 1;
  for (int d = 0; d < nd; ++d) {
    const float* prev = D[(d + 1) & 1];
    float* cur = D[d & 1];
#pragma unroll
    for (int k = 0; k < XPT; ++k) {
      const int x = tid + 256 * k;
      if (x >= tx) break;
      const int y = d - x;
      float p = 0.f;
      const bool vis = y >= 0 && y < ty && x >= max(0, tx + y - ty) && x < min(tx, y + 1);
      if (vis) {
        float vp;
        if (x == 0) vp = y == 0 ? 0.f : prev[0];                 // path[0, y-1]
        else if (y == 0) vp = prev[x - 1];                        // path[x-1, 0]
        else vp = fmaxf(prev[x - 1], prev[x]);                    // max(path[x-1, y], path[x, y-1])
        p = vp + v[(size_t)x * Ty + y];
      }
      cur[x] = p;
      dg[(size_t)d * Tx + x] = p;
    }
    __syncthreads();
  }
  if (tid != 0) return;
  // backtrack (one lane; the diagonal table is this workgroup's own writes)
  int index = tx - 1;
  for (int y = ty - 1; y >= 0; --y) {
    o[(size_t)index * Ty + y] = 1.f;
    if (y > 0 && index > 0) {
      const float a = dg[(size_t)(index - 1 + y - 1) * Tx + index - 1];  // path[index-1, y-1]
      const float c = dg[(size_t)(index + y - 1) * Tx + index];          // path[index, y-1]
      if (a > c) --index;
    }
  }
}

size_t mas_workspace_bytes(int B, int Tx, int Ty) { return (size_t)B * (Tx + Ty) * Tx * sizeof(float); }

int maximum_path(const float* value, const int* t_xs, const int* t_ys, int B, int Tx, int Ty, float* out,
                 void* ws, size_t ws_bytes, hipStream_t st) {
  MT_REQUIRE(B > 0 && Tx > 0 && Ty > 0, "maximum_path: empty input");
  MT_REQUIRE(Tx <= MAS_MAXX, "maximum_path: %d tokens > %d", Tx, MAS_MAXX);
  MT_REQUIRE(ws && ws_bytes >= mas_workspace_bytes(B, Tx, Ty), "maximum_path: workspace too small");
  MT_CHECK_HIP(hipMemsetAsync(out, 0, (size_t)B * Tx * Ty * sizeof(float), st));
  hipLaunchKernelGGL(mas_kernel, dim3(B), dim3(256), 0, st, value, t_xs, t_ys, Tx, Ty, (float*)ws, out);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
