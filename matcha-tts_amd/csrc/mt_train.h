// Training-step primitives (fp32) — see mt_train.hip.
#pragma once
#include <stddef.h>

#include "mt_common.h"

namespace mt {

struct GemmF32 {  // C[z] = alpha op(A[z]) op(B[z]) + beta C[z]; op(A) is M x K, op(B) K x N, C row-major
  int transA, transB, M, N, K;
  float alpha, beta;
  const float* A;
  int lda;
  long long sA;
  const float* B;
  int ldb;
  long long sB;
  float* C;
  int ldc;
  long long sC;
  int batch;
  const float* bias;   // optional, per output column: C += bias[n] (after alpha / beta)
  const float* rmask;  // optional, per output row of each batch [batch][M]: C *= rmask[m] (last)
  float* ws;           // split-K partials (gemm_f32_workspace_floats); NULL: no split
  size_t ws_floats;
  int opfmt;  // operands rounded to: 0 none (exact fp32 MFMA), 1 fp16, 2 bf16 (16-bit MFMA, fp32 accumulation)
};
size_t gemm_f32_workspace_floats(int M, int N, int K, int batch);
int gemm_f32(const GemmF32& g, hipStream_t st);

int im2col(const float* x, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
           float* cols, hipStream_t st);
int col2im(const float* dcols, const float* mask, int B, int T, int C, int k, int stride, int pad, int dil, int Tout,
           float* dx, int accumulate, hipStream_t st);

enum EwOp {
  EW_AXPBY = 0,     // alpha a + beta b
  EW_MUL = 1,       // alpha a b
  EW_MISH = 2,      // mish(a)
  EW_MISH_BWD = 3,  // c * mish'(a)
  EW_SILU = 4,
  EW_SILU_BWD = 5,  // c * silu'(a)
  EW_RELU = 6,
  EW_RELU_BWD = 7,  // c * [a > 0]
  EW_EXP = 8,
  EW_SQDIFF = 9,    // (a - b)^2
  EW_SIN = 10,
  EW_COS = 11,
  EW_LOG = 12,      // log(alpha + a)
  EW_RECIP = 13,    // alpha / a
};
struct EwArgs {  // out[i] (+)= op(a[i], b[bidx(i)], c[i]); bidx = ((i/d0)%m0)*s0 + ((i/d1)%m1)*s1
  int op;
  size_t n;
  const float* a;
  const float* b;
  const float* c;
  float* out;
  float alpha, beta;
  size_t d0, m0, s0, d1, m1, s1;
  int accumulate;
};
int ew(const EwArgs& e, hipStream_t st);

int copy_cols(const float* src, int lds, int soff, float* dst, int ldd, int doff, int rows, int n, int accumulate,
              hipStream_t st);
int seq_mask(const long long* lengths, int B, int T, float* out, hipStream_t st);

size_t colsum_scratch_floats(int rows, int C, int seg);
int colsum(const float* a, const float* b, int rows, int C, int seg, float* out, int accumulate, float* scratch,
           hipStream_t st);
int sum_all(const float* a, const float* b, size_t n, float* out, float* scratch, hipStream_t st);

int dropout(const float* a, size_t n, float p, unsigned seed, float* out, hipStream_t st);
int groupnorm_fwd(const float* x, const float* gamma, const float* beta, int B, int T, int C, int G, float eps,
                  float* y, float* mean, float* rstd, hipStream_t st);
int groupnorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int B,
                  int T, int C, int G, float* dx, float* dgp, float* dbp, hipStream_t st);
int layernorm_fwd(const float* x, const float* gamma, const float* beta, int rows, int C, float eps, float* y,
                  float* mean, float* rstd, hipStream_t st);
int layernorm_bwd(const float* dy, const float* x, const float* gamma, const float* mean, const float* rstd, int rows,
                  int C, float* dx, hipStream_t st);
int snake_fwd(const float* x, const float* la, const float* lb, size_t n, int C, float* y, hipStream_t st);
int snake_bwd(const float* x, const float* la, const float* lb, const float* dy, size_t n, int C, float* dx, float* ga,
              float* gb, hipStream_t st);
int softmax_fwd(const float* s, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk, float scale,
                int mode, float* p, hipStream_t st);
int softmax_bwd(const float* p, const float* dp, const float* kmask, const float* qmask, int BH, int H, int Tq, int Tk,
                float scale, float* ds, hipStream_t st);
int rope(float* x, int B, int T, int H, int dh, int d, const float* theta, int inverse, hipStream_t st);
int embed_fwd(const long long* ids, size_t ntok, const float* table, int C, float scale, float* out, hipStream_t st);
int embed_bwd(const long long* ids, size_t ntok, const float* dout, int V, int C, float scale, float* dtable,
              hipStream_t st);
int adam_step(float* p, const float* g, float* m, float* v, size_t n, const float* gscale, float lr, float b1,
              float b2, float eps, int step, hipStream_t st);
int clip_factor(const float* sumsq, float max_norm, float inv_world, float* out, float* norm_out, hipStream_t st);
int unscale_found_inf(float* g, size_t n, float inv_scale, float* found, float* scratch, hipStream_t st);

}  // namespace mt
