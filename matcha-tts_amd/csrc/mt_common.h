// Common device/host definitions for the MI355X (gfx950) Matcha-TTS synthesis path.
//
// Activation layout in HBM is frame-major, channel-contiguous: [B][T][C]. A Conv1d
// over that layout is an implicit GEMM with K = taps x C_in contiguous per tap, which
// feeds MFMA fragments with 16-byte loads (DESIGN.md "Data layout").
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mt {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) __bf16 bf16x4;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

typedef __bf16 bf16;

enum DType { F32 = 0, BF16 = 1 };

// ---------------------------------------------------------------------------
// element conversions
// ---------------------------------------------------------------------------
__device__ __forceinline__ float to_f(float x) { return x; }
__device__ __forceinline__ float to_f(bf16 x) { return (float)x; }
template <class T> __device__ __forceinline__ T from_f(float x);
template <> __device__ __forceinline__ float from_f<float>(float x) { return x; }
template <> __device__ __forceinline__ bf16 from_f<bf16>(float x) { return (bf16)x; }

// A 16-byte vector of T viewed as floats: bf16 -> 8 values, f32 -> 4 values.
template <class T> struct Vec16;
template <> struct Vec16<float> {
  static constexpr int N = 4;
  f32x4 v;
  __device__ __forceinline__ float get(int i) const { return v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = x; }
};
template <> struct Vec16<bf16> {
  static constexpr int N = 8;
  bf16x8 v;
  __device__ __forceinline__ float get(int i) const { return (float)v[i]; }
  __device__ __forceinline__ void set(int i, float x) { v[i] = (bf16)x; }
};

template <class T>
__device__ __forceinline__ Vec16<T> load16(const T* p) {
  Vec16<T> r;
  r.v = *reinterpret_cast<const decltype(r.v)*>(p);
  return r;
}
template <class T>
__device__ __forceinline__ void store16(T* p, const Vec16<T>& r) {
  *reinterpret_cast<decltype(r.v)*>(p) = r.v;
}
template <class T>
__device__ __forceinline__ Vec16<T> zero16() {
  Vec16<T> r;
#pragma unroll
  for (int i = 0; i < Vec16<T>::N; ++i) r.set(i, 0.f);
  return r;
}

// ---------------------------------------------------------------------------
// MFMA: one 16-byte fragment pair (A row-slab, B col-slab) of 64 bytes of K per row.
//   bf16: v_mfma_f32_16x16x32_bf16 — lane l holds A[l&15][8(l>>4)+j], B[8(l>>4)+j][l&15]
//   f32 : v_mfma_f32_16x16x4_f32 x4 — lane group g=l>>4 supplies k = 4g+s on step s, i.e.
//         the 16 channels of a 64-byte chunk are visited in the permuted order
//         {s, 4+s, 8+s, 12+s}; A and B use the same permutation so the sum is the same.
// C/D: col = l&15, row = 4(l>>4)+i (cdna_hip_programming.md §3).
// ---------------------------------------------------------------------------
__device__ __forceinline__ f32x4 mfma16(const bf16x8& a, const bf16x8& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mfma16(const f32x4& a, const f32x4& b, f32x4 c) {
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[0], b[0], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[1], b[1], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[2], b[2], c, 0, 0, 0);
  c = __builtin_amdgcn_mfma_f32_16x16x4f32(a[3], b[3], c, 0, 0, 0);
  return c;
}

// channels per 64-byte K chunk
template <class T> struct Chunk { static constexpr int CH = 64 / sizeof(T); };

// ---------------------------------------------------------------------------
// math helpers (reference semantics: torch.nn.Mish, F.leaky_relu, SiLU)
// ---------------------------------------------------------------------------
// mish(x) = x * tanh(softplus(x)); with e = exp(x): tanh(log1p(e)) = e(e+2) / (e(e+2)+2).
// torch's softplus uses threshold 20 (returns x), where tanh(.) == 1 in fp32 anyway.
// The quotient as n * rcp(n + 2) (v_rcp_f32, ≤ 1 ulp): built without fast-math, __fdividef compiled to the full IEEE
// division sequence (two v_div_scale, five fma, v_div_fmas, v_div_fixup: ≈ 12 VALU per element), which made the
// GroupNorm + Mish passes (gn_apply, the final projection's operand transform, VE_GNRES) VALU-bound. Branch-free:
// past the threshold exp overflows and the unselected side may be NaN.
__device__ __forceinline__ float mish_f(float x) {
  const float e = __expf(x);
  const float n = e * (e + 2.f);
  const float m = x * (n * __builtin_amdgcn_rcpf(n + 2.f));
  return x > 20.f ? x : m;
}
__device__ __forceinline__ float lrelu_f(float x, float slope) { return x > 0.f ? x : x * slope; }
// v / d as the product with rd = RN(1 / d) plus one FMA correction step (Markstein), the sign restored for v = -0
// (the correction's +0 + -0 is +0): 4 VALU instead of the IEEE division sequence (v_div_scale x 2, v_rcp, 5 FMAs,
// v_div_fmas, v_div_fixup). Equal to the IEEE quotient for every finite fp32 v at d = 1, 2, 3, 4, 5, 7, 8, checked
// exhaustively on gfx950 (tools/div_check.hip; d = 6 differs on subnormal results); callers require div_rn_ok(d).
// v = +-inf: q is the IEEE quotient +-inf itself (the correction's inf - inf would make it a NaN); |q| <= |v| for
// d >= 1, so q is infinite only then and finite v take the 4-VALU path's result.
__device__ __forceinline__ float div_rn(float v, float d, float rd) {
  const float q = v * rd;
  const float r = __builtin_fmaf(-q, d, v);
  const float c = __builtin_copysignf(__builtin_fmaf(r, rd, q), v);
  return __builtin_isinf(q) ? q : c;
}
inline bool div_rn_ok(float d) { return d == 1.f || d == 2.f || d == 3.f || d == 4.f || d == 5.f || d == 7.f || d == 8.f; }

// Raw buffer resources (gfx9 dword3 0x00020000): a 32-bit per-lane byte offset from a wave-uniform base, range-checked
// against num_records (an offset at or past it reads zero, also into LDS, and drops a store). Build them from
// wave-uniform values only (readfirstlane what the compiler cannot prove uniform), or every access through them
// becomes a readfirstlane loop. The LDS-DMA and store kernels (mt_rbconv, the pair kernels) put each lane's whole
// offset in voffset, so a negative offset (a frame before the utterance) wraps past the range as well.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base, unsigned num_records) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), (short)0, (int)num_records, 0x00020000);
}
// 16 bytes per lane into lds_wave_base + 16 * lane (buffer_load_dwordx4 ... lds)
__device__ __forceinline__ void buf_lds16(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff, char* lds_wave_base) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds_wave_base, 16, voff, soff, 0, 0);
}

// bf16 epilogue helpers: two channels of one packed word as packed fp32 math (v_pk_add_f32 / v_pk_mul_f32), one
// v_cvt_pk_bf16_f32 (RNE) per word, lrelu as max(x, slope * x) — equal to x > 0 ? x : slope * x for every non-NaN
// x when 0 <= slope <= 1 (files using it build with -mno-amdgpu-ieee so the max needs no NaN canonicalize)
typedef float f32x2 __attribute__((ext_vector_type(2)));
// a * b + c with one rounding per lane (v_pk_fma_f32). Epilogues that two kernels must compute to the same bits spell
// their multiply-adds out with it: left to -ffp-contract the compiler fuses them differently per code shape.
__device__ __forceinline__ f32x2 fma2(f32x2 a, f32x2 b, f32x2 c) { return __builtin_elementwise_fma(a, b, c); }
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ uint32_t pk_bf16(f32x2 v) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
}
__device__ __forceinline__ f32x2 unpk_bf16(uint32_t w) {
  return f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xffff0000u)};
}
__device__ __forceinline__ f32x2 lrelu2(f32x2 t, float slope) {
  const f32x2 m = t * slope;
  return f32x2{__builtin_fmaxf(t.x, m.x), __builtin_fmaxf(t.y, m.y)};
}
// lrelu of the two bf16 of a packed word, rounded back (the producer-side activated copy's rounding)
__device__ __forceinline__ uint32_t lrelu_pk(uint32_t w, float slope) { return pk_bf16(lrelu2(unpk_bf16(w), slope)); }
// lrelu of two fp32 values rounded ONCE to packed bf16 (a conv epilogue's activated output: the reference's fp32
// arithmetic rounds nothing there; rounding the pre-activation first as well only adds error and VALU work)
__device__ __forceinline__ uint32_t lrelu_pk_f(f32x2 v, float slope) { return pk_bf16(lrelu2(v, slope)); }
__device__ __forceinline__ uint32_t lrelu_pk_f_sel(f32x2 v, float slope) {
  const f32x2 m = v * slope;
  return pk_bf16(f32x2{v.x > 0.f ? v.x : m.x, v.y > 0.f ? v.y : m.y});
}
// the same with the compare / select lrelu (for files built with IEEE mode on, where a max needs a canonicalize)
__device__ __forceinline__ uint32_t lrelu_pk_sel(uint32_t w, float slope) {
  const f32x2 t = unpk_bf16(w), m = t * slope;
  return pk_bf16(f32x2{t.x > 0.f ? t.x : m.x, t.y > 0.f ? t.y : m.y});
}
__device__ __forceinline__ float silu_f(float x) { return x / (1.f + expf(-x)); }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}


// XCD-aligned block order (speed only, never correctness): block i of an n-block grid runs on XCD i % 8 (the
// dispatcher's round-robin); returns the chunk index block i should process so that each XCD takes a CONTIGUOUS
// range of chunks, in proportion to its block count — the same frame-range-to-XCD map mt_vconv's XCD-major tile
// walk uses, so a kernel reads what its neighbour launch wrote from its own XCD's L2. remap = 0: identity.
__device__ __forceinline__ int xcd_chunk(int i, int n, int remap) {
  if (!remap) return i;
  const int x = i & 7, j = i >> 3;
  return x * (n >> 3) + min(x, n & 7) + j;
}

}  // namespace mt

// ---------------------------------------------------------------------------
// error plumbing shared by the C ABI
// ---------------------------------------------------------------------------
namespace mt {
void set_error(const char* fmt, ...);
}
#define MT_CHECK_HIP(expr)                                                         \
  do {                                                                             \
    hipError_t _e = (expr);                                                        \
    if (_e != hipSuccess) {                                                        \
      ::mt::set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(_e),       \
                      __FILE__, __LINE__);                                         \
      return -(int)_e - 1000;                                                      \
    }                                                                              \
  } while (0)
#define MT_REQUIRE(cond, ...)                                                      \
  do {                                                                             \
    if (!(cond)) {                                                                 \
      ::mt::set_error(__VA_ARGS__);                                                \
      return -1;                                                                   \
    }                                                                              \
  } while (0)
