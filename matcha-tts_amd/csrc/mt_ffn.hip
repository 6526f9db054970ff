// Fused FeedForward of the CFM decoder's BasicTransformerBlock (bf16, gfx950):
//
//   x += W2 . snake(W1 . LN3(x) + b1) + b2        (model.py:580-609 SnakeBeta, 733-741 ff(norm3(x)) + x)
//
// The two-launch path (mt_vconv: FF1 with the LayerNorm / SnakeBeta epilogue -> a [frames][1024] bf16 tensor in HBM
// -> FF2 with the residual epilogue) moves the 1024-wide intermediate through HBM twice (at the north-star batch
// 2 x 396 MB per level-0 block) and runs two short-K GEMMs whose K loops are bound by the per-CU LDS-DMA fill.
// Here one persistent workgroup per CU walks 128-frame tiles; per tile:
//   - the tile's x rows (128 frames x 256 channels, 64 KiB) are staged once and stay in LDS (FF1's B operand and
//     FF2's residual);
//   - for each 128-channel chunk j of the intermediate: FF1 (4 steps, one 64-channel K chunk of x each) ->
//     epilogue: LayerNorm fold, bias, SnakeBeta, bf16 round -> h_j in LDS (32 KiB); FF2 (4 steps, one 64-channel
//     K chunk of h_j x one 128-row half of the output each) accumulates into the tile's 256 x 128 fp32
//     accumulators, which stay in registers across all 8 chunks;
//   - epilogue: + b2 + x (from LDS) [* mask] -> x in place.
// Weights stream through a 3-slot ring of 16 KiB slots (128 rows x 64 channels), one slot per step: 64 steps and
// 1 MiB per tile (L2-resident: every workgroup reads the same 1 MiB). Each step is one counted vmcnt wait, one
// barrier, two LDS-DMA pieces per wave (the weights of step s + 2), 12 ds_read_b128 and 16 MFMAs per wave.
// Waves: 2 along rows x 4 along frames (64 rows x 32 frames each, v_mfma_f32_16x16x32_bf16).
//
// Same bits as the two-launch path: every FF1 / FF2 output element accumulates its products in the same order
// (K chunks of 64 ascending, two 32-wide K-slices each, from a zero accumulator), and both epilogues are mt_vconv's
// packed ones (VE_LN | VE_LNP | VE_SNAKE, VE_RESID [| VE_MASK]) operation for operation; h is rounded to bf16 where
// the two-launch path stores it (tests/test_gpu_ffn.py).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mt_ffn.h"
#include "mt_vconv.h"

#ifndef FFN_NVE
#define FFN_NVE 4  // VALU instructions the scheduler places after each MFMA of an overlapped epilogue step
#endif

namespace mt {

namespace {
constexpr int FC = 256, FE = 1024, FBN = 128, FNT = 512;
constexpr int FCHUNK = FBN * 128;             // one 64-channel chunk of the tile's 128 frames (128-byte rows)
constexpr int XR_OFF = 0;                     // x rows: 4 chunks
constexpr int H_OFF = XR_OFF + 4 * FCHUNK;    // h_j: 2 chunks
constexpr int W_OFF = H_OFF + 2 * FCHUNK;     // weight ring
constexpr int FNW = 3, FWSLOT = 128 * 128;    // slot: 128 weight rows x 64 channels
constexpr int TAB_OFF = W_OFF + FNW * FWSLOT; // b1, wsum, alpha, ibeta: [1024] floats each
constexpr int FLDS = TAB_OFF + 4 * FE * 4;
static_assert(FLDS <= 160 * 1024, "LDS budget");
}  // namespace

__device__ __forceinline__ void ff_glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void ff_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int I, int N, class F>
__device__ __forceinline__ void ff_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    ff_for<I + 1, N>(f);
  }
}

template <bool MASK, bool OVL, bool UNI, bool PFB = false>
__global__ __launch_bounds__(FNT) void ffn_kernel(FfnArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[FLDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int g4 = lane >> 4, l16 = lane & 15, lrow = lane >> 3, lp = lane & 7;
  const int NF = a.frames;
  const int ntiles = (NF + FBN - 1) / FBN;
  // XCD-major tile ownership (as mt_vconv's): the 8 XCDs own contiguous frame ranges, so the x rows the block's
  // previous launch wrote are read from the same XCD's L2
  const int G = gridDim.x, g = blockIdx.x;
  const int xcd = g & 7, lw = g >> 3;
  const int gx = (G - xcd + 7) >> 3;
  const int sx = xcd * (G >> 3) + min(xcd, G & 7);
  const int xt0 = (int)((long)ntiles * sx / G), xt1 = (int)((long)ntiles * (sx + gx) / G);
  const int t0 = xt0 + lw;
  const int nmine = t0 < xt1 ? (xt1 - t0 + gx - 1) / gx : 0;
  if (nmine == 0) return;

  // ---- per-channel tables (loaded before any LDS-DMA is in flight; first read after four step barriers) ----
  {
    float* tb = reinterpret_cast<float*>(smem + TAB_OFF);
    for (int i = tid; i < FE; i += FNT) {
      tb[i] = a.b1[i];
      tb[FE + i] = a.wsum[i];
      tb[2 * FE + i] = a.alpha[i];
      tb[3 * FE + i] = a.ibeta[i];
    }
  }
  const int ch16 = wm * 64 + (g4 & 1) * 16 + (g4 >> 1) * 8;  // + fp * 32 (+ ch * 128): this lane's 8 channels

  // ---- staging ----
  const char* w1b = reinterpret_cast<const char*>(a.w1);
  const char* w2b = reinterpret_cast<const char*>(a.w2);
  int woff[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = 8 * (wave * 2 + i) + lrow;
    woff[i] = r * 128 + ((lp ^ (r & 6)) * 16);
  }
  // weights of step (j, u): u < 4: FF1 rows j*128 .. +127 of x chunk u; u >= 4: FF2 rows ch*128 .. +127 of h chunk
  // 2j + jc (jc = (u - 4) >> 1, ch = (u - 4) & 1)
  auto issue_w = [&](int j, int u, int slot) __attribute__((always_inline)) {
#if defined(FFN_EXP) && (FFN_EXP & 1)
    return;  // timing ablation (tools/exp_build.sh): no weight stream, WRONG results
#endif
    const char* base = u < 4 ? w1b + ((size_t)u * FE + j * 128) * 128
                             : w2b + ((size_t)(2 * j + ((u - 4) >> 1)) * FC + ((u - 4) & 1) * 128) * 128;
    // opaque LDS destination: a known constant range makes the compiler wait for the DMA before every ds_read it
    // cannot prove disjoint; the ordering is ours (counted waits + barrier)
    int so = W_OFF + slot * FWSLOT + wave * 2048;
    asm volatile("" : "+s"(so));
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      int wo = woff[i];
      asm volatile("" : "+v"(wo));
      ff_glds16(base + wo, smem + so + i * 1024);
    }
  };
  const char* xg = reinterpret_cast<const char*>(a.x);
  const char* zg = reinterpret_cast<const char*>(a.zero);
  auto issue_x = [&](int n0) __attribute__((always_inline)) {
    int xo = XR_OFF;
    asm volatile("" : "+s"(xo));
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int p = wave + 8 * i;  // piece: chunk p >> 4, rows 8 (p & 15) .. + 7
      const int kc = p >> 4, r = 8 * (p & 15) + lrow;
      const int q = lp ^ (r & 6);
      const int f = n0 + r;
      const char* src = f < NF ? xg + ((size_t)f * FC + kc * 64) * 2 + q * 16 : zg + q * 16;
      ff_glds16(src, smem + xo + kc * FCHUNK + (p & 15) * 1024);
    }
  };
  // per-frame operands of a tile (this lane's 2 frames): LayerNorm partials, mask
  f32x4 lnr[2][2];
  float mkr[2];
  auto frame_loads = [&](int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) {
      const int f = min(n0 + wn * 32 + fn * 16 + l16, NF - 1);
      if constexpr (!UNI) {
        const f32x4* pp = reinterpret_cast<const f32x4*>(a.ln_stats + 8 * (size_t)f);
        lnr[fn][0] = pp[0];
        lnr[fn][1] = pp[1];
      }
      mkr[fn] = MASK ? a.emask[f] : 1.f;
    }
  };

  // ---- fragments / MFMA ----
  struct Frag {
    bf16x8 A[4], B[2];
  };
  Frag F0, F1;
  // K-slice ks of a step: A = 4 row fragments (rows wm*64 + 16 fm + l16) of the slot, B = 2 frame fragments (frames
  // wn*32 + 16 fn + l16) of the 16 KiB chunk image at boff
  auto read_frag = [&](Frag& F, int ks, int slot, int boff) __attribute__((always_inline)) {
    int la = 0, lb = 0;
    asm volatile("" : "+v"(la), "+v"(lb));  // per-step addresses (no hoisting of every step's into live VGPRs)
    const char* pa = smem + W_OFF + slot * FWSLOT + (wm * 64 + l16) * 128 + la;
    const char* pb = smem + boff + (wn * 32 + l16) * 128 + lb;
    const int o = ((ks * 4 + g4) ^ (l16 & 6)) * 16;
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048 + o);
#pragma unroll
    for (int f = 0; f < 2; ++f) F.B[f] = *reinterpret_cast<const bf16x8*>(pb + f * 2048 + o);
  };
  // the two halves of read_frag (PFB: the next step's frame fragments are read at this step's end, its weight
  // fragments after its barrier, so a step's wait needs only its own weights: two steps of DMA cover)
  auto read_A = [&](Frag& F, int ks, int slot) __attribute__((always_inline)) {
    int la = 0;
    asm volatile("" : "+v"(la));
    const char* pa = smem + W_OFF + slot * FWSLOT + (wm * 64 + l16) * 128 + la;
    const int o = ((ks * 4 + g4) ^ (l16 & 6)) * 16;
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048 + o);
  };
  auto read_B = [&](Frag& F, int ks, int boff) __attribute__((always_inline)) {
    int lb = 0;
    asm volatile("" : "+v"(lb));
    const char* pb = smem + boff + (wn * 32 + l16) * 128 + lb;
    const int o = ((ks * 4 + g4) ^ (l16 & 6)) * 16;
#pragma unroll
    for (int f = 0; f < 2; ++f) F.B[f] = *reinterpret_cast<const bf16x8*>(pb + f * 2048 + o);
  };
  f32x4 acc1[4][2], acc2[2][4][2];
  // NV > 0: NV VALU instructions (an overlapped epilogue's) after each MFMA as well
  auto mma = [&](f32x4 (&acc)[4][2], const Frag& F, auto nvc) __attribute__((always_inline)) {
    constexpr int NV = decltype(nvc)::value;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma16(F.A[fm], F.B[fn], acc[fm][fn]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      if (i < 6) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read (the other slice's fragments)
      if (NV > 0) __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);  // VALU
    }
  };
  using NV0 = std::integral_constant<int, 0>;
  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  float2 lns[2];
  // FF1 epilogue of chunk j, fragment group (fp, fn): mt_vconv's VE_LN | VE_LNP | VE_SNAKE packed epilogue -> 16 bytes
  // of h_j (bf16) per lane in the LDS row layout (8 consecutive channels)
  // half h (row block fm = 2 fp + h) of a group: o[0..1]
  auto ff1_half = [&](int j, int fp, int fn, int h, uint32_t* o) __attribute__((always_inline)) {
    int lt = 0;
    asm volatile("" : "+v"(lt));  // per-use table addresses (else every group's are hoisted and kept live)
    const float* tb = reinterpret_cast<const float*>(smem + TAB_OFF + lt);
    {
        {
          const int fm = 2 * fp + h;
          const int m = j * 128 + wm * 64 + fm * 16 + 4 * g4;
          const f32x4 bias4 = *reinterpret_cast<const f32x4*>(tb + m);
          const f32x4 ws4 = *reinterpret_cast<const f32x4*>(tb + FE + m);
          const f32x4 al4 = *reinterpret_cast<const f32x4*>(tb + 2 * FE + m);
          const f32x4 ib4 = *reinterpret_cast<const f32x4*>(tb + 3 * FE + m);
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            // mt_vconv's VE_LN | VE_SNAKE packed epilogue, its multiply-adds spelled out the same way (fma2)
            f32x2 v = f32x2{acc1[fm][fn][2 * u], acc1[fm][fn][2 * u + 1]};
            v = fma2(f32x2{-lns[fn].x, -lns[fn].x}, f32x2{ws4[2 * u], ws4[2 * u + 1]}, v);
            v = fma2(v, f32x2{lns[fn].y, lns[fn].y}, f32x2{bias4[2 * u], bias4[2 * u + 1]});
            const f32x2 arg = v * f32x2{al4[2 * u], al4[2 * u + 1]};
            const f32x2 sn = f32x2{__sinf(arg.x), __sinf(arg.y)};
            v = fma2(f32x2{ib4[2 * u], ib4[2 * u + 1]}, sn * sn, v);
            o[u] = pk_bf16(v);
          }
        }
    }
  };
  auto ff1_pack = [&](uint32_t (&o)[2][2]) __attribute__((always_inline)) {
    swap16(o[0][0], o[1][0]);
    swap16(o[0][1], o[1][1]);
    return u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
  };
  auto ff1_group = [&](int j, int fp, int fn, u32x4& out) __attribute__((always_inline)) {
    uint32_t o[2][2];
    ff1_half(j, fp, fn, 0, o[0]);
    ff1_half(j, fp, fn, 1, o[1]);
    out = ff1_pack(o);
  };
  auto h_store = [&](int fp, int fn, const u32x4& v) __attribute__((always_inline)) {  // into h's chunk wm
    const int row = wn * 32 + fn * 16 + l16;
    const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
    *reinterpret_cast<u32x4*>(smem + H_OFF + wm * FCHUNK + row * 128 + ((q ^ (row & 6)) * 16)) = v;
  };
  auto acc1_zero = [&]() __attribute__((always_inline)) {
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) acc1[fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
  };
  // a tile's first step, after its barrier (the rows have landed): the LayerNorm statistics of its frames. UNI: first
  // x = bf16(x + o_b) in place and the per-slab (mean, M2) into h's space (free until chunk 0's FF1 epilogue),
  // with attn_uni_apply_kernel's arithmetic (mt_attn.hip), then a barrier
  auto tile_start = [&](int n0) __attribute__((always_inline)) {
    if constexpr (UNI) {
      float* st = reinterpret_cast<float*>(smem + H_OFF);
#pragma unroll 2
      for (int i = 0; i < FBN * 32 / FNT; ++i) {  // 2 at a time: their o_b loads in flight together, few registers
        const int task = tid + FNT * i;
        const int r = task >> 5, cl = task & 31, slab = cl >> 3, q = cl & 7;
        const int f = min(n0 + r, NF - 1);
        const float* ob = a.ovec + (size_t)(f / a.T) * FC + slab * 64 + q * 8;
        const f32x4 o0 = *reinterpret_cast<const f32x4*>(ob), o1 = *reinterpret_cast<const f32x4*>(ob + 4);
        char* px = smem + XR_OFF + slab * FCHUNK + r * 128 + ((q ^ (r & 6)) * 16);
        u32x4 w = *reinterpret_cast<const u32x4*>(px);
        const float obv[8] = {o0[0], o0[1], o0[2], o0[3], o1[0], o1[1], o1[2], o1[3]};
        float v[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const bf16 lo = (bf16)(__uint_as_float(w[e] << 16) + obv[2 * e]);
          const bf16 hi = (bf16)(__uint_as_float(w[e] & 0xffff0000u) + obv[2 * e + 1]);
          v[2 * e] = (float)lo;
          v[2 * e + 1] = (float)hi;
          w[e] = (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
        }
        *reinterpret_cast<u32x4*>(px) = w;
        float sm = ((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]));
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) sm += __shfl_xor(sm, o, 64);
        const float mu = sm * (1.f / 64.f);
        float q2 = 0.f;
#pragma unroll
        for (int e = 0; e < 8; ++e) q2 = __builtin_fmaf(v[e] - mu, v[e] - mu, q2);  // as attn_uni_apply_kernel
#pragma unroll
        for (int o = 1; o < 8; o <<= 1) q2 += __shfl_xor(q2, o, 64);
        if (q == 0) *reinterpret_cast<float2*>(st + 8 * r + 2 * slab) = float2{mu, q2};
      }
      ff_barrier();
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        const int r = wn * 32 + fn * 16 + l16;
        lnr[fn][0] = *reinterpret_cast<const f32x4*>(st + 8 * r);
        lnr[fn][1] = *reinterpret_cast<const f32x4*>(st + 8 * r + 4);
      }
    }
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) lns[fn] = ln_merge4(lnr[fn][0], lnr[fn][1], a.ln_eps);
  };
  auto ff1_epilogue = [&](int j) __attribute__((always_inline)) {
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < 2; ++fn) {
        u32x4 v;
        ff1_group(j, fp, fn, v);
        h_store(fp, fn, v);
      }
    acc1_zero();
  };
  // FF2 epilogue: mt_vconv's VE_RESID [| VE_MASK] packed epilogue, residual = the staged x rows, x overwritten
  auto ff2_epilogue = [&](int n0) __attribute__((always_inline)) {
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) {
          const int row = wn * 32 + fn * 16 + l16;
          const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
          const u32x4 rv =
              *reinterpret_cast<const u32x4*>(smem + XR_OFF + (ch * 2 + wm) * FCHUNK + row * 128 + ((q ^ (row & 6)) * 16));
          uint32_t rx0 = rv[0], rx1 = rv[1], ry0 = rv[2], ry1 = rv[3];
          swap16(rx0, ry0);  // back to the accumulator layout
          swap16(rx1, ry1);
          uint32_t o1[2][2];
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int fm = 2 * fp + h;
            // FF2 bias from global memory (L2-resident; registers are scarce across the K loop)
            const f32x4 bias4 = *reinterpret_cast<const f32x4*>(a.b2 + ch * 128 + wm * 64 + fm * 16 + 4 * g4);
            const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              f32x2 v = f32x2{acc2[ch][fm][fn][2 * u], acc2[ch][fm][fn][2 * u + 1]} + f32x2{bias4[2 * u], bias4[2 * u + 1]};
              v = v + unpk_bf16(rr[u]);
              if constexpr (MASK) v = v * mkr[fn];
              o1[h][u] = pk_bf16(v);
            }
          }
          swap16(o1[0][0], o1[1][0]);
          swap16(o1[0][1], o1[1][1]);
          const int n = n0 + row;
          const size_t off = (size_t)n * FC + ch * 128 + fp * 32 + ch16;
          *reinterpret_cast<u32x4*>(n < NF ? a.x + off : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        }
  };

  // ---- OVL: each chunk's FF1 epilogue overlapped with the previous chunk's FF2 steps ----
  // Per tile the steps run as P = FF1(0); blocks b = 0..6 = [FF1(b+1), FF2(b)]; E = FF2(7). The FF1 epilogue of chunk
  // b+1 is computed in registers during FF2(b)'s four steps (one 16-byte fragment group per step, its VALU interleaved
  // with the MFMAs) and stored into h at the next block's first step (every wave's FF2(b) reads of h are done after
  // that barrier); FF2(b+1) reads it three barriers later. h_0 (P) and h_7 (E, one extra barrier) are stored
  // unoverlapped. Same per-element operations and accumulation order as the serial schedule.
  u32x4 hreg[4];
  int cur_n0 = 0;  // the OVL schedule's current tile
  // one step: U = 0..3 FF1 x chunk U, 4..7 FF2 (h chunk (U-4)>>1, output half (U-4)&1) of chunk j; the weights of step
  // s + 2 are (j2, U2); PF: prefetch the next step's first K-slice (U1: its kind); EG: the overlapped epilogue group
  // (-1: none) of chunk je; HW: store hreg into h after the barrier (XB: then one more barrier)
  auto ostep = [&](auto Uc, int j, int j2, auto U2c, int slot, int slot1, int slot2, auto PFc, auto U1c, auto R0c,
                   auto EGc, int je, auto HWc, auto XBc, auto FIc) __attribute__((always_inline)) {
    constexpr int U = decltype(Uc)::value, U2 = decltype(U2c)::value, U1 = decltype(U1c)::value;
    constexpr bool PF = decltype(PFc)::value, R0 = decltype(R0c)::value, HW = decltype(HWc)::value;
    constexpr bool XB = decltype(XBc)::value, FI = decltype(FIc)::value;
    constexpr int EG = decltype(EGc)::value;
    __builtin_amdgcn_sched_barrier(0);
    vc_wait_vmcnt<0>();
    ff_barrier();
    if constexpr (FI) tile_start(cur_n0);
    issue_w(j2, U2, slot2);
    if constexpr (HW) {
#pragma unroll
      for (int g = 0; g < 4; ++g) h_store(g >> 1, g & 1, hreg[g]);
    }
    if constexpr (XB) ff_barrier();
    constexpr int boff = U < 4 ? XR_OFF + U * FCHUNK : H_OFF + ((U - 4) >> 1) * FCHUNK;
    if constexpr (R0) read_frag(F0, 0, slot, boff);
    read_frag(F1, 1, slot, boff);
    // the overlapped epilogue group, beside this step's MFMAs
    if constexpr (EG >= 0) ff1_group(je, EG >> 1, EG & 1, hreg[EG]);
    using NVE = std::integral_constant<int, (EG >= 0 ? FFN_NVE : 0)>;
    if constexpr (U < 4) mma(acc1, F0, NV0{});
    else mma(acc2[(U - 4) & 1], F0, NVE{});
    if constexpr (PF) {
      constexpr int boff1 = U1 < 4 ? XR_OFF + U1 * FCHUNK : H_OFF + ((U1 - 4) >> 1) * FCHUNK;
      read_frag(F0, 0, slot1, boff1);
    }
    if constexpr (U < 4) mma(acc1, F1, NV0{});
    else mma(acc2[(U - 4) & 1], F1, NVE{});
  };
  using T_ = std::true_type;
  using F_ = std::false_type;
  using NOEG = std::integral_constant<int, -1>;
  auto sel3 = [](int q, int k) {
    const int v = q + k;
    return v >= 3 ? v - 3 : v;
  };
  auto ovl_tiles = [&](Frag& F0r, Frag& F1r, int& qsr) __attribute__((always_inline)) {
    (void)F0r;
    (void)F1r;
    for (int ti = 0; ti < nmine; ++ti) {
      const int n0 = (t0 + ti * gx) * FBN;
      cur_n0 = n0;
#pragma unroll
      for (int ch = 0; ch < 2; ++ch)
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) acc2[ch][fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
      // P: FF1(0), steps 0..3; weights of steps 2, 3 (P) then 4, 5 (block 0: FF1(1) x chunks 0, 1)
      {
        const int q = qsr;
        ff_for<0, 4>([&](auto rc) __attribute__((always_inline)) {
          constexpr int r = decltype(rc)::value;
          using U2 = std::integral_constant<int, (r + 2 < 4 ? r + 2 : r - 2)>;
          using U1 = std::integral_constant<int, (r + 1 < 4 ? r + 1 : 0)>;
          using FI = std::integral_constant<bool, r == 0>;
          ostep(rc, 0, r + 2 < 4 ? 0 : 1, U2{}, sel3(q, r % 3), sel3(q, (r + 1) % 3), sel3(q, (r + 2) % 3), T_{}, U1{}, FI{},
                NOEG{}, 0, F_{}, F_{}, FI{});
        });
        __builtin_amdgcn_sched_barrier(0);
#pragma unroll
        for (int g = 0; g < 4; ++g) ff1_group(0, g >> 1, g & 1, hreg[g]);
        acc1_zero();
        qsr = sel3(q, 1);  // 4 steps
      }
      // blocks b = 0..6: FF1(b+1) x chunks 0..3, then FF2(b) (h chunk 0 halves 0, 1, h chunk 1 halves 0, 1)
      for (int b = 0; b < 7; ++b) {
        const int q = qsr;
        ff_for<0, 8>([&](auto rc) __attribute__((always_inline)) {
          constexpr int r = decltype(rc)::value;
          const int j = r < 4 ? b + 1 : b;
          // the weights of step s + 2: this block's step r + 2, or the next block's (or E's) first two
          using U2 = std::integral_constant<int, (r + 2 < 8 ? r + 2 : r - 6)>;
          const int j2 = r + 2 < 8 ? (r + 2 < 4 ? b + 1 : b) : b + 2;
          using U1 = std::integral_constant<int, (r + 1 < 8 ? r + 1 : 0)>;
          using EG = std::integral_constant<int, (r >= 4 ? r - 4 : -1)>;
          using HW = std::integral_constant<bool, r == 0>;
          if constexpr (r < 6) {
            ostep(rc, j, j2, U2{}, sel3(q, r % 3), sel3(q, (r + 1) % 3), sel3(q, (r + 2) % 3), T_{}, U1{}, F_{}, EG{}, b + 1,
                  HW{}, F_{}, F_{});
          } else {
            // r = 6, 7: the next weights are block b+1's FF1 chunks 0, 1 or, after block 6, E's FF2(7) steps 0, 1; the
            // last step prefetches block b+1's first slice (not E's: h is rewritten at E's first step)
            if (b < 6) {
              using PF = std::integral_constant<bool, true>;
              ostep(rc, j, b + 2, U2{}, sel3(q, r % 3), sel3(q, (r + 1) % 3), sel3(q, (r + 2) % 3), PF{}, U1{}, F_{},
                    EG{}, b + 1, HW{}, F_{}, F_{});
            } else {
              using PF = std::integral_constant<bool, r == 6>;
              using U2E = std::integral_constant<int, 4 + r - 6>;
              ostep(rc, j, 7, U2E{}, sel3(q, r % 3), sel3(q, (r + 1) % 3), sel3(q, (r + 2) % 3), PF{}, U1{}, F_{},
                    EG{}, b + 1, HW{}, F_{}, F_{});
            }
          }
        });
        acc1_zero();
        qsr = sel3(q, 2);  // 8 steps
      }
      // E: FF2(7) steps 0..3 (h_7 stored after the first barrier, published by a second); the next weights: E's
      // steps 2, 3, then the next tile's P steps 0, 1
      {
        const int q = qsr;
        ff_for<0, 4>([&](auto rc) __attribute__((always_inline)) {
          constexpr int r = decltype(rc)::value;
          using U = std::integral_constant<int, 4 + r>;
          using U2 = std::integral_constant<int, (r + 2 < 4 ? 4 + r + 2 : r - 2)>;
          using U1 = std::integral_constant<int, 4 + r + 1>;
          using PF = std::integral_constant<bool, r < 3>;
          using FIRST = std::integral_constant<bool, r == 0>;
          ostep(U{}, 7, r + 2 < 4 ? 7 : 0, U2{}, sel3(q, r % 3), sel3(q, (r + 1) % 3), sel3(q, (r + 2) % 3), PF{}, U1{},
                FIRST{}, NOEG{}, 0, FIRST{}, FIRST{}, F_{});
        });
        qsr = sel3(q, 1);
      }
      __builtin_amdgcn_sched_barrier(0);
      ff2_epilogue(n0);
      if (ti + 1 < nmine) {
        ff_barrier();
        const int n1 = (t0 + (ti + 1) * gx) * FBN;
        frame_loads(n1);
        issue_x(n1);
      }
    }
  };

  // ---- prologue: weights of steps 0, 1; tile 0's per-frame operands and rows ----
  issue_w(0, 0, 0);
  issue_w(0, 1, 1);
  frame_loads(t0 * FBN);
  issue_x(t0 * FBN);
#pragma unroll
  for (int fm = 0; fm < 4; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn) acc1[fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
  int qs = 0;  // ring slot of the current chunk's step 0 (the launch's step count mod 3)
  if constexpr (OVL) {
    ovl_tiles(F0, F1, qs);
  } else
  for (int ti = 0; ti < nmine; ++ti) {
    const int n0 = (t0 + ti * gx) * FBN;
#pragma unroll
    for (int ch = 0; ch < 2; ++ch)
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc2[ch][fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int j = 0; j < 8; ++j) {
      ff_for<0, 8>([&](auto uc) __attribute__((always_inline)) {
        constexpr int u = decltype(uc)::value;
        auto sel = [&](int k) {  // (qs + k) % 3
          const int v = qs + k;
          return v >= 3 ? v - 3 : v;
        };
        const int slot = sel(u % 3), slot1 = sel((u + 1) % 3), slot2 = sel((u + 2) % 3);
        // the wait publishes this step's weights AND the next one's (its first K-slice is read at this step's end;
        // issued one step ago); at a tile's first step also the tile's rows and per-frame operands (everything)
        __builtin_amdgcn_sched_barrier(0);
        if constexpr (PFB) {
          if (u == 0 && j == 0) vc_wait_vmcnt<0>();
          else vc_wait_vmcnt<2>();  // this step's weights (issued two steps ago); the next step's may be in flight
        } else {
          vc_wait_vmcnt<0>();
        }
        ff_barrier();
        if (u == 0 && j == 0) tile_start(n0);
        // weights of step s + 2 into the slot of step s - 1 (every wave's reads of it ended before this barrier)
        if constexpr (u + 2 < 8) issue_w(j, u + 2, slot2);
        else issue_w(j + 1 < 8 ? j + 1 : 0, u + 2 - 8, slot2);  // the next chunk's (or the next tile's) steps
        constexpr int boff = u < 4 ? XR_OFF + u * FCHUNK : H_OFF + ((u - 4) >> 1) * FCHUNK;
        // step 0 of a tile and FF2's first step (h_j was written after the previous step): no prefetched slice
        if constexpr (PFB) {
          read_A(F0, 0, slot);
          if (u == 4 || (u == 0 && j == 0)) read_B(F0, 0, boff);
        } else {
          if (u == 4 || (u == 0 && j == 0)) read_frag(F0, 0, slot, boff);
        }
        read_frag(F1, 1, slot, boff);
        if constexpr (u < 4) mma(acc1, F0, NV0{});
        else mma(acc2[(u - 4) & 1], F0, NV0{});
        // the next step's first K-slice (its weights were published by this step's wait), except before FF2's first
        // step and at the tile end
        if constexpr (u != 3 && u != 7) {
          constexpr int boff1 = (u + 1) < 4 ? XR_OFF + (u + 1) * FCHUNK : H_OFF + (((u + 1) - 4) >> 1) * FCHUNK;
          if constexpr (PFB) read_B(F0, 0, boff1);
          else read_frag(F0, 0, slot1, boff1);
        } else if constexpr (u == 7) {
          if (j < 7) {
            if constexpr (PFB) read_B(F0, 0, XR_OFF);
            else read_frag(F0, 0, slot1, XR_OFF);
          }
        }
        if constexpr (u < 4) mma(acc1, F1, NV0{});
        else mma(acc2[(u - 4) & 1], F1, NV0{});
        if constexpr (u == 3) {
          __builtin_amdgcn_sched_barrier(0);
          ff1_epilogue(j);
        }
      });
      qs = qs + 2 >= 3 ? qs - 1 : qs + 2;  // 8 steps per chunk: (qs + 8) % 3
    }
    __builtin_amdgcn_sched_barrier(0);
    ff2_epilogue(n0);
    // the next tile's rows replace this one's: every wave's residual reads of them are done after this barrier
    if (ti + 1 < nmine) {
      ff_barrier();
      const int n1 = (t0 + (ti + 1) * gx) * FBN;
      frame_loads(n1);
      issue_x(n1);
    }
  }
  // the prefetched weights past the last tile (valid addresses, never read) land before the LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

namespace {
int g_ffn = -1;
int ffn_knob() {
  if (g_ffn < 0) {
    const char* e = getenv("MT_FFN");
    g_ffn = e && e[0] >= '0' && e[0] <= '3' ? e[0] - '0' : 3;
  }
  return g_ffn;
}
int ffn_cus() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}
}  // namespace

int ffn_set(int enable) {  // 0 off, 1 serial schedule, 2 overlapped FF1 epilogues, 3 serial + frame-only prefetch
  const int prev = ffn_knob();
  g_ffn = enable < 0 ? 0 : enable > 3 ? 1 : enable;
  return prev;
}
int ffn_on() { return ffn_knob(); }

namespace {
int g_ffn_min = -1;
}
int ffn_min_frames() {
  if (g_ffn_min < 0) {
    const char* e = getenv("MT_FFN_MIN");
    g_ffn_min = e ? std::max(0, atoi(e)) : 16384;
  }
  return g_ffn_min;
}
int ffn_set_min_frames(int frames) {
  const int prev = ffn_min_frames();
  g_ffn_min = std::max(0, frames);
  return prev;
}

// the FFN_EXP value this file was built with (mt_build_experiments: nonzero = a timing-experiment build)
int ffn_exp_flags() {
#if defined(FFN_EXP)
  return FFN_EXP == 0 ? 0 : FFN_EXP;
#else
  return 0;
#endif
}

int launch_ffn(const FfnArgs& a, hipStream_t st) {
  MT_REQUIRE(a.x && (a.ln_stats || a.ovec) && a.w1 && a.b1 && a.wsum && a.alpha && a.ibeta && a.w2 && a.b2 && a.zero && a.trash &&
                 a.frames > 0,
             "ffn: null argument / empty");
  const int ntiles = (a.frames + FBN - 1) / FBN;
  const int G = std::min(ntiles, ffn_cus());
  MT_REQUIRE(!a.ovec || a.T > 0, "ffn: ovec needs T");
  const int mode = ffn_knob();  // 1 serial, 2 overlapped FF1 epilogues, 3 serial with frame-only prefetch
  void (*kern)(FfnArgs);
  if (mode == 2)
    kern = a.ovec ? (a.emask ? ffn_kernel<true, true, true> : ffn_kernel<false, true, true>)
                  : (a.emask ? ffn_kernel<true, true, false> : ffn_kernel<false, true, false>);
  else if (mode == 3)
    kern = a.ovec ? (a.emask ? ffn_kernel<true, false, true, true> : ffn_kernel<false, false, true, true>)
                  : (a.emask ? ffn_kernel<true, false, false, true> : ffn_kernel<false, false, false, true>);
  else  // 1 (3 is the default: the frame fragments prefetched, two steps of weight-DMA cover)
    kern = a.ovec ? (a.emask ? ffn_kernel<true, false, true> : ffn_kernel<false, false, true>)
                  : (a.emask ? ffn_kernel<true, false, false> : ffn_kernel<false, false, false>);
  hipLaunchKernelGGL(kern, dim3(G), dim3(FNT), 0, st, a);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
