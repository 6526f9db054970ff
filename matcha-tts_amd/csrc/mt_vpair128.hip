// Fused HiFi-GAN ResBlock1 PAIR for the 128-channel stage (stage 2 of v1), bf16, gfx950 — the 128-channel
// sibling of mt_vpair.hip:
//
//   t = conv_{k, d}(lrelu(x)) ;  y = conv_{k, 1}(lrelu(t)) + x          (hifigan/models.py:90-97)
//   (the last pair of resblock j: xs = [xs +] y [/ nk], + lrelu(xs) for the next upsampler, models.py:187-192)
//
// Per layer (mt_vconv) this pair moves x_act in, t out, t back in, x in, y and y_act out: six 128-channel
// tensors. Fused it moves x in and y out. The price is LDS: a 128-channel row is 256 bytes, so a tile is only
// 192 conv1 frames (the intermediate t is 192 x 128 channels), and conv2 keeps BN = 192 - 2 h2 of them
// (h2 = (k - 1) / 2: 190 / 186 / 182 output frames for k = 3 / 7 / 11).
//
// One persistent 512-thread workgroup per CU walks the tiles. Waves: 2 along rows (64 output channels each)
// x 4 along frames (48 frames = 3 fragments each). Per tile:
//   1. the RAW input rows (192 conv1 frames + the conv1 halo 2 h1 <= 40 rows: k <= 7 at d = 5, k = 11 at d <= 3;
//      a k = 11, d = 5 pair is not supported here and runs per layer on mt_vconv — the default vocoder fuses only
//      the k = 3 resblock on this kernel) of both 64-channel planes land
//      in LDS by global_load_lds_dwordx4 (issued during the previous tile's second conv); each lane reads its
//      residual rows out of them, then one in-place VALU pass turns them into lrelu(rows);
//   2. conv1: 128 rows x 192 frames over (chunk, tap) steps; epilogue lrelu(round(acc + b1)), zero outside
//      [0, L) -> T (two 64-channel planes in LDS);
//   3. conv2: 128 rows x 192 frames over T (frames past BN discarded); epilogue + b2 + x [+ xs, / nk] -> y
//      (+ lrelu(y)).
// A step is one (64-channel chunk, tap) pair: a 16 KiB weight slot of the mt_vconv image [2][k][128][64]
// (3-slot LDS ring, two steps in flight) and 24 MFMAs per wave. Steps run chunk-major, taps ascending, two
// K = 32 slices each: the per-output MFMA accumulation order of mt_vconv's K loop, and its rounding points
// (every stored tensor rounded to bf16 once, activated outputs lrelu'd in fp32 first), so the results are the
// same bits as the per-layer mt_vconv path.
// LDS: T planes (2 x 192 rows) | X planes (2 x XROWS = 232 rows) | weight ring | biases | the ragged tile map. Rows are 128 B
// with the 16-byte unit XOR-swizzled by (row & 6) (mt_vconv's conflict-free layout). conv2's discarded last
// fragments read up to 2 h2 rows past a T plane: into the next plane / the X planes, never outside LDS.
#include <algorithm>
#include <type_traits>

#include "mt_probe.h"
#include "mt_ts.h"
#include "mt_vpair.h"

namespace mt {

namespace {
constexpr int NT = 512, C = 128;
constexpr int FN = 3;                // 16-frame fragments per wave
constexpr int WNC = 16 * FN;         // frames per wave (4 waves along frames)
constexpr int NF1 = 4 * WNC;         // conv1 frames per tile (192)
constexpr int XROWS = NF1 + 40;      // staged input rows >= NF1 + 2 h1 (k <= 7 at d = 5; room for the ragged map)
constexpr int XPL = XROWS * 128;     // one 64-channel plane of X
constexpr int TPL = NF1 * 128;       // one 64-channel plane of T
constexpr int WSLOT = C * 128;       // one step: 128 output rows x 64 input channels (16 KiB)
constexpr int NWS = 3;
constexpr int T_OFF = 0, X_OFF = 2 * TPL, W_OFF = X_OFF + 2 * XPL, PAR_OFF = W_OFF + NWS * WSLOT;
constexpr int RAG_OFF = PAR_OFF + 2 * C * 4;
constexpr int LDS_BYTES = RAG_OFF + RAG_LDS;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(XROWS % 8 == 0, "X staged 8 rows per DMA instruction");
// the compile-time K loop (vpair128_kernel<EF, K>, K > 0) stages a fixed XPW row pieces per wave (8 rows of one plane
// each: 4 XPW blocks per plane, the rows past R1 zero) so that every vmcnt count is a constant; spread over the
// first XSP of conv2's steps
constexpr int XPW = 7;
#ifndef VP128_XSP
#define VP128_XSP 4
#endif
static_assert(32 * XPW <= XROWS, "fixed row staging fits the X planes");
#ifndef VP128_BUF
#define VP128_BUF 1  // 1: the compile-time kernel's LDS-DMA and the y / y2 stores through buffer resources (mt_common.h)
#endif
}  // namespace

// the compile-time K loop's schedule of vpair128_kernel<EF, K> (K > 0; registered by launch_vpair128 for the CPU replay)
template <int EF, int K>
using Vp128Sched = VpkSched<EF, 2 * (K > 0 ? K : 1), XPW, FN, (VP128_XSP < 2 * K ? VP128_XSP : 2 * (K > 0 ? K : 1)), NWS>;

namespace {

__device__ __forceinline__ void glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void wait_vmcnt(int n) {
  if (n < 7) {
    if (n < 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else if (n < 4) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  } else if (n < 15) {
    if (n < 10) asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
  } else {
    if (n < 23) asm volatile("s_waitcnt vmcnt(15)" ::: "memory");
    else if (n < 31) asm volatile("s_waitcnt vmcnt(23)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(31)" ::: "memory");
  }
}

__device__ __forceinline__ void barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// a compile-time K-loop step's barrier (mt_vpair.hip vp_step_barrier): no LDS write in flight, no lgkmcnt drain
__device__ __forceinline__ void step_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
}  // namespace

// K > 0: the compile-time K loop (k = K): steps unrolled, ring slots and vmcnt counts constants (VpkSched), step
// barriers without an lgkmcnt drain except each conv's first, phantom prefetches past the workgroup's last tile
template <int EF, int K = 0>
__global__ __launch_bounds__(NT) void vpair128_kernel(VPairArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;  // 64-row half, 48-frame quarter
  const int g4 = lane >> 4, l16 = lane & 15, lrow = lane >> 3, lp = lane & 7;
  const int k = K > 0 ? K : a.taps, d = a.dil, L = a.L;
  const int h1 = d * (k - 1) / 2, h2 = (k - 1) / 2;
  const int BN = NF1 - 2 * h2;  // output frames per tile
  const int R1 = NF1 + 2 * h1;  // staged rows per plane
  const int nxi = (R1 + 7) / 8; // DMA instructions per plane
  const int ntn = (L + BN - 1) / BN;
  // ragged batch: the live tiles of each utterance (mt_ragged.h)
  const bool rag = a.lens != nullptr;
  int* rtc = reinterpret_cast<int*>(smem + RAG_OFF);
  int* rlv = rtc + RAG_MAXB;
  if (rag) {
    rag_build(rtc, rlv, a.lens, a.lmul, L, 0, L, a.B, BN, tid);
    __syncthreads();
  }
  const int ntiles = __builtin_amdgcn_readfirstlane(rag ? rtc[a.B - 1] : a.B * ntn);  // scalar: so is the tile walk
  const int G = gridDim.x, g = blockIdx.x;
  const int gl = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int nmine = gl < ntiles ? (ntiles - gl + G - 1) / G : 0;
  if (nmine == 0) return;
  for (int i = tid; i < C; i += NT) {
    reinterpret_cast<float*>(smem + PAR_OFF)[i] = a.b1[i];
    reinterpret_cast<float*>(smem + PAR_OFF)[C + i] = a.b2[i];
  }
  __syncthreads();

  int issued = 0, xmk = 0;
  int wmk[NWS] = {};
  const int ns = 2 * k;          // steps per conv: (chunk, tap), chunk-major
  const int S = nmine * 2 * ns;  // weight steps of this workgroup
  RagWalk walk;
  auto tile_of = [&](int ti) {  // (utterance, first frame, valid frames) of tile ti
    const int tile = __builtin_amdgcn_readfirstlane(gl + ti * G);
    if (rag) return walk.at(rtc, rlv, a.B, BN, tile);
    RagTile t;
    t.b = tile / ntn;
    t.n0 = (tile - t.b * ntn) * BN;
    t.lv = L;
    return t;
  };
  RagTile nxt;  // the tile stage_x staged last (the next tile of the loop)
  // VP128_BUF: this lane's byte offsets within a weight piece (row 16 wave + lrow of the step's block; + 8 rows for
  // the second piece) and a row piece (row lrow of 8 of one plane); the 16-byte unit is swizzled by lrow & 6
  const int wlane = (16 * wave + lrow) * 128 + ((lp ^ (lrow & 6)) * 16);
  const int xlane = lrow * (C * 2) + ((lp ^ (lrow & 6)) * 16);
  auto stage_w = [&](int s) {  // step m of conv1 or conv2: image block (chunk m / k, tap m % k)
    const int r2 = s % (2 * ns);
    const int m = r2 < ns ? r2 : r2 - ns;
    const bf16* w = (r2 < ns ? a.w1 : a.w2) + (size_t)m * C * 64;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const int r = 16 * wave + 8 * u + lrow;
      glds16(w + r * 64 + (lp ^ (r & 6)) * 8, smem + W_OFF + (s % NWS) * WSLOT + (16 * wave + 8 * u) * 128);
    }
    issued += 2;
    wmk[s % NWS] = issued;
  };
  // K > 0: the weights of tile step q (mod S) into ring slot `slot` (opaque offsets: with a constant LDS destination
  // the compiler tracks the DMA and waits for it before every ds_read it cannot prove disjoint)
  auto stage_w_ct = [&](auto qc, int slot) __attribute__((always_inline)) {
    constexpr int NSK = 2 * (K > 0 ? K : 1), q = decltype(qc)::value % (2 * NSK);
    constexpr int m = q < NSK ? q : q - NSK;
    const bf16* w = (q < NSK ? a.w1 : a.w2) + (size_t)m * C * 64;
    int so = W_OFF + slot * WSLOT + 16 * wave * 128;
    asm volatile("" : "+s"(so));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if constexpr (VP128_BUF && K > 0) {
        // the step's [C][64] block as the scalar offset, the lane's row unit as the (fixed) vector offset
        const auto wr = buf_rsrc(q < NSK ? a.w1 : a.w2, (unsigned)(NSK * C * 64 * 2));
        buf_lds16(wr, (unsigned)(wlane + u * 8 * 128), (unsigned)(m * C * 64 * 2), smem + so + 8 * u * 128);
      } else {
        const int r = 16 * wave + 8 * u + lrow;
        int off = r * 64 + (lp ^ (r & 6)) * 8;
        asm volatile("" : "+v"(off));
        glds16(w + off, smem + so + 8 * u * 128);
      }
    }
  };
  const bf16* sx_xb = a.x;
  int sx_f0 = 0, sx_lv = 0;
  auto stage_x_begin = [&](int ti) {
    nxt = tile_of(K > 0 ? min(ti, nmine - 1) : ti);  // K > 0: past the last tile a phantom copy of it (never read)
    sx_xb = a.x + (size_t)__builtin_amdgcn_readfirstlane(nxt.b) * L * C;
    sx_f0 = __builtin_amdgcn_readfirstlane(nxt.n0 - h2 - h1), sx_lv = __builtin_amdgcn_readfirstlane(nxt.lv);
  };
  auto stage_x_piece = [&](int j) {  // rows 8 blk .. 8 blk + 7 of plane p (j = 2 blk + p)
    const int p = j & 1, blk = j >> 1;
    if constexpr (VP128_BUF && K > 0) {
      // the utterance as a buffer of its sx_lv valid frames: row r = frame sx_f0 + r, plane p = channels 64 p ..;
      // offsets of frames before the utterance wrap past the range (zero padding on both sides); rows past R1 are
      // staged too and never read
      buf_lds16(buf_rsrc(sx_xb, (unsigned)sx_lv * (C * 2)), (unsigned)(xlane + (sx_f0 + 8 * blk) * C * 2 + p * 128), 0u,
                smem + X_OFF + p * XPL + blk * 1024);
      return;
    }
    const int r = 8 * blk + lrow;
    const int q = lp ^ (r & 6);
    const int f = sx_f0 + r;
    const bool ok = r < R1 && f >= 0 && f < sx_lv;
    glds16(ok ? sx_xb + (size_t)f * C + p * 64 + q * 8 : a.zero + q * 8, smem + X_OFF + p * XPL + blk * 1024);
  };
  auto stage_x = [&](int ti) {  // raw rows of tile ti, both planes: row r = frame n0 - h2 - h1 + r
    stage_x_begin(ti);
    if constexpr (K > 0) {
#pragma unroll
      for (int i = 0; i < XPW; ++i) stage_x_piece(wave + 8 * i);
    } else {
      for (int j = wave; j < 2 * nxi; j += 8) {
        stage_x_piece(j);
        ++issued;
      }
      xmk = issued;
    }
  };

  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  const int ha = l16 & 6;

  f32x4 acc[4][FN];
  struct Frag {
    bf16x8 A[4], B[FN];
  };
  // K-slice ks of a step: A = this wave's 4 row fragments of the slot, B = FN frame fragments at rows
  // rb + 16 fn of plane `pl`
  auto read_frag = [&](Frag& F, int ks, int slot, const char* pl, int rb0) {
    const char* pa = smem + W_OFF + slot * WSLOT + (wm * 64 + l16) * 128 + (((ks * 4 + g4) ^ ha) * 16);
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int rb = rb0 + fn * 16;
      F.B[fn] = *reinterpret_cast<const bf16x8*>(pl + rb * 128 + (((ks * 4 + g4) ^ (rb & 6)) * 16));
    }
  };
  // first: the conv's first K-slice starts the accumulators from the MFMA's zero C operand
  auto mma_slice = [&](const Frag& F, auto first) {
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        acc[fm][fn] = mfma16(F.A[fm], F.B[fn], decltype(first)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn]);
    constexpr int NR = 4 + FN, NMF = 4 * FN;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NR, 0);
  };
  // one conv over the two planes of `src` (plane stride `pst`): steps (chunk c, tap t), the lane's first B row
  // of tap t at rb0 + t * tstride; each step's second K-slice is read under its first, the next step's first
  // under its second
  Frag F0, F1;
  int s = 0;
  VP_TS_DECL
  auto conv = [&](const char* src, int pst, int rb0, int tstride, auto&& at_first_step) {
    auto step = [&](int m, auto first) {
      const bool more = m + 1 < ns;
#if defined(VPAIR_TS)
      if (s % (2 * ns) < ns) VP_TS(4); else VP_TS(7);
#endif
      wait_vmcnt(issued - wmk[(more ? s + 1 : s) % NWS]);  // this step's weights and the next step's
      barrier();
      VP_TS(6);
      if (s + NWS - 1 < S) stage_w(s + NWS - 1);
      const int sl = s % NWS;
      const int c = m >= k ? 1 : 0, t = m - c * k;
      if constexpr (decltype(first)::value) {
        at_first_step();
        read_frag(F0, 0, sl, src, rb0);
      }
      read_frag(F1, 1, sl, src + c * pst, rb0 + t * tstride);
      mma_slice(F0, first);
      if (more) {
        const int c2 = m + 1 >= k ? 1 : 0, t2 = m + 1 - c2 * k;
        read_frag(F0, 0, (s + 1) % NWS, src + c2 * pst, rb0 + t2 * tstride);
      }
      mma_slice(F1, std::false_type{});
    };
    step(0, std::true_type{});
    ++s;
    for (int m = 1; m < ns; ++m, ++s) step(m, std::false_type{});
  };
  // K > 0: conv CV (0: conv1 = tile steps 0 .. NS-1, 1: conv2 = NS .. S-1) unrolled; the tile's ring slots from its
  // slot base sb (S % 3 != 0 rotates it per tile)
  using SCH = Vp128Sched<EF, K>;
  auto slot_of = [&](int sb, int q) __attribute__((always_inline)) {  // ring slot of tile step q (q may pass S)
    const int v = sb + q % NWS;
    return v >= NWS ? v - NWS : v;
  };
  // at_step(m): the step's other VMEM operations after its weight DMA (VpkSched::after_w)
  auto conv_ct = [&](auto cvc, const char* src, int pst, int rb0, int tstride, int sb, bool first_tile,
                     auto&& at_step) __attribute__((always_inline)) {
    constexpr int CV = decltype(cvc)::value, NSK = SCH::NS;
    vc_for<0, NSK>([&](auto mc) {
      constexpr int m = decltype(mc)::value, st = CV * NSK + m;
      constexpr bool more = m + 1 < NSK;
      constexpr int c = m >= K ? 1 : 0, t = m - c * K;
      constexpr int c2 = m + 1 >= K ? 1 : 0, t2 = m + 1 - c2 * K;
      if constexpr (CV == 0) VP_TS(4); else VP_TS(7);
      if constexpr (st == 0) {
        if (first_tile) vc_wait_vmcnt<SCH::wait_first0>();
        else vc_wait_vmcnt<SCH::wait(0)>();
      } else {
        vc_wait_vmcnt<SCH::wait(st)>();
      }
      if constexpr (m == 0) barrier();
      else step_barrier();
      VP_TS(6);
      stage_w_ct(std::integral_constant<int, st + NWS - 1>{}, slot_of(sb, st + NWS - 1));
      const int sl = slot_of(sb, st);
      int lb = 0;  // opaque per-step row base: hoisted per-step fragment addresses would take hundreds of VGPRs
      asm volatile("" : "+v"(lb));
      at_step(mc);
      if constexpr (m == 0) read_frag(F0, 0, sl, src, rb0 + lb);
      read_frag(F1, 1, sl, src + c * pst, rb0 + lb + t * tstride);
      mma_slice(F0, std::integral_constant<bool, m == 0>{});
      if constexpr (more) read_frag(F0, 0, slot_of(sb, st + 1), src + c2 * pst, rb0 + lb + t2 * tstride);
      mma_slice(F1, std::false_type{});
    });
  };

  // ---- prologue ----
  stage_x(0);
  if constexpr (K > 0) {
    vc_for<0, SCH::PW>([&](auto qc) { stage_w_ct(qc, decltype(qc)::value); });
  } else {
#pragma unroll
    for (int p = 0; p < NWS - 1; ++p)
      if (p < S) stage_w(p);
  }
  int sb = 0;  // K > 0: ring slot of the tile's step 0

  const float* par = reinterpret_cast<const float*>(smem + PAR_OFF);
  const int ch16 = (g4 & 1) * 16 + (g4 >> 1) * 8;  // + fp * 32: this lane's 8 channels after the pair swap
  const char* xpl = smem + X_OFF + wm * XPL;        // this wave's rows' plane of X
  for (int ti = 0; ti < nmine; ++ti) {
    const int b = nxt.b, n0 = nxt.n0;  // staged by the previous stage_x (tile ti)
    const int Lt = nxt.lv;             // this utterance's frames (conv2's zero padding starts there)
    // ---- 1. the residual rows of this lane's outputs (output frame n0 + i = raw row i + h2 + h1), then the
    // in-place lrelu of the landed raw rows ----
    VP_TS(10);
    if constexpr (K > 0) {
      if (ti == 0) vc_wait_vmcnt<SCH::xwait_first>();
      else vc_wait_vmcnt<SCH::xwait>();
    } else {
      wait_vmcnt(issued - xmk);
    }
    VP_TS(0);
    barrier();
    VP_TS(1);
    u32x4 rv[2][FN], yv[2][FN];  // residual x and (VE_ACCUM) old xs of this lane's outputs
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int r = wn * WNC + fn * 16 + l16 + h2 + h1;
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        rv[fp][fn] = *reinterpret_cast<const u32x4*>(xpl + r * 128 + ((q ^ (r & 6)) * 16));
      }
    barrier();
    VP_TS(2);
    for (int e = tid; e < 2 * XROWS * 8; e += NT) {
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + X_OFF + e * 16);
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = lrelu_pk(v[w], a.slope);
      *reinterpret_cast<u32x4*>(smem + X_OFF + e * 16) = v;
    }
    VP_TS(3);
    // ---- 2. conv1 (published by its first step's barrier) ----
    int ymk = 0;
    auto accum_loads = [&] {
      // VE_ACCUM: the old-xs rows of this tile's outputs, loaded now and consumed after conv2 (asm, so the
      // counted wait below retires them instead of a compiler vmcnt(0) that would drain the row staging)
      if constexpr ((EF & VE_ACCUM) != 0) {
#pragma unroll
        for (int fp = 0; fp < 2; ++fp)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            const int i = min(n0 + wn * WNC + fn * 16 + l16, L - 1);
            asm volatile("global_load_dwordx4 %0, %1, off"
                         : "=v"(yv[fp][fn])
                         : "v"(a.y + ((size_t)b * L + i) * C + wm * 64 + fp * 32 + ch16)
                         : "memory");
          }
        issued += 2 * FN;
        ymk = issued;
      }
    };
    if constexpr (K > 0) {
      conv_ct(std::integral_constant<int, 0>{}, smem + X_OFF, XPL, wn * WNC + l16, d, sb, ti == 0, [&](auto mc) {
        if constexpr (decltype(mc)::value == 0) accum_loads();
      });
    } else {
      conv(smem + X_OFF, XPL, wn * WNC + l16, d, accum_loads);
    }
    VP_TS(4);
    // epilogue: lrelu(round(acc + b1)) -> T row j (frame n0 - h2 + j), zero outside [0, L)
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = wn * WNC + fn * 16 + l16;
        const int f = n0 - h2 + j;
        const bool ok = f >= 0 && f < Lt;
        uint32_t o[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + wm * 64 + fm * 16 + 4 * g4);
          // lrelu(acc + b1) rounded once to bf16 (conv2's operand); zero outside [0, L)
          o[h][0] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][0], acc[fm][fn][1]} + f32x2{b4[0], b4[1]}, a.slope) : 0u;
          o[h][1] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][2], acc[fm][fn][3]} + f32x2{b4[2], b4[3]}, a.slope) : 0u;
        }
        swap16(o[0][0], o[1][0]);
        swap16(o[0][1], o[1][1]);
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        *reinterpret_cast<u32x4*>(smem + T_OFF + wm * TPL + j * 128 + ((q ^ (j & 6)) * 16)) =
            u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
      }
    VP_TS(5);
    // ---- 3. conv2 ----
    // every wave is past conv1's reads of the row planes: stage the next tile's raw rows into them (K > 0: spread
    // over conv2's first steps, a phantom copy of the last tile after it, so the counts stay constant)
    if constexpr (K > 0) {
      conv_ct(std::integral_constant<int, 1>{}, smem + T_OFF, TPL, wn * WNC + l16, 1, sb, false, [&](auto mc) {
        constexpr int m = decltype(mc)::value;
        if constexpr (m == 0) stage_x_begin(ti + 1);
        vc_for<0, XPW>([&](auto ic) {
          constexpr int i = decltype(ic)::value;
          if constexpr (i * SCH::XSP / XPW == m) stage_x_piece(wave + 8 * i);
        });
      });
      sb = slot_of(sb, SCH::S);
    } else {
      conv(smem + T_OFF, TPL, wn * WNC + l16, 1, [&] {
        if (ti + 1 < nmine) stage_x(ti + 1);
      });
    }
    VP_TS(7);
    // epilogue: + b2 + x [+ xs] [/ nk] -> y [, lrelu(y) -> y2]
    if constexpr ((EF & VE_ACCUM) != 0) {
      if constexpr (K > 0) vc_wait_vmcnt<SCH::accwait>();
      else wait_vmcnt(issued - ymk);
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+v"(yv[fp][fn]));  // no use of yv before the wait
    }
    VP_TS(8);
    const size_t ybase = (size_t)__builtin_amdgcn_readfirstlane(b) * L * C;
    const auto yr = buf_rsrc(a.y + ybase, (unsigned)L * (C * 2));
    const auto y2r = buf_rsrc(((EF & VE_DUAL) ? a.y2 : a.y) + ybase, (unsigned)L * (C * 2));
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int i = wn * WNC + fn * 16 + l16;  // output frame n0 + i
        uint32_t rx0 = rv[fp][fn][0], rx1 = rv[fp][fn][1], ry0 = rv[fp][fn][2], ry1 = rv[fp][fn][3];
        swap16(rx0, ry0);  // back to the accumulator layout
        swap16(rx1, ry1);
        uint32_t yx0 = 0, yx1 = 0, yy0 = 0, yy1 = 0;
        if constexpr ((EF & VE_ACCUM) != 0) {
          yx0 = yv[fp][fn][0], yx1 = yv[fp][fn][1], yy0 = yv[fp][fn][2], yy1 = yv[fp][fn][3];
          swap16(yx0, yy0);
          swap16(yx1, yy1);
        }
        uint32_t o1[2][2], o2[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + C + wm * 64 + fm * 16 + 4 * g4);
          const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
          const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
          // round(acc + b2 + x [+ xs] [/ nk]) and its lrelu, two channels per packed op
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            f32x2 v = f32x2{acc[fm][fn][2 * u], acc[fm][fn][2 * u + 1]} + f32x2{b4[2 * u], b4[2 * u + 1]};
            v = v + unpk_bf16(rr[u]);
            if constexpr ((EF & VE_ACCUM) != 0) v = unpk_bf16(yy[u]) + v;
            if constexpr ((EF & VE_DIV) != 0) v = f32x2{div_rn(v.x, a.div, 1.f / a.div), div_rn(v.y, a.div, 1.f / a.div)};
            o1[h][u] = pk_bf16(v);
            o2[h][u] = lrelu_pk(o1[h][u], a.slope);  // the stored state's activated copy
          }
        }
        swap16(o1[0][0], o1[1][0]);
        swap16(o1[0][1], o1[1][1]);
        if constexpr (VP128_BUF) {
          // the utterance's [L][C] output as a buffer: frames past L fall outside it (store dropped), the tile's
          // discarded frames i >= BN get an offset past any range; every lane still stores
          const unsigned vo = i < BN ? (unsigned)(((n0 + i) * C + wm * 64 + fp * 32 + ch16) * 2) : 0x80000000u;
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]}, yr, vo, 0, 0);
          if constexpr ((EF & VE_DUAL) != 0) {
            swap16(o2[0][0], o2[1][0]);
            swap16(o2[0][1], o2[1][1]);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]}, y2r, vo, 0, 0);
          }
          continue;
        }
        const bool ok = i < BN && n0 + i < L;
        const size_t o = ((size_t)b * L + n0 + i) * C + wm * 64 + fp * 32 + ch16;
        *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        if constexpr ((EF & VE_DUAL) != 0) {
          swap16(o2[0][0], o2[1][0]);
          swap16(o2[0][1], o2[1][1]);
          *reinterpret_cast<u32x4*>(ok ? a.y2 + o : a.trash + 8 * lane) = u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]};
        }
      }
    issued += 2 * FN * ((EF & VE_DUAL) ? 2 : 1);
    VP_TS(9);
  }
  if constexpr (K > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the phantom DMA lands before the wave ends
  VP_TS(11);
  VP_TS_END(wave, lane);
}

bool vpair128_supported(int k, int d) {
  return k >= 3 && k % 2 == 1 && NF1 - (k - 1) > 0 && NF1 + d * (k - 1) <= XROWS;
}

static int vp128_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_vpair128(int ef, const VPairArgs& a, hipStream_t st) {
  MT_REQUIRE(!(ef & VE_DIV) || div_rn_ok(a.div), "vpair128: VE_DIV divisor %g outside the exactly-checked set (div_rn)", (double)a.div);
  ef &= ~VE_Y2ONLY;  // stores y as well (VE_Y2ONLY is an option, mt_vconv.h)
  MT_REQUIRE(a.x && a.w1 && a.w2 && a.b1 && a.b2 && a.y && a.zero && a.trash && a.B > 0 && a.L > 0,
             "vpair128: null argument / empty");
  MT_REQUIRE(vpair128_supported(a.taps, a.dil), "vpair128: k %d d %d", a.taps, a.dil);
  MT_REQUIRE(!(ef & VE_DUAL) || a.y2, "vpair128: y2");
  MT_REQUIRE(a.y != a.x, "vpair128: y must not alias x (neighbour tiles read x's halo)");
  const int BN = NF1 - (a.taps - 1);
  const long ntiles = (long)a.B * ((a.L + BN - 1) / BN);
  MT_REQUIRE(ntiles < (1L << 31), "vpair128: too many tiles");
  const int G = (int)std::min<long>(ntiles, vp128_cu_count());
  // probe: the pair is two of the family's convs (SURVEY §8d algorithmic FLOPs and layer-boundary bytes)
  const double flops = 2.0 * 2.0 * C * C * a.taps * (double)a.B * a.L;
  const double bytes = 2.0 * (2.0 * 2.0 * C * (double)a.B * a.L) + 2.0 * 2.0 * C * C * a.taps;
  probe_begin(PROBE_VCONV, st);
  // the compile-time K loop for k = 3 (mt_vpair_set_kernels bit VPK_CTK128) when its fixed row staging covers R1
  const bool ct3 = a.taps == 3 && (vpair_kernels() & VPK_CTK128) != 0 && NF1 + 2 * a.dil <= 32 * XPW;
  auto go = [&](auto ec) {
    constexpr int E = decltype(ec)::value;
    if (ct3) {
      (void)VpkReg<3, Vp128Sched<E, 3>, E>::reg;
      hipLaunchKernelGGL((vpair128_kernel<E, 3>), dim3(G), dim3(NT), 0, st, a);
    }
    else hipLaunchKernelGGL((vpair128_kernel<E>), dim3(G), dim3(NT), 0, st, a);
  };
  switch (ef) {
    case 0: go(std::integral_constant<int, 0>{}); break;
    case VE_ACCUM: go(std::integral_constant<int, VE_ACCUM>{}); break;
    case VE_ACCUM | VE_DIV: go(std::integral_constant<int, VE_ACCUM | VE_DIV>{}); break;
    case VE_ACCUM | VE_DIV | VE_DUAL: go(std::integral_constant<int, VE_ACCUM | VE_DIV | VE_DUAL>{}); break;
    case VE_DIV: go(std::integral_constant<int, VE_DIV>{}); break;
    case VE_DIV | VE_DUAL: go(std::integral_constant<int, VE_DIV | VE_DUAL>{}); break;
    default: set_error("vpair128: epilogue %d not compiled in", ef); return -1;
  }
  MT_CHECK_HIP(hipGetLastError());
  probe_end(PROBE_VCONV, st, flops, bytes, PROBE_TAG_VPAIR128);
  const int rec[VCLOG_FIELDS] = {ef | 0x10000, C, BN, 0, (int)ntiles, G, a.taps, C, C, a.B, a.L};
  vclog_record(rec);
  return 0;
}

VP_TS_BINDER(vpair128_ts_bind)

}  // namespace mt
