// Fused HiFi-GAN ResBlock1 PAIR for the 64-channel stage (bf16, gfx950):
//
//   t = conv_{k, d}(lrelu(x)) ;  y = conv_{k, 1}(lrelu(t)) + x          (hifigan/models.py:90-97)
//   (the last pair of resblock j: xs = [xs +] y [/ nk], + lrelu(xs) for the next upsampler, models.py:187-192)
//
// One persistent 512-thread workgroup per CU walks tiles of 368 output frames of one utterance. Per tile:
//   1. the RAW input rows (384 conv1 frames + the conv1 halo, <= 448 rows x 64 channels) land in LDS by
//      global_load_lds_dwordx4 (issued during the previous tile's second conv); one in-place VALU pass
//      turns them into lrelu(rows), so no producer has to store an activated copy;
//   2. conv1: 64 rows x 384 frames (frames n0-8 .. n0+375) over k taps, B = the activated rows shifted by
//      t*d; epilogue lrelu(round(acc + b1)), zero outside [0, L) (conv2's zero padding) -> T in LDS;
//   3. conv2: 64 rows x 368 frames over k taps of T; epilogue + b2 + x (the residual rows, read from the
//      staged raw rows before step 1's in-place pass) [+ xs, / nk] -> y (+ lrelu(y)).
// Waves: 8 along frames (48 frames = 3 fragments each), all 64 rows. Weights stream two taps (16 KiB) per
// step (48 MFMAs per wave between barriers) through a 3-slot LDS ring; each step's wait covers the next
// step's weights too, so the next step's first K-slice fragments are read under this step's MFMAs (the mt_vconv pipeline: counted vmcnt, one
// s_barrier per step, XOR-swizzled 128-byte rows).
// HBM traffic per pair: x read once (+ halo) and y written once, instead of the per-layer path's x_act read, t written and read back, x read, y and y_act written.
// Rounding points are mt_vconv's per-layer ones (conv1's activated output lrelu(acc + b1) rounded once from fp32,
// y = round(acc + b2 + x) and its activated copy lrelu(y), rounded) and the MFMA accumulation
// order per output is the same (taps ascending, one 64-channel chunk, two K-slices), so the results are the
// same bits as the per-layer vconv path. The epilogues and the in-place lrelu pass run as packed fp32 pairs (the
// kernels are VALU-issue-bound: DESIGN.md §4), and each conv's first K-slice starts from the MFMA's zero C
// operand. k = 3 pairs run vpair3_kernel below (weights resident, double-buffered rows).
#include <algorithm>
#include <type_traits>
#include <cstdlib>
#include <cstring>

#include "mt_probe.h"
#include "mt_ts.h"
#include "mt_vpair.h"

#ifndef VP_BUF
#define VP_BUF 1  // 1: the compile-time ring kernel's LDS-DMA and every pair kernel's y / y2 stores through buffer resources
                  // (mt_common.h buf_rsrc: no per-piece 64-bit address VALU, zero padding by the range check)
#endif

#ifndef VPAIR_EXP
#define VPAIR_EXP 0  // timing experiments (tools/exp_build.sh): bits drop parts of the pair kernels' work
#endif

namespace mt {

namespace {
constexpr int NT = 512, C = 64;
constexpr int FN = 3;                // 16-frame fragments per wave (8 waves along frames, all 64 rows each)
constexpr int WNC = 16 * FN;         // frames per wave
constexpr int NF1 = 8 * WNC;         // conv1 frames per tile: n0 - HALO2 .. n0 - HALO2 + 383
constexpr int HALO2 = 8;             // >= (k - 1) / 2 of conv2
constexpr int BN = NF1 - 2 * HALO2;  // output frames per tile (368)
constexpr int XROWS = NF1 + 64;      // staged input rows >= NF1 + 2 * h1, h1 = d (k - 1) / 2 <= 32
constexpr int XBUF = XROWS * 128;
constexpr int TROWS = NF1 + 16;      // conv2's last (discarded) fragment reads up to row NF1 - 1 + 16
constexpr int TBUF = TROWS * 128;
constexpr int TAPW = 64 * 128;       // one tap: 64 output rows x 64 input channels
constexpr int WSLOT = 2 * TAPW;      // a step = two taps (the last step of an odd-k conv uses one)
constexpr int NWS = 3;
constexpr int T_OFF = XBUF, W_OFF = T_OFF + TBUF, PAR_OFF = W_OFF + NWS * WSLOT;
constexpr int RAG_OFF = PAR_OFF + 2 * C * 4;
constexpr int LDS_BYTES = RAG_OFF + RAG_LDS;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
}  // namespace

// the compile-time K loop's schedule of vpair_kernel<EF, K> (K > 0; registered by launch_vpair for the CPU replay)
template <int EF, int K>
using VpSched = VpkSched<EF, (K > 0 ? (K + 1) / 2 : 2), XROWS / 64, FN, (K > 0 ? (K + 1) / 2 : 2), NWS>;

__device__ __forceinline__ void vp_glds16(const void* src, char* lds) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds, 16, 0, 0);
}

__device__ __forceinline__ void vp_wait_vmcnt(int n) {
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

__device__ __forceinline__ void vp_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}
// a K-loop step's barrier: publishes LDS-DMA data (each wave waited for its own with vmcnt) and frees the ring slot
// of two steps back. No LDS write is in flight there, and the reads still in flight (the next step's first K-slice)
// touch neither the slot the step's DMA overwrites nor anything another wave writes, so no lgkmcnt drain: the
// compiler waits for them where the MFMAs use them
__device__ __forceinline__ void vp_step_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}


template <int EF, int K = 0>
__global__ __launch_bounds__(NT) void vpair_kernel(VPairArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, l16 = lane & 15, lrow = lane >> 3, lp = lane & 7;
  const int k = K > 0 ? K : a.taps, d = a.dil, L = a.L;
  const int h1 = d * (k - 1) / 2, h2 = (k - 1) / 2;
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
  const int ns = (k + 1) / 2;    // steps per conv
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
  // VP_BUF: this lane's byte offsets within a weight piece (row 8 wave + lrow of a tap block) and a row piece (row
  // lrow of 8); the 16-byte unit is swizzled by row & 6 = lrow & 6 in both
  const int wlane = (8 * wave + lrow) * 128 + ((lp ^ (lrow & 6)) * 16);
  const int xlane = lrow * 128 + ((lp ^ (lrow & 6)) * 16);
  auto stage_w = [&](int s) {  // taps 2m, 2m+1 (clamped to k-1) of conv1 or conv2, m = step within the conv
    const int r2 = s % (2 * ns);
    const int m = r2 < ns ? r2 : r2 - ns;
    const bf16* w = r2 < ns ? a.w1 : a.w2;
    const int r = 8 * wave + lrow;
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      const bf16* base = w + (size_t)min(2 * m + u, k - 1) * C * 64;
      vp_glds16(base + r * 64 + (lp ^ (r & 6)) * 8, smem + W_OFF + (s % NWS) * WSLOT + u * TAPW + wave * 1024);
    }
    issued += 2;
    wmk[s % NWS] = issued;
  };
  // K > 0: the weights of tile step q (mod S) into ring slot `slot` (an opaque offset: with a constant LDS destination
  // the compiler tracks the DMA and waits for it before every ds_read it cannot prove disjoint)
  auto stage_w_ct = [&](auto qc, int slot) __attribute__((always_inline)) {
    constexpr int NSK = (K + 1) / 2, q = decltype(qc)::value % (2 * NSK);
    constexpr int m = q < NSK ? q : q - NSK;
    const bf16* w = q < NSK ? a.w1 : a.w2;
    const int r = 8 * wave + lrow;
    int so = W_OFF + slot * WSLOT + wave * 1024;
    asm volatile("" : "+s"(so));
#pragma unroll
    for (int u = 0; u < 2; ++u) {
      if constexpr (VP_BUF && K > 0) {
        // tap block min(2m + u, k - 1) as the scalar offset, the lane's row unit as the (fixed) vector offset
        const auto wr = buf_rsrc(w, (unsigned)(K * C * 64 * 2));
        const unsigned tb = (unsigned)((2 * m + u < K - 1 ? 2 * m + u : K - 1) * C * 64 * 2);
        buf_lds16(wr, (unsigned)wlane, tb, smem + so + u * TAPW);
      } else {
        const bf16* base = w + (size_t)min(2 * m + u, k - 1) * C * 64;
        int off = r * 64 + (lp ^ (r & 6)) * 8;
        asm volatile("" : "+v"(off));
        vp_glds16(base + off, smem + so + u * TAPW);
      }
    }
  };
  const bf16* sx_xb = a.x;
  int sx_f0 = 0, sx_lv = 0;
  auto stage_x_begin = [&](int ti) {
    nxt = tile_of(K > 0 ? min(ti, nmine - 1) : ti);  // K > 0: past the last tile a phantom copy of it (never read)
    sx_xb = a.x + (size_t)__builtin_amdgcn_readfirstlane(nxt.b) * L * C;
    sx_f0 = __builtin_amdgcn_readfirstlane(nxt.n0 - HALO2 - h1), sx_lv = __builtin_amdgcn_readfirstlane(nxt.lv);
  };
  auto stage_x_piece = [&](int i) {  // this wave's row piece i (rows 8 j .. 8 j + 7, j = wave + 8 i)
    const int j = wave + 8 * i;
    if constexpr (VP_BUF && K > 0) {
      // the utterance as a buffer of its sx_lv valid frames: row r = frame sx_f0 + r; offsets of frames before the
      // utterance wrap past the range, so the range check reads the zero padding on both sides (rows past
      // NF1 + 2 h1 are staged too and never read)
      buf_lds16(buf_rsrc(sx_xb, (unsigned)sx_lv * (C * 2)), (unsigned)(xlane + (sx_f0 + 8 * j) * C * 2), 0u,
                smem + j * 1024);
      return;
    }
    const int r = 8 * j + lrow;
    const int q = lp ^ (r & 6);
    const int f = sx_f0 + r;
    const bool ok = r < NF1 + 2 * h1 && f >= 0 && f < sx_lv;
    vp_glds16(ok ? sx_xb + (size_t)f * C + q * 8 : a.zero + q * 8, smem + j * 1024);
  };
  auto stage_x = [&](int ti) {  // raw rows of tile ti: row r = frame n0 - HALO2 - h1 + r
    stage_x_begin(ti);
#pragma unroll
    for (int i = 0; i < XROWS / 64; ++i) stage_x_piece(i);
    issued += XROWS / 64;
    xmk = issued;
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
  // K-slice ks of tap u of a step: A = the slot's 4 row fragments of that tap, B = FN frame fragments at
  // rows rb + 16 fn of `src`
  auto read_frag = [&](Frag& F, int ks, int slot, int u, const char* src, int rb0) {
    if constexpr ((VPAIR_EXP & 32) != 0) {  // timing experiment 32: no fragment reads (wrong results)
#pragma unroll
      for (int f = 0; f < 4; ++f) asm volatile("" : "+v"(F.A[f]));
#pragma unroll
      for (int f = 0; f < FN; ++f) asm volatile("" : "+v"(F.B[f]));
      return;
    }
    const char* pa = smem + W_OFF + slot * WSLOT + u * TAPW + l16 * 128 + (((ks * 4 + g4) ^ ha) * 16);
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int rb = rb0 + fn * 16;
      F.B[fn] = *reinterpret_cast<const bf16x8*>(src + rb * 128 + (((ks * 4 + g4) ^ (rb & 6)) * 16));
    }
  };
  // 4 x FN MFMAs of one K-slice with the reads of another slice interleaved, one per MFMA issue slot
  // first: the conv's first K-slice starts the accumulators from the MFMA's zero C operand
  auto mma_slice = [&](const Frag& F, auto first) {
#pragma unroll
    for (int i = 0; i < 4 * FN; ++i) {
      const int fm = i / FN, fn = i % FN;
      if constexpr ((VPAIR_EXP & 8) != 0) {  // timing experiment: no MFMAs (wrong results)
        asm volatile("" ::"v"(F.A[fm]), "v"(F.B[fn]));
        if (decltype(first)::value) acc[fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else
        acc[fm][fn] = mfma16(F.A[fm], F.B[fn], decltype(first)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn]);
    }
    constexpr int NR = 4 + FN, NMF = 4 * FN;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NR, 0);
  };
  // one conv over `src`: ns steps of two taps (row of tap t for this lane's first fragment: rb0 + t * tstride);
  // slices in order (tap, K-slice), each read under the previous slice's MFMAs, the next step's first slice
  // under this step's last
  Frag F0 = {}, F1 = {};
  int s = 0;
  VP_TS_DECL
  auto conv = [&](const char* src, int rb0, int tstride, auto&& at_first_step) {
    auto step = [&](int m, auto first) {
      const bool more = m + 1 < ns, two = 2 * m + 1 < k;
#if defined(VPAIR_TS)
      if (s % (2 * ns) < ns) VP_TS(4); else VP_TS(7);
#endif
      if constexpr ((VPAIR_EXP & 16) == 0) {  // timing experiment 16: no per-step wait / barrier (wrong results)
        // this step's weights (staged two steps ago) and the next step's, whose first K-slice is read at this
        // step's end
        vp_wait_vmcnt(issued - wmk[(more ? s + 1 : s) % NWS]);
        vp_barrier();
      }
      VP_TS(6);
      if (s + NWS - 1 < S) stage_w(s + NWS - 1);
      const int sl = s % NWS, t0 = 2 * m;
      if constexpr (decltype(first)::value) {
        at_first_step();
        read_frag(F0, 0, sl, 0, src, rb0);
      }
      read_frag(F1, 1, sl, 0, src, rb0 + t0 * tstride);
      mma_slice(F0, first);
      if (two) {
        read_frag(F0, 0, sl, 1, src, rb0 + (t0 + 1) * tstride);
        mma_slice(F1, std::false_type{});
        read_frag(F1, 1, sl, 1, src, rb0 + (t0 + 1) * tstride);
        mma_slice(F0, std::false_type{});
      }
      if (more) read_frag(F0, 0, (s + 1) % NWS, 0, src, rb0 + (t0 + 2) * tstride);
      mma_slice(F1, std::false_type{});
    };
    step(0, std::true_type{});
    ++s;
    for (int m = 1; m < ns; ++m, ++s) step(m, std::false_type{});
  };
  // K > 0: conv CV (0: conv1 steps 0 .. NS-1 of the tile, 1: conv2 steps NS .. S-1) unrolled: ring slots from the
  // tile's slot base sb (S % 3 != 0 rotates it per tile), counted waits (VpkSched), step barriers without an lgkmcnt
  // drain (vp_step_barrier) except a conv's first, which also publishes the activated rows / T
  using SCH = VpSched<EF, K>;
  auto slot_of = [&](int sb, int q) __attribute__((always_inline)) {  // ring slot of tile step q (q may pass S)
    const int v = sb + q % NWS;
    return v >= NWS ? v - NWS : v;
  };
  // at_step(m): the step's other VMEM operations after its weight DMA (VpkSched::after_w)
  auto conv_ct = [&](auto cvc, const char* src, int rb0, int tstride, int sb, bool first_tile,
                     auto&& at_step) __attribute__((always_inline)) {
    constexpr int CV = decltype(cvc)::value, NSK = SCH::NS;
    vc_for<0, NSK>([&](auto mc) {
      constexpr int m = decltype(mc)::value, st = CV * NSK + m;
      constexpr bool more = m + 1 < NSK, two = 2 * m + 1 < K;
      if constexpr (CV == 0) VP_TS(4); else VP_TS(7);
      if constexpr (st == 0) {
        if (first_tile) vc_wait_vmcnt<SCH::wait_first0>();
        else vc_wait_vmcnt<SCH::wait(0)>();
      } else {
        vc_wait_vmcnt<SCH::wait(st)>();
      }
      if constexpr (m == 0) vp_barrier();
      else vp_step_barrier();
      VP_TS(6);
      stage_w_ct(std::integral_constant<int, st + NWS - 1>{}, slot_of(sb, st + NWS - 1));
      const int sl = slot_of(sb, st);
      constexpr int t0 = 2 * m;
      int lb = 0;  // opaque per-step row base: hoisted per-step fragment addresses would take hundreds of VGPRs
      asm volatile("" : "+v"(lb));
      at_step(mc);
      if constexpr (m == 0) read_frag(F0, 0, sl, 0, src, rb0 + lb);
      read_frag(F1, 1, sl, 0, src, rb0 + lb + t0 * tstride);
      mma_slice(F0, std::integral_constant<bool, m == 0>{});
      if constexpr (two) {
        read_frag(F0, 0, sl, 1, src, rb0 + lb + (t0 + 1) * tstride);
        mma_slice(F1, std::false_type{});
        read_frag(F1, 1, sl, 1, src, rb0 + lb + (t0 + 1) * tstride);
        mma_slice(F0, std::false_type{});
      }
      if constexpr (more) read_frag(F0, 0, slot_of(sb, st + 1), 0, src, rb0 + lb + (t0 + 2) * tstride);
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
  for (int ti = 0; ti < nmine; ++ti) {
    const int b = nxt.b, n0 = nxt.n0;  // staged by the previous stage_x (tile ti)
    const int Lt = nxt.lv;             // this utterance's frames (conv2's zero padding starts there)
    // ---- 1. the residual rows of this lane's outputs (output frame n0 + i = raw row i + HALO2 + h1), then
    // the in-place lrelu of the landed raw rows ----
    VP_TS(10);
    if constexpr (K > 0) {
      if (ti == 0) vc_wait_vmcnt<SCH::xwait_first>();
      else vc_wait_vmcnt<SCH::xwait>();
    } else {
      vp_wait_vmcnt(issued - xmk);
    }
    VP_TS(0);
    vp_barrier();
    VP_TS(1);
    u32x4 rv[2][FN], yv[2][FN];  // residual x and (VE_ACCUM) old xs of this lane's outputs
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int r = wave * WNC + fn * 16 + l16 + HALO2 + h1;
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        rv[fp][fn] = *reinterpret_cast<const u32x4*>(smem + r * 128 + ((q ^ (r & 6)) * 16));
      }
    vp_barrier();
    VP_TS(2);
#pragma unroll
    for (int i = 0; i < ((VPAIR_EXP & 1) ? 0 : XROWS * 8 / NT); ++i) {
      const int e = tid + i * NT;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + e * 16);
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = lrelu_pk(v[w], a.slope);
      *reinterpret_cast<u32x4*>(smem + e * 16) = v;
    }
    VP_TS(3);
    // ---- 2. conv1 (published by its first step's barrier) ----
    int ymk = 0;
    auto accum_loads = [&] {
      // VE_ACCUM: the old-xs rows of this tile's outputs, loaded now and consumed after conv2. Issued as asm so
      // that the counted wait below retires them: hipcc drains EVERY in-flight LDS-DMA (vmcnt(0)) before the use
      // of a compiler-visible load result, which would expose the next tile's row staging at each epilogue.
      if constexpr ((EF & VE_ACCUM) != 0) {
#pragma unroll
        for (int fp = 0; fp < 2; ++fp)
#pragma unroll
          for (int fn = 0; fn < FN; ++fn) {
            const int i = min(n0 + wave * WNC + fn * 16 + l16, L - 1);
            asm volatile("global_load_dwordx4 %0, %1, off"
                         : "=v"(yv[fp][fn])
                         : "v"(a.y + ((size_t)b * L + i) * C + fp * 32 + ch16)
                         : "memory");
          }
        issued += 2 * FN;
        ymk = issued;
      }
    };
    if constexpr (K > 0) {
      conv_ct(std::integral_constant<int, 0>{}, smem, wave * WNC + l16, d, sb, ti == 0, [&](auto mc) {
        if constexpr (decltype(mc)::value == 0) accum_loads();
      });
    } else {
      conv(smem, wave * WNC + l16, d, accum_loads);
    }
    VP_TS(4);
    // epilogue: lrelu(round(acc + b1)) -> T row j (frame n0 - HALO2 + j), zero outside [0, L)
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = wave * WNC + fn * 16 + l16;
        const int f = n0 - HALO2 + j;
        const bool ok = f >= 0 && f < Lt;
        uint32_t o[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + fm * 16 + 4 * g4);
          // lrelu(acc + b1) rounded once to bf16 (conv2's operand); zero outside [0, L)
          if constexpr ((VPAIR_EXP & 2) != 0) {  // timing experiment: no epilogue arithmetic (wrong results)
            o[h][0] = __float_as_uint(acc[fm][fn][0] + acc[fm][fn][1]);
            o[h][1] = __float_as_uint(acc[fm][fn][2] + acc[fm][fn][3]);
            continue;
          }
          o[h][0] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][0], acc[fm][fn][1]} + f32x2{b4[0], b4[1]}, a.slope) : 0u;
          o[h][1] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][2], acc[fm][fn][3]} + f32x2{b4[2], b4[3]}, a.slope) : 0u;
        }
        swap16(o[0][0], o[1][0]);
        swap16(o[0][1], o[1][1]);
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        *reinterpret_cast<u32x4*>(smem + T_OFF + j * 128 + ((q ^ (j & 6)) * 16)) =
            u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
      }
    VP_TS(5);
    // ---- 3. conv2 ----
    if constexpr (K > 0) {
      // every wave is past conv1's reads of the row buffer: stage the next tile's raw rows into it (a phantom copy of
      // the last tile after it, so the counts stay constant)
      conv_ct(std::integral_constant<int, 1>{}, smem + T_OFF, wave * WNC + l16 + HALO2 - h2, 1, sb, false,
              [&](auto mc) {
                constexpr int m = decltype(mc)::value;
                if constexpr (m == 0) stage_x_begin(ti + 1);
                vc_for<0, SCH::NXP>([&](auto ic) {
                  constexpr int i = decltype(ic)::value;
                  if constexpr (i * SCH::XSP / SCH::NXP == m) stage_x_piece(i);
                });
              });
      sb = slot_of(sb, SCH::S);
    } else {
      conv(smem + T_OFF, wave * WNC + l16 + HALO2 - h2, 1, [&] {
        if (ti + 1 < nmine) stage_x(ti + 1);
      });
    }
    VP_TS(7);
    // epilogue: + b2 + x [+ xs] [/ nk] -> y [, lrelu(y) -> y2]
    if constexpr ((EF & VE_ACCUM) != 0) {
      if constexpr (K > 0) vc_wait_vmcnt<SCH::accwait>();
      else vp_wait_vmcnt(issued - ymk);
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+v"(yv[fp][fn]));  // no use of yv before the wait
    }
    VP_TS(8);
    static_assert(BN == 8 * WNC - 16 && WNC > 16, "only the last wave's last fragment lies past BN");
    const size_t ybase = (size_t)__builtin_amdgcn_readfirstlane(b) * L * C;
    const auto yr = buf_rsrc(a.y + ybase, (unsigned)L * (C * 2));
    const auto y2r = buf_rsrc(((EF & VE_DUAL) ? a.y2 : a.y) + ybase, (unsigned)L * (C * 2));
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int i = wave * WNC + fn * 16 + l16;  // output frame n0 + i
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
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + C + fm * 16 + 4 * g4);
          const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
          const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
          // round(acc + b2 + x [+ xs] [/ nk]) and its lrelu, two channels per packed op
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if constexpr ((VPAIR_EXP & 4) != 0) {  // timing experiment: no epilogue arithmetic (wrong results)
              o1[h][u] = o2[h][u] = __float_as_uint(acc[fm][fn][2 * u] + acc[fm][fn][2 * u + 1]) ^ rr[u] ^ yy[u];
              continue;
            }
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
        if constexpr (VP_BUF) {
          // the utterance's [L][C] output as a buffer: frames past L fall outside it (store dropped); the discarded
          // frames i >= BN (the last wave's last fragment) get an offset past any range; every lane still stores
          const bool keep = !(fn == FN - 1 && wave == 7);
          const unsigned vo = keep ? (unsigned)(((n0 + i) * C + fp * 32 + ch16) * 2) : 0x80000000u;
          if constexpr ((EF & VE_Y2ONLY) == 0)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]}, yr, vo, 0, 0);
          if constexpr ((EF & VE_DUAL) != 0) {
            swap16(o2[0][0], o2[1][0]);
            swap16(o2[0][1], o2[1][1]);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]}, y2r, vo, 0, 0);
          }
          continue;
        }
        const bool ok = i < BN && n0 + i < L;
        const size_t o = ((size_t)b * L + n0 + i) * C + fp * 32 + ch16;
        if constexpr ((EF & VE_Y2ONLY) == 0)
          *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        if constexpr ((EF & VE_DUAL) != 0) {
          swap16(o2[0][0], o2[1][0]);
          swap16(o2[0][1], o2[1][1]);
          *reinterpret_cast<u32x4*>(ok ? a.y2 + o : a.trash + 8 * lane) = u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]};
        }
      }
    issued += 2 * FN * ((EF & VE_DUAL) && !(EF & VE_Y2ONLY) ? 2 : 1);
    VP_TS(9);
  }
  if constexpr (K > 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // phantom prefetches land before LDS is freed
  VP_TS(11);
  VP_TS_END(wave, lane);
}

// ---- k = 3 pairs: HBM-bound (stage 3 at B = 256: 2.5 ms per pair for 6.3 GB of x in / y out), so this variant
// keeps the pair's 48 KiB of weights resident (no ring, four barriers per tile) and double-buffers the row
// staging: tiles of 256 conv1 frames (2 fragments per wave, HALO2 = h2 = 1, 254 output frames) and the NEXT
// tile's rows issued at the start of this one. Same fragments, accumulation order and rounding points as
// vpair_kernel (taps ascending, two K-slices each), so the same bits.
namespace {
// FNT 16-frame fragments per wave; DB: two row buffers (the next tile's rows issued at the start of this one)
template <int FNT, bool DB>
struct K3G {
  static constexpr int FN = FNT, WNC = 16 * FN, NF1 = 8 * WNC, HALO2 = 1, BN = NF1 - 2 * HALO2;
  static constexpr int XROWS = NF1 + 16;  // >= NF1 + 2 d for d <= 8
  static constexpr int XBUF = XROWS * 128, NXB = DB ? 2 : 1;
  static constexpr int TROWS = NF1 + 8;   // conv2 reads rows <= NF1 - 1 + 2
  static constexpr int T_OFF = NXB * XBUF, W_OFF = T_OFF + TROWS * 128, PAR_OFF = W_OFF + 6 * TAPW;
  static constexpr int RAG_OFF = PAR_OFF + 2 * C * 4;
  static constexpr int LDS = RAG_OFF + RAG_LDS;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(XROWS % 8 == 0, "rows staged 8 per DMA");
};
}  // namespace

template <int EF, int FNT, bool DB>
__global__ __launch_bounds__(NT) void vpair3_kernel(VPairArgs a) {
  using G3 = K3G<FNT, DB>;
  __shared__ __attribute__((aligned(1024))) char smem[G3::LDS];
  constexpr int FN = G3::FN, WNC = G3::WNC, NF1 = G3::NF1, HALO2 = G3::HALO2, BN = G3::BN;
  constexpr int K3_XROWS = G3::XROWS, K3_XBUF = G3::XBUF, K3_T_OFF = G3::T_OFF, K3_W_OFF = G3::W_OFF;
  constexpr int K3_PAR_OFF = G3::PAR_OFF;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, l16 = lane & 15, lrow = lane >> 3, lp = lane & 7;
  const int d = a.dil, L = a.L;
  const int h1 = d;  // k = 3: h1 = d, h2 = 1 = HALO2
  const int ntn = (L + BN - 1) / BN;
  // ragged batch: the live tiles of each utterance (mt_ragged.h)
  const bool rag = a.lens != nullptr;
  int* rtc = reinterpret_cast<int*>(smem + G3::RAG_OFF);
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
    reinterpret_cast<float*>(smem + K3_PAR_OFF)[i] = a.b1[i];
    reinterpret_cast<float*>(smem + K3_PAR_OFF)[C + i] = a.b2[i];
  }
  __syncthreads();

  int issued = 0;
  int xmk[2] = {0, 0};
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
  // both convs' 3 taps: DMA j moves rows (j & 7) * 8 .. + 7 of tap j / 8 (conv (j / 8) / 3)
  for (int j = wave; j < 48; j += 8) {
    const int tp = j >> 3, r = (j & 7) * 8 + lrow;
    const bf16* w = (tp < 3 ? a.w1 : a.w2) + (size_t)(tp % 3) * C * 64;
    vp_glds16(w + r * 64 + (lp ^ (r & 6)) * 8, smem + K3_W_OFF + tp * TAPW + (j & 7) * 1024);
    ++issued;
  }
  const bf16* sx_xb = a.x;
  int sx_f0 = 0, sx_R1 = 0, sx_lv = 0, sx_buf = 0;
  auto stage_x_begin = [&](int ti) {
    nxt = tile_of(ti);
    const bool live = ti < nmine;
    sx_xb = a.x + (size_t)(live ? nxt.b : 0) * L * C;
    sx_f0 = nxt.n0 - HALO2 - h1, sx_R1 = live ? NF1 + 2 * h1 : 0, sx_lv = nxt.lv;
    sx_buf = DB ? ti & 1 : 0;
  };
  auto stage_x_piece = [&](int j) {  // DMA j (rows 8 j .. 8 j + 7) of the tile begun by stage_x_begin
    const int r = 8 * j + lrow;
    const int q = lp ^ (r & 6);
    const int f = sx_f0 + r;
    const bool ok = r < sx_R1 && f >= 0 && f < sx_lv;
    vp_glds16(ok ? sx_xb + (size_t)f * C + q * 8 : a.zero + q * 8, smem + sx_buf * K3_XBUF + j * 1024);
    ++issued;
  };
  auto stage_x = [&](int ti) {  // raw rows of tile ti into buffer ti & 1: row r = frame n0 - HALO2 - h1 + r
    stage_x_begin(ti);
    for (int j = wave; j < K3_XROWS / 8; j += 8) stage_x_piece(j);
    xmk[DB ? ti & 1 : 0] = issued;
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
  auto read_frag = [&](Frag& F, int ks, int tp, const char* src, int rb0) {
    const char* pa = smem + K3_W_OFF + tp * TAPW + l16 * 128 + (((ks * 4 + g4) ^ ha) * 16);
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int rb = rb0 + fn * 16;
      F.B[fn] = *reinterpret_cast<const bf16x8*>(src + rb * 128 + (((ks * 4 + g4) ^ (rb & 6)) * 16));
    }
  };
  // first: the conv's first K-slice starts the accumulators from the MFMA's zero C operand
  auto mma_slice = [&](const Frag& F, auto first) {
#pragma unroll
    for (int i = 0; i < 4 * FN; ++i) {
      const int fm = i / FN, fn = i % FN;
      if constexpr ((VPAIR_EXP & 8) != 0) {  // timing experiment: no MFMAs (wrong results)
        asm volatile("" ::"v"(F.A[fm]), "v"(F.B[fn]));
        if (decltype(first)::value) acc[fm][fn] = f32x4{0.f, 0.f, 0.f, 0.f};
      } else
        acc[fm][fn] = mfma16(F.A[fm], F.B[fn], decltype(first)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn]);
    }
    constexpr int NR = 4 + FN, NMF = 4 * FN;
#pragma unroll
    for (int i = 0; i < NMF; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      if (i < NR) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
  };
  // one conv (tp0 = 0: conv1, 3: conv2): taps ascending, two K-slices each, each slice read under the previous
  Frag F0, F1;
  // after_tap(tp): called after tap tp's MFMAs are issued (VP_XSPREAD: the next tile's row pieces)
  auto conv = [&](int tp0, const char* src, int rb0, int tstride, auto&& after_tap) {
    read_frag(F0, 0, tp0, src, rb0);
    read_frag(F1, 1, tp0, src, rb0);
    mma_slice(F0, std::true_type{});
    read_frag(F0, 0, tp0 + 1, src, rb0 + tstride);
    mma_slice(F1, std::false_type{});
    after_tap(tp0);
#pragma unroll
    for (int t = 1; t < 3; ++t) {
      read_frag(F1, 1, tp0 + t, src, rb0 + t * tstride);
      mma_slice(F0, std::false_type{});
      if (t < 2) read_frag(F0, 0, tp0 + t + 1, src, rb0 + (t + 1) * tstride);
      mma_slice(F1, std::false_type{});
      after_tap(tp0 + t);
    }
  };
  // DB: the next tile's rows go out one DMA piece per tap (piece p of this wave, j = wave + 8 p, after tap p of the
  // tile's six) instead of one burst at the tile start: a burst stalls its wave on the DMA issue while nothing else
  // is in flight, and VE_ACCUM's wait for its old-xs loads (issued before the rows) waited for the whole burst;
  // spread, the pieces issue among the MFMAs (pairlab: 0.96x the burst's time, 0.86x with VE_ACCUM)
  auto spread = [&](int tp) {
    if constexpr (DB) {
      __builtin_amdgcn_sched_barrier(0);
      const int j = wave + 8 * tp;
      if (j < K3_XROWS / 8) stage_x_piece(j);
      if (tp == 5) xmk[sx_buf] = issued;
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  static_assert(!DB || (K3_XROWS / 8 + 7) / 8 <= 6, "row pieces per wave fit the taps");

  stage_x(0);
  const float* par = reinterpret_cast<const float*>(smem + K3_PAR_OFF);
  const int ch16 = (g4 & 1) * 16 + (g4 >> 1) * 8;
  VP_TS_DECL
  for (int ti = 0; ti < nmine; ++ti) {
    const int b = nxt.b, n0 = nxt.n0;  // staged by the previous stage_x (tile ti)
    const int Lt = nxt.lv;             // this utterance's frames (conv2's zero padding starts there)
    char* xs = smem + (DB ? ti & 1 : 0) * K3_XBUF;
    // ---- 1. rows landed (the first wait also covers the weights); old-xs loads, then the next tile's rows
    // into the other buffer (vmcnt retires in order); residual rows; in-place lrelu ----
    VP_TS(10);
    vp_wait_vmcnt(issued - xmk[DB ? ti & 1 : 0]);
    VP_TS(0);
    vp_barrier();
    VP_TS(1);
    u32x4 rv[2][FN], yv[2][FN];
    int ymk = 0;
    if constexpr ((EF & VE_ACCUM) != 0) {
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int i = min(n0 + wave * WNC + fn * 16 + l16, L - 1);
          asm volatile("global_load_dwordx4 %0, %1, off"
                       : "=v"(yv[fp][fn])
                       : "v"(a.y + ((size_t)b * L + i) * C + fp * 32 + ch16)
                       : "memory");
        }
      issued += 2 * FN;
      ymk = issued;
    }
    if constexpr (DB) stage_x_begin(ti + 1);  // its pieces issue between the convs' taps (spread)
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int r = wave * WNC + fn * 16 + l16 + HALO2 + h1;
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        rv[fp][fn] = *reinterpret_cast<const u32x4*>(xs + r * 128 + ((q ^ (r & 6)) * 16));
      }
    vp_barrier();
    VP_TS(2);
    for (int e = tid; e < ((VPAIR_EXP & 1) ? 0 : K3_XBUF / 16); e += NT) {
      u32x4 v = *reinterpret_cast<const u32x4*>(xs + e * 16);
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = lrelu_pk(v[w], a.slope);
      *reinterpret_cast<u32x4*>(xs + e * 16) = v;
    }
    vp_barrier();
    VP_TS(3);
    // ---- 2. conv1 -> T ----
    conv(0, xs, wave * WNC + l16, d, spread);
    VP_TS(4);
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int j = wave * WNC + fn * 16 + l16;
        const int f = n0 - HALO2 + j;
        const bool ok = f >= 0 && f < Lt;
        uint32_t o[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + fm * 16 + 4 * g4);
          // lrelu(acc + b1) rounded once to bf16 (conv2's operand); zero outside [0, L)
          if constexpr ((VPAIR_EXP & 2) != 0) {  // timing experiment: no epilogue arithmetic (wrong results)
            o[h][0] = __float_as_uint(acc[fm][fn][0] + acc[fm][fn][1]);
            o[h][1] = __float_as_uint(acc[fm][fn][2] + acc[fm][fn][3]);
            continue;
          }
          o[h][0] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][0], acc[fm][fn][1]} + f32x2{b4[0], b4[1]}, a.slope) : 0u;
          o[h][1] = ok ? lrelu_pk_f(f32x2{acc[fm][fn][2], acc[fm][fn][3]} + f32x2{b4[2], b4[3]}, a.slope) : 0u;
        }
        swap16(o[0][0], o[1][0]);
        swap16(o[0][1], o[1][1]);
        const int q = fp * 4 + (g4 & 1) * 2 + (g4 >> 1);
        *reinterpret_cast<u32x4*>(smem + K3_T_OFF + j * 128 + ((q ^ (j & 6)) * 16)) =
            u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
      }
    VP_TS(5);
    vp_barrier();  // T published (single buffer: every wave is past conv1's reads of the rows)
    if constexpr (!DB) stage_x(ti + 1);
    VP_TS(6);
    // ---- 3. conv2 -> y ----
    conv(3, smem + K3_T_OFF, wave * WNC + l16, 1, spread);
    VP_TS(7);
    if constexpr ((EF & VE_ACCUM) != 0) {
      vp_wait_vmcnt(issued - ymk);
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+v"(yv[fp][fn]));
    }
    VP_TS(8);
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int i = wave * WNC + fn * 16 + l16;
        uint32_t rx0 = rv[fp][fn][0], rx1 = rv[fp][fn][1], ry0 = rv[fp][fn][2], ry1 = rv[fp][fn][3];
        swap16(rx0, ry0);
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
          const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + C + fm * 16 + 4 * g4);
          const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
          const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
          // round(acc + b2 + x [+ xs] [/ nk]) and its lrelu, two channels per packed op
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            if constexpr ((VPAIR_EXP & 4) != 0) {  // timing experiment: no epilogue arithmetic (wrong results)
              o1[h][u] = o2[h][u] = __float_as_uint(acc[fm][fn][2 * u] + acc[fm][fn][2 * u + 1]) ^ rr[u] ^ yy[u];
              continue;
            }
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
        const bool ok = i < BN && n0 + i < L;
        const size_t o = ((size_t)b * L + n0 + i) * C + fp * 32 + ch16;
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
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing row DMAs land before LDS is freed
  VP_TS(11);
  VP_TS_END(wave, lane);
}

static int g_vpk = -1;
int vpair_kernels() {
  if (g_vpk < 0) {
    const char* e = getenv("MT_VPAIRK");
    g_vpk = e ? atoi(e) & VPK_ALL : VPK_ALL;
  }
  return g_vpk;
}
int vpair_set_kernels(int mask) {
  const int prev = vpair_kernels();
  g_vpk = mask & VPK_ALL;
  return prev;
}

// the VPAIR_EXP value this file was built with (mt_build_experiments: nonzero = a timing-experiment build)
int vpair_exp_flags() { return VPAIR_EXP; }

bool vpair_supported(int C_, int k, int d) {
  return C_ == C && k >= 2 && (k - 1) / 2 <= HALO2 && NF1 + d * (k - 1) <= XROWS;
}

static int vp_cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_vpair(int ef, const VPairArgs& a, hipStream_t st) {
  MT_REQUIRE(!(ef & VE_DIV) || div_rn_ok(a.div), "vpair: VE_DIV divisor %g outside the exactly-checked set (div_rn)", (double)a.div);
  MT_REQUIRE(a.x && a.w1 && a.w2 && a.b1 && a.b2 && a.y && a.zero && a.trash && a.B > 0 && a.L > 0,
             "vpair: null argument / empty");
  MT_REQUIRE(vpair_supported(C, a.taps, a.dil) && a.taps % 2 == 1, "vpair: k %d d %d", a.taps, a.dil);
  MT_REQUIRE(!(ef & VE_DUAL) || a.y2, "vpair: y2");
  MT_REQUIRE(a.y != a.x, "vpair: y must not alias x (neighbour tiles read x's halo)");
  // k = 3: resident weights; MT_VPAIR3 (A/B knob, read once) picks the geometry: "2d" (default) 2 fragments per
  // wave + double-buffered rows, "2" / "3" 2 / 3 fragments single-buffered, "0" the weight-ring kernel
  static const int k3mode = [] {
    const char* e = getenv("MT_VPAIR3");
    return !e ? 1 : !strcmp(e, "0") ? 0 : !strcmp(e, "2") ? 2 : !strcmp(e, "3") ? 3 : 1;
  }();
  const bool k3 = a.taps == 3 && a.dil <= 8 && k3mode != 0;
  if (k3 || !(ef & VE_DUAL)) ef &= ~VE_Y2ONLY;  // only the ring kernel drops the raw store (VE_Y2ONLY)
  const int bn = !k3 ? BN : k3mode == 3 ? K3G<3, false>::BN : K3G<2, true>::BN;
  const long ntiles = (long)a.B * ((a.L + bn - 1) / bn);
  const int G = (int)std::min<long>(ntiles, vp_cu_count());
  // probe: the pair is two of the family's convs (SURVEY §8d algorithmic FLOPs and layer-boundary bytes)
  const double flops = 2.0 * 2.0 * C * C * a.taps * (double)a.B * a.L;
  const double bytes = 2.0 * (2.0 * 2.0 * C * (double)a.B * a.L) + 2.0 * 2.0 * C * C * a.taps;
  probe_begin(PROBE_VCONV, st);
  if (k3) {
    auto go = [&](auto kern) { hipLaunchKernelGGL(kern, dim3(G), dim3(NT), 0, st, a); };
#define MT_VP3(E)                                                       \
  (k3mode == 3 ? go(vpair3_kernel<E, 3, false>) : k3mode == 2 ? go(vpair3_kernel<E, 2, false>) \
               : go(vpair3_kernel<E, 2, true>))
    switch (ef) {
      case 0: MT_VP3(0); break;
      case VE_ACCUM: MT_VP3(VE_ACCUM); break;
      case VE_ACCUM | VE_DIV: MT_VP3(VE_ACCUM | VE_DIV); break;
      case VE_ACCUM | VE_DIV | VE_DUAL: MT_VP3(VE_ACCUM | VE_DIV | VE_DUAL); break;
      case VE_DIV: MT_VP3(VE_DIV); break;
      case VE_DIV | VE_DUAL: MT_VP3(VE_DIV | VE_DUAL); break;
      default: set_error("vpair: epilogue %d not compiled in", ef); return -1;
    }
#undef MT_VP3
  } else {
    // k = 7 / 11 (the vocoder's): the compile-time K loop; other kernel sizes the runtime-k loop (same bits)
    const bool ctk = (vpair_kernels() & VPK_CTK) != 0;
    auto ring = [&](auto efc) {
      constexpr int E = decltype(efc)::value;
      if (!ctk) hipLaunchKernelGGL((vpair_kernel<E>), dim3(G), dim3(NT), 0, st, a);
      else if (a.taps == 7) {
        (void)VpkReg<2, VpSched<E, 7>, E>::reg;
        hipLaunchKernelGGL((vpair_kernel<E, 7>), dim3(G), dim3(NT), 0, st, a);
      } else if (a.taps == 11) {
        (void)VpkReg<2, VpSched<E, 11>, E>::reg;
        hipLaunchKernelGGL((vpair_kernel<E, 11>), dim3(G), dim3(NT), 0, st, a);
      }
      else hipLaunchKernelGGL((vpair_kernel<E>), dim3(G), dim3(NT), 0, st, a);
    };
    switch (ef) {
      case 0: ring(std::integral_constant<int, 0>{}); break;
      case VE_ACCUM: ring(std::integral_constant<int, VE_ACCUM>{}); break;
      case VE_ACCUM | VE_DIV: ring(std::integral_constant<int, VE_ACCUM | VE_DIV>{}); break;
      case VE_ACCUM | VE_DIV | VE_DUAL: ring(std::integral_constant<int, VE_ACCUM | VE_DIV | VE_DUAL>{}); break;
      case VE_ACCUM | VE_DIV | VE_DUAL | VE_Y2ONLY:
        ring(std::integral_constant<int, VE_ACCUM | VE_DIV | VE_DUAL | VE_Y2ONLY>{});
        break;
      case VE_DIV: ring(std::integral_constant<int, VE_DIV>{}); break;
      case VE_DIV | VE_DUAL: ring(std::integral_constant<int, VE_DIV | VE_DUAL>{}); break;
      default: set_error("vpair: epilogue %d not compiled in", ef); return -1;
    }
  }
  MT_CHECK_HIP(hipGetLastError());
  probe_end(PROBE_VCONV, st, flops, bytes, PROBE_TAG_VPAIR);
  const int rec[VCLOG_FIELDS] = {ef | 0x10000, C, bn, 0, (int)ntiles, G, a.taps, C, C, a.B, a.L};
  vclog_record(rec);
  return 0;
}

VP_TS_BINDER(vpair_ts_bind)

}  // namespace mt
