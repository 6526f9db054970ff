// Fused HiFi-GAN ResBlock1 PAIR for the 32-channel (last) stage, bf16, gfx950 — the 32-channel sibling of
// mt_vpair.hip:
//
//   t = conv_{k, d}(lrelu(x)) ;  y = conv_{k, 1}(lrelu(t)) + x          (hifigan/models.py:90-97)
//   (the last pair of resblock j: xs = [xs +] y [/ nk], models.py:187-192)
//
// One persistent 512-thread workgroup per CU walks tiles of 752 output frames of one utterance. Per tile:
//   1. the RAW input rows (768 conv1 frames + the conv1 halo, <= 896 rows x 32 channels = 64 B) land in LDS by
//      global_load_lds_dwordx4 (issued during the previous tile's second conv); one in-place VALU pass turns
//      them into lrelu(rows);
//   2. conv1: 32 rows x 768 frames over k taps; epilogue lrelu(round(acc + b1)), zero outside [0, L) -> T;
//   3. conv2: 32 rows x 752 frames over k taps of T; epilogue + b2 + x (the residual rows, read from the
//      staged raw rows before step 1's in-place pass) [+ xs, / nk] -> y.
// A tap is one K = 32 MFMA slice and a wave covers 96 frames (6 fragments) x both 16-row fragments. ALL of the
// pair's weights (2 convs x k taps x 2 KiB <= 52 KiB, read straight from the generic [32 rows][k][32] packing)
// land in LDS once per launch, so the conv loops run with no weight DMA and no barrier: a tile has four
// barriers (rows landed, residuals read, rows activated, T written) where a 3-slot weight ring of 4-tap steps
// had 2 + 2 ceil(k / 4).
// LDS rows are 64 bytes (four 16-byte chunks); chunk c of row r lives in slot c ^ ((r >> 1) & 2). With the
// ds_read_b128 lane groups ({0-3,12-15,20-27}, ...; MI355X_MICROARCH.md §LDS) every B-fragment read (16
// consecutive rows from any start row, chunk g4) and every A-fragment read is conflict-free, and so are the
// 8-lane groups of the epilogue's ds_write_b128 (checked exhaustively over start rows when the layout was chosen).
// The per-output accumulation order (taps ascending, one K = 32 slice per tap) equals the generic per-layer conv
// path's (mt_conv.hip); the rounding points are mt_vconv's (conv1's activated output and y's activated copy rounded
// once from fp32), so against the generic path (which activates the rounded t) results agree to bf16 rounding.
#include <algorithm>
#include <type_traits>

#include "mt_probe.h"
#include "mt_ts.h"
#include "mt_vpair.h"

namespace mt {

namespace {
constexpr int NT = 512, C = 32;
constexpr int FN = 6;                // 16-frame fragments per wave (8 waves along frames, both row fragments)
constexpr int WNC = 16 * FN;         // frames per wave
constexpr int NF1 = 8 * WNC;         // conv1 frames per tile: n0 - HALO2 .. n0 - HALO2 + 767
constexpr int HALO2 = 8;             // >= (k - 1) / 2 of conv2
constexpr int BN = NF1 - 2 * HALO2;  // output frames per tile (752)
constexpr int RB = C * 2;            // bytes per LDS row
constexpr int XROWS = NF1 + 128;     // staged input rows >= NF1 + 2 * h1, h1 = d (k - 1) / 2 <= 64
constexpr int XBUF = XROWS * RB;
constexpr int TROWS = NF1 + 16;      // conv2's last (discarded) fragment reads up to row NF1 - 1 + 16
constexpr int TBUF = TROWS * RB;
constexpr int KMAX = 11;             // largest kernel size whose weights stay resident
constexpr int TAPW = C * RB;         // one tap: 32 output rows x 32 input channels (2 KiB)
constexpr int T_OFF = XBUF, W_OFF = T_OFF + TBUF, PAR_OFF = W_OFF + 2 * KMAX * TAPW;  // W: [conv][tap]
constexpr int RAG_OFF = PAR_OFF + 2 * C * 4;
constexpr int LDS_BYTES = RAG_OFF + RAG_LDS;
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
static_assert(XROWS % 128 == 0 && TAPW == 2 * 1024, "two 1 KiB DMAs per tap");

__device__ __forceinline__ int swz(int r) { return (r >> 1) & 2; }

#ifndef VP32_BUF
#define VP32_BUF 1  // 1: row staging and the y / y2 stores through buffer resources (mt_rbconv's RB_BUF)
#endif

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
}  // namespace

template <int EF>
__global__ __launch_bounds__(NT) void vpair32_kernel(VPairArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int g4 = lane >> 4, l16 = lane & 15, lrow = lane >> 2, lp = lane & 3;
  const int k = a.taps, d = a.dil, L = a.L;
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

  // VE_POST (the vocoder's last pair): conv2's outputs are frames n0 - PS + i (PS = 3: the 3-frame halo conv_post
  // reads on each side of the tile's BN outputs lies inside the frames conv2 computes validly, i < NF1 - 2 h2 - ... );
  // xs goes to LDS as conv_post's input (post_taps) and only the waveform is stored
  constexpr bool POST = (EF & VE_POST) != 0;
  constexpr int PS = POST ? 3 : 0;
  static_assert(!POST || ((EF & VE_ACCUM) && (EF & VE_DIV) && !(EF & VE_DUAL)), "VE_POST: the stage's final xs");
  int issued = 0, xmk = 0;
  RagWalk walk;
  auto tile_of = [&](int ti) __attribute__((always_inline)) {  // (utterance, first frame, valid frames) of tile ti
    const int tile = __builtin_amdgcn_readfirstlane(gl + ti * G);
    if (rag) return walk.at(rtc, rlv, a.B, BN, tile);
    RagTile t;
    t.b = tile / ntn;
    t.n0 = (tile - t.b * ntn) * BN;
    t.lv = L;
    return t;
  };
  RagTile nxt;  // the tile stage_x staged last (the next tile of the loop)
  // every tap of both convs from the generic packing [32 rows][k][32]: DMA j moves tap (j / 2) % k of conv
  // j / 2k, rows (j & 1) * 16 .. + 15
  auto stage_weights = [&]() {
    for (int j = wave; j < 4 * k; j += 8) {
      const int cv = j / (2 * k), t = (j >> 1) - cv * k, r = (j & 1) * 16 + lrow;
      const bf16* w = cv ? a.w2 : a.w1;
      glds16(w + ((size_t)r * k + t) * C + (lp ^ swz(r)) * 8, smem + W_OFF + (cv * k + t) * TAPW + (j & 1) * 1024);
      ++issued;
    }
  };
  // raw rows of tile ti: row r = frame n0 - HALO2 - h1 + r (zero rows past this workgroup's last tile)
  // VP32_BUF: this lane's byte offset within a 16-row piece (row lrow, 16-byte chunk lp ^ swz(row); a piece starts
  // at a multiple of 16 rows, so swz(row) = swz(lrow))
  const int xlane = lrow * RB + ((lp ^ swz(lrow)) * 16);
  auto stage_x = [&](int ti) __attribute__((always_inline)) {
    nxt = tile_of(ti);
    if constexpr (VP32_BUF) {
      // the utterance as a buffer of its lv valid frames (past the workgroup's last tile: an empty one, zero rows):
      // row r = frame f0 + r at byte offset (f0 + r) * RB; negative offsets wrap past num_records, so the range
      // check reads the conv's zero padding on both sides; rows past R1 are staged too and never read
      const int b = __builtin_amdgcn_readfirstlane(nxt.b);
      const int f0 = __builtin_amdgcn_readfirstlane(nxt.n0 - HALO2 - h1);
      const unsigned nrec = ti < nmine ? (unsigned)__builtin_amdgcn_readfirstlane(nxt.lv) * RB : 0u;
      const auto xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x + (size_t)b * L * C), (short)0, (int)nrec,
                                                        0x00020000);
#pragma unroll
      for (int i = 0; i < XROWS / 128; ++i) {
        const int j = wave + 8 * i;
        __builtin_amdgcn_raw_ptr_buffer_load_lds(xr, (__attribute__((address_space(3))) void*)(smem + j * 1024), 16,
                                                 (unsigned)(xlane + (f0 + 16 * j) * RB), 0, 0, 0);
      }
      issued += XROWS / 128;
      xmk = issued;
      return;
    }
    const bool live = ti < nmine;
    const bf16* xb = a.x + (size_t)(live ? nxt.b : 0) * L * C;
    const int f0 = nxt.n0 - HALO2 - h1, R1 = live ? NF1 + 2 * h1 : 0, lv = nxt.lv;
#pragma unroll
    for (int i = 0; i < XROWS / 128; ++i) {
      const int j = wave + 8 * i;
      const int r = 16 * j + lrow;
      const int q = lp ^ swz(r);
      const int f = f0 + r;
      const bool ok = r < R1 && f >= 0 && f < lv;
      glds16(ok ? xb + (size_t)f * C + q * 8 : a.zero + q * 8, smem + j * 1024);
    }
    issued += XROWS / 128;
    xmk = issued;
  };

  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };

  f32x4 acc[2][FN];
  struct Frag {
    bf16x8 A[2], B[FN];
  };
  // tap t of conv cv: A = the tap's 2 row fragments, B = FN frame fragments at rows rb0 + 16 fn
  auto read_frag = [&](Frag& F, int cv, int t, const char* src, int rb0) __attribute__((always_inline)) {
    const char* pa = smem + W_OFF + (cv * k + t) * TAPW + l16 * RB + ((g4 ^ swz(l16)) * 16);
#pragma unroll
    for (int f = 0; f < 2; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 16 * RB);
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int rb = rb0 + fn * 16;
      F.B[fn] = *reinterpret_cast<const bf16x8*>(src + rb * RB + ((g4 ^ swz(rb)) * 16));
    }
  };
  // 2 x FN MFMAs of one tap with the reads of another tap interleaved, one per MFMA issue slot; the first tap of
  // a conv starts the accumulators from the MFMA's zero C operand (no accumulator-zeroing moves)
  auto mma_tap = [&](const Frag& F, auto first) __attribute__((always_inline)) {
#pragma unroll
    for (int fm = 0; fm < 2; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn)
        acc[fm][fn] = mfma16(F.A[fm], F.B[fn], decltype(first)::value ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn]);
    constexpr int NR = 2 + FN, NMF = 2 * FN;
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NR, 0);
  };
  // one conv over `src` (row of tap t for this lane's first fragment: rb0 + t * tstride), taps ascending, each
  // tap's fragments read under the previous tap's MFMAs; no barrier inside (weights resident, `src` published)
  Frag F0, F1;
  auto conv = [&](int cv, const char* src, int rb0, int tstride) __attribute__((always_inline)) {
    read_frag(F0, cv, 0, src, rb0);
    read_frag(F1, cv, 1, src, rb0 + tstride);  // k >= 3 (odd)
    mma_tap(F0, std::true_type{});
    for (int t = 1; t < k; t += 2) {  // taps t (in F1) and t + 1 (into F0)
      read_frag(F0, cv, t + 1, src, rb0 + (t + 1) * tstride);
      mma_tap(F1, std::false_type{});
      if (t + 2 < k) read_frag(F1, cv, t + 2, src, rb0 + (t + 2) * tstride);
      mma_tap(F0, std::false_type{});
    }
  };

  // ---- prologue: the weights, then the first tile's rows (the first row wait covers both) ----
  stage_weights();
  stage_x(0);

  const float* par = reinterpret_cast<const float*>(smem + PAR_OFF);
  const int ch16 = (g4 & 1) * 16 + (g4 >> 1) * 8;  // this lane's 8 channels after the fragment swap
  const int qc = (g4 & 1) * 2 + (g4 >> 1);         // ... as a 16-byte chunk index
  VP_TS_DECL
  for (int ti = 0; ti < nmine; ++ti) {
    const int b = nxt.b, n0 = nxt.n0;  // staged by the previous stage_x (tile ti)
    const int Lt = nxt.lv;             // this utterance's frames (conv2's zero padding starts there)
    // ---- 1. the residual rows of this lane's outputs (output frame n0 + i = raw row i + HALO2 + h1), then
    // the in-place lrelu of the landed raw rows ----
    VP_TS(10);
    wait_vmcnt(issued - xmk);
    VP_TS(0);
    barrier();
    VP_TS(1);
    u32x4 rv[FN], yv[FN];  // residual x and (VE_ACCUM) old xs of this lane's outputs
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int r = wave * WNC + fn * 16 + l16 + HALO2 + h1 - PS;
      rv[fn] = *reinterpret_cast<const u32x4*>(smem + r * RB + ((qc ^ swz(r)) * 16));
    }
    barrier();
    VP_TS(2);
#pragma unroll
    for (int i = 0; i < XBUF / 16 / NT; ++i) {
      const int e = tid + i * NT;
      u32x4 v = *reinterpret_cast<const u32x4*>(smem + e * 16);
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = lrelu_pk(v[w], a.slope);
      *reinterpret_cast<u32x4*>(smem + e * 16) = v;
    }
    barrier();  // activated rows published
    VP_TS(3);
    // ---- 2. conv1 ----
    int ymk = 0;
    // VE_ACCUM: the old-xs rows of this tile's outputs, loaded now and consumed after conv2. Issued as asm so that
    // the counted wait below retires them: hipcc drains EVERY in-flight LDS-DMA (vmcnt(0)) before the use of a
    // compiler-visible load result, which would expose the next tile's row staging at each epilogue.
    if constexpr ((EF & VE_ACCUM) != 0) {
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int i = min(max(n0 - PS + wave * WNC + fn * 16 + l16, 0), L - 1);
        asm volatile("global_load_dwordx4 %0, %1, off"
                     : "=v"(yv[fn])
                     : "v"(a.y + ((size_t)b * L + i) * C + ch16)
                     : "memory");
      }
      issued += FN;
      ymk = issued;
    }
    conv(0, smem, wave * WNC + l16, d);
    VP_TS(4);
    // epilogue: lrelu(round(acc + b1)) -> T row j (frame n0 - HALO2 + j), zero outside [0, L)
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int j = wave * WNC + fn * 16 + l16;
      const int f = n0 - HALO2 + j;
      const bool ok = f >= 0 && f < Lt;
      uint32_t o[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + h * 16 + 4 * g4);
        // lrelu(acc + b1) rounded once to bf16 (conv2's operand); zero outside [0, L)
        o[h][0] = ok ? lrelu_pk_f(f32x2{acc[h][fn][0], acc[h][fn][1]} + f32x2{b4[0], b4[1]}, a.slope) : 0u;
        o[h][1] = ok ? lrelu_pk_f(f32x2{acc[h][fn][2], acc[h][fn][3]} + f32x2{b4[2], b4[3]}, a.slope) : 0u;
      }
      swap16(o[0][0], o[1][0]);
      swap16(o[0][1], o[1][1]);
      *reinterpret_cast<u32x4*>(smem + T_OFF + j * RB + ((qc ^ swz(j)) * 16)) = u32x4{o[0][0], o[0][1], o[1][0], o[1][1]};
    }
    VP_TS(5);
    // ---- 3. conv2 ----
    barrier();  // T published; every wave is past conv1's reads of the row buffer: stage the next tile's rows
    stage_x(ti + 1);
    VP_TS(6);
    conv(1, smem + T_OFF, wave * WNC + l16 + HALO2 - h2 - PS, 1);
    VP_TS(7);
    // epilogue: + b2 + x [+ xs] [/ nk] -> y [, lrelu(y) -> y2]
    if constexpr ((EF & VE_ACCUM) != 0) {
      wait_vmcnt(issued - ymk);
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) asm volatile("" : "+v"(yv[fn]));  // no use of yv before the wait
    }
    VP_TS(8);
    static_assert(BN == 8 * WNC - 16, "only the last wave's last fragment lies past BN");
    const int bu = __builtin_amdgcn_readfirstlane(b);
    const auto yr = __builtin_amdgcn_make_buffer_rsrc(a.y + (size_t)bu * L * C, (short)0, (int)((unsigned)L * RB), 0x00020000);
    const auto y2r = __builtin_amdgcn_make_buffer_rsrc(((EF & VE_DUAL) ? a.y2 : a.y) + (size_t)bu * L * C, (short)0,
                                                       (int)((unsigned)L * RB), 0x00020000);
    if constexpr (POST) barrier();  // every wave is past conv2's reads of T: xs replaces it as conv_post's input
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) {
      const int i = wave * WNC + fn * 16 + l16;  // output frame n0 - PS + i
      uint32_t rx0 = rv[fn][0], rx1 = rv[fn][1], ry0 = rv[fn][2], ry1 = rv[fn][3];
      swap16(rx0, ry0);  // back to the accumulator layout
      swap16(rx1, ry1);
      uint32_t yx0 = 0, yx1 = 0, yy0 = 0, yy1 = 0;
      if constexpr ((EF & VE_ACCUM) != 0) {
        yx0 = yv[fn][0], yx1 = yv[fn][1], yy0 = yv[fn][2], yy1 = yv[fn][3];
        swap16(yx0, yy0);
        swap16(yx1, yy1);
      }
      uint32_t o1[2][2], o2[2][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const f32x4 b4 = *reinterpret_cast<const f32x4*>(par + C + h * 16 + 4 * g4);
        const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
        const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
        // round(acc + b2 + x [+ xs] [/ nk]) and its lrelu, two channels per packed op
#pragma unroll
        for (int u = 0; u < 2; ++u) {
          f32x2 v = f32x2{acc[h][fn][2 * u], acc[h][fn][2 * u + 1]} + f32x2{b4[2 * u], b4[2 * u + 1]};
          v = v + unpk_bf16(rr[u]);
          if constexpr ((EF & VE_ACCUM) != 0) v = unpk_bf16(yy[u]) + v;
          if constexpr ((EF & VE_DIV) != 0) v = f32x2{div_rn(v.x, a.div, 1.f / a.div), div_rn(v.y, a.div, 1.f / a.div)};
          o1[h][u] = pk_bf16(v);
          o2[h][u] = lrelu_pk(o1[h][u], a.slope);  // the stored state's activated copy
        }
      }
      swap16(o1[0][0], o1[1][0]);
      swap16(o1[0][1], o1[1][1]);
      if constexpr (POST) {
        // conv_post's input v = bf16(lrelu(xs, 0.01)) of frame n0 - 3 + i into T row i (zero outside the utterance:
        // conv_post's zero padding), the layout post_taps reads
        const int f = n0 - PS + i;
        const bool in = f >= 0 && f < Lt;
        u32x4 v = {0u, 0u, 0u, 0u};
        if (in) v = u32x4{lrelu_pk(o1[0][0], a.post_slope), lrelu_pk(o1[0][1], a.post_slope),
                          lrelu_pk(o1[1][0], a.post_slope), lrelu_pk(o1[1][1], a.post_slope)};
        *reinterpret_cast<u32x4*>(smem + T_OFF + i * RB + ((qc ^ swz(i)) * 16)) = v;
        continue;
      }
      if constexpr (VP32_BUF) {
        // the utterance's [L][C] output as a buffer: frames past L fall outside it (store dropped); the discarded
        // frames i >= BN of the last wave's last fragment get an offset past any range (every lane still stores, so
        // the issue counts are unchanged)
        const bool keep = !(fn == FN - 1 && wave == 7);
        const unsigned vo = keep ? (unsigned)(((n0 + i) * C + ch16) * 2) : 0x80000000u;
        __builtin_amdgcn_raw_buffer_store_b128(u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]}, yr, vo, 0, 0);
        if constexpr ((EF & VE_DUAL) != 0) {
          swap16(o2[0][0], o2[1][0]);
          swap16(o2[0][1], o2[1][1]);
          __builtin_amdgcn_raw_buffer_store_b128(u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]}, y2r, vo, 0, 0);
        }
        continue;
      }
      const bool ok = i < BN && n0 + i < L;
      const size_t o = ((size_t)b * L + n0 + i) * C + ch16;
      *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
      if constexpr ((EF & VE_DUAL) != 0) {
        swap16(o2[0][0], o2[1][0]);
        swap16(o2[0][1], o2[1][1]);
        *reinterpret_cast<u32x4*>(ok ? a.y2 + o : a.trash + 8 * lane) = u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]};
      }
    }
    if constexpr (POST) {
      // conv_post of the tile's BN frames (post_taps / post_combine: 6 blocks of 16 per wave), tanh(. + bias), the
      // waveform stored (frames past the utterance: 0, as post_conv_kernel; past L or BN: dropped by the range check)
      barrier();
      const float* wbase = a.wav + (size_t)bu * L;
      const auto wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), (short)0, (int)((unsigned)L * 4), 0x00020000);
      // conv_post's A operand fetched here (cache-resident) rather than held through the tile loop (VGPR pressure)
      const bf16x8 wt = post_wtaps(a.post_w, lane);
      const float pb = a.post_b[0];
      // the blocks' sums sit in lanes 0..15 of each result: up to 4 blocks gathered into one register (16-lane row
      // q = block 4 g + q, by permlane16 / permlane32 swaps) so tanh runs once per 64 outputs, one store per group
      static_assert(FN == 6, "two groups of blocks: 4 + 2");
      float sv[FN];
      f32x4 dp = post_taps(smem + T_OFF, wave * WNC, wt, lane);
#pragma unroll
      for (int fb = 0; fb < FN; ++fb) {  // rows up to wave * WNC + WNC + 15 < TROWS
        const f32x4 dn = post_taps(smem + T_OFF, wave * WNC + (fb + 1) * 16, wt, lane);
        sv[fb] = post_combine(dp, dn, lane);
        dp = dn;
      }
      auto gather = [&](float b0, float b1, float b2, float b3) __attribute__((always_inline)) {
        uint32_t x0 = __float_as_uint(b0), x1 = __float_as_uint(b1), x2 = __float_as_uint(b2), x3 = __float_as_uint(b3);
        swap16(x0, x1);  // x0 rows: (b0, b1, ., .)
        swap16(x2, x3);  // x2 rows: (b2, b3, ., .)
        const auto r = __builtin_amdgcn_permlane32_swap(x0, x2, false, false);
        return __uint_as_float(r[0]);  // rows (b0, b1, b2, b3)
      };
#pragma unroll
      for (int grp = 0; grp < 2; ++grp) {
        const float g = grp == 0 ? gather(sv[0], sv[1], sv[2], sv[3]) : gather(sv[4], sv[5], 0.f, 0.f);
        const int o = wave * WNC + grp * 64 + lane;  // output frame n0 + o
        const float th = post_tanh(g + pb), val = n0 + o < Lt ? th : 0.f;
        const bool live = (grp == 0 || lane < 32) && o < BN;
        __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(val), wr, live ? (unsigned)((n0 + o) * 4) : 0x80000000u, 0, 0);
      }
    }
    issued += POST ? 2 : FN * ((EF & VE_DUAL) ? 2 : 1);
    VP_TS(9);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the trailing row / weight DMAs land before LDS is freed
  VP_TS(11);
  VP_TS_END(wave, lane);
}

bool vpair32_supported(int k, int d) {
  return k >= 3 && k % 2 == 1 && k <= KMAX && (k - 1) / 2 <= HALO2 && NF1 + d * (k - 1) <= XROWS;
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_vpair32(int ef, const VPairArgs& a, hipStream_t st) {
  MT_REQUIRE(!(ef & VE_DIV) || div_rn_ok(a.div), "vpair32: VE_DIV divisor %g outside the exactly-checked set (div_rn)", (double)a.div);
  ef &= ~VE_Y2ONLY;  // stores y as well (VE_Y2ONLY is an option, mt_vconv.h)
  MT_REQUIRE(a.x && a.w1 && a.w2 && a.b1 && a.b2 && a.y && a.zero && a.trash && a.B > 0 && a.L > 0,
             "vpair32: null argument / empty");
  MT_REQUIRE(vpair32_supported(a.taps, a.dil) && a.taps % 2 == 1, "vpair32: k %d d %d", a.taps, a.dil);
  MT_REQUIRE(!(ef & VE_DUAL) || a.y2, "vpair32: y2");
  MT_REQUIRE(!(ef & VE_POST) || (a.post_w && a.post_b && a.wav && (ef & ~VE_POST) == (VE_ACCUM | VE_DIV) &&
                                 (a.taps - 1) / 2 + 3 <= HALO2),
             "vpair32: VE_POST needs conv_post's weights, bias and the waveform, the stage's final (ACCUM | DIV) pair "
             "and k <= %d", 2 * (HALO2 - 3) + 1);
  MT_REQUIRE(a.y != a.x, "vpair32: y must not alias x (neighbour tiles read x's halo)");
  const long ntiles = (long)a.B * ((a.L + BN - 1) / BN);
  const int G = (int)std::min<long>(ntiles, cu_count());
  const double flops = 2.0 * 2.0 * C * C * a.taps * (double)a.B * a.L;
  const double bytes = 2.0 * (2.0 * 2.0 * C * (double)a.B * a.L) + 2.0 * 2.0 * C * C * a.taps;
  probe_begin(PROBE_VCONV, st);
  switch (ef) {
    case 0: hipLaunchKernelGGL((vpair32_kernel<0>), dim3(G), dim3(NT), 0, st, a); break;
    case VE_ACCUM: hipLaunchKernelGGL((vpair32_kernel<VE_ACCUM>), dim3(G), dim3(NT), 0, st, a); break;
    case VE_ACCUM | VE_DIV: hipLaunchKernelGGL((vpair32_kernel<VE_ACCUM | VE_DIV>), dim3(G), dim3(NT), 0, st, a); break;
    case VE_ACCUM | VE_DIV | VE_DUAL:
      hipLaunchKernelGGL((vpair32_kernel<VE_ACCUM | VE_DIV | VE_DUAL>), dim3(G), dim3(NT), 0, st, a);
      break;
    case VE_DIV: hipLaunchKernelGGL((vpair32_kernel<VE_DIV>), dim3(G), dim3(NT), 0, st, a); break;
    case VE_DIV | VE_DUAL: hipLaunchKernelGGL((vpair32_kernel<VE_DIV | VE_DUAL>), dim3(G), dim3(NT), 0, st, a); break;
    case VE_ACCUM | VE_DIV | VE_POST:
      hipLaunchKernelGGL((vpair32_kernel<VE_ACCUM | VE_DIV | VE_POST>), dim3(G), dim3(NT), 0, st, a);
      break;
    default: set_error("vpair32: epilogue %d not compiled in", ef); return -1;
  }
  MT_CHECK_HIP(hipGetLastError());
  probe_end(PROBE_VCONV, st, flops, bytes, PROBE_TAG_VPAIR32);
  const int rec[VCLOG_FIELDS] = {ef | 0x10000, C, BN, 0, (int)ntiles, G, a.taps, C, C, a.B, a.L};
  vclog_record(rec);
  return 0;
}

VP_TS_BINDER(vpair32_ts_bind)

}  // namespace mt
