// HiFi-GAN ResBlock1 convs of the wide stages (stage 1: C = 256 at 8T, stage 2: C = 128 at 64T; hifigan/models.py
// :90-97, 183-192) as a persistent LDS-DMA implicit GEMM whose K loop is scheduled at COMPILE time (gfx950, bf16).
//
// Same GEMM, tiles, staging images and MFMA order as mt_vconv's 128-row k >= 2 path (results are bit-identical to
// it), but specialised on (C_in = C_out = C, taps K): a tile's S = (C / 64) * K steps are unrolled, so every ring
// slot, row buffer, tap offset and `s_waitcnt vmcnt(N)` count is an immediate. mt_vconv carries those as
// wave-uniform runtime cursors: ~150 scalar instructions between a step's barrier and its MFMA block (a three-level
// vmcnt branch tree, cursor wrap-arounds, per-step tile decode), which both waves of a SIMD issue at the same time,
// so the MFMA pipe idles through them. Here a step is: one counted wait, one barrier, the step's
// LDS-DMA pieces (addresses: a per-tile base plus constants), 16 ds_read_b128 interleaved with 32 MFMAs per wave.
//
// Geometry (= mt_vconv BM 128, BN 256): 8 waves (2 along rows x 4 along frames, 64 x 64 each, FN = 4 fragments of 16
// frames, v_mfma_f32_16x16x32_bf16); a step = one (64-channel chunk c, tap t): a 16 KiB weight slot of a 4-slot ring
// (steps q+1 .. q+3 in flight behind step q) and the chunk's 256 + (K-1) d <= 320 input rows in one of two 40 KiB
// buffers (staged once per chunk at the chunk's first step, read by every tap shifted by t * d rows). Rows are 128 B
// with the 16-byte unit XOR-swizzled by (row & 6): conflict-free ds_read_b128 for every shift.
//
// Counted waits (VcSched, mt_vconv.h): the loader waves issue, per step and in program order, [the epilogue's residual
// / accumulator loads on a tile's last step] [row pieces of the next chunk on its first TX taps] [the weight pieces of
// step s + 3] [the epilogue stores on a tile's last step]; the data a wait needs was issued at step s - 2 (weights)
// or over the previous chunk's first taps (rows), so the operations issued after it are a compile-time function of
// the step's position in the tile. Tile 0's first waits count the prologue's staging instead (wait_first).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mt_probe.h"
#include "mt_ragged.h"
#include "mt_ts.h"
#include "mt_vconv.h"

#ifndef RB_ACTIN_NV
#define RB_ACTIN_NV 0  // VE_ACTIN pass step: VALU instructions scheduled after each MFMA
#endif

#ifndef RB_RAGWALK
#define RB_RAGWALK 1  // ragged tile lookup: 1 the incremental walk (mt_ragged.h RagWalk), 0 a binary search per tile
#endif

#ifndef RB_EPI_AT
#define RB_EPI_AT 2  // the step (counted from the tile's end) that issues the epilogue's loads
#endif

#ifndef RB_DMA_AT
#define RB_DMA_AT 1  // where a step's loader DMA issue sits: 0 after the barrier, 1 between its K-slices, 2 after both
#endif

#ifndef RB_BUF
#define RB_BUF 7  // bits: LDS-DMA of 1 the weights, 2 the rows, 4 the epilogue stores through buffer resources (SGPR
                  // bases: no per-piece 64-bit address VALU; zero padding rows and frames past L by the range check
                  // instead of compares / selects)
#endif

#ifndef RB_LMAX
#define RB_LMAX 1  // 1: the epilogue's lrelu as max(v, slope v) (IEEE mode off; equal to the compare / select form on
                   // non-NaN values, which mt_vconv uses)
#endif

#ifndef RB_EXP
#define RB_EXP 0  // timing experiments (tools/exp_build.sh, tools/rblab): bits drop parts of the work (wrong results):
                  // 1 epilogue operand loads, 2 the y2 store, 4 the K loop's DMA issue, 8 its step barriers, 16 MFMAs
#endif

namespace mt {

namespace {
constexpr int RBM = 128, RBN = 256, RNT = 512;
constexpr int RWSLOT = RBM * 128;           // 128 rows x 64 bf16 channels
constexpr int RNW = 4;                       // weight ring slots
constexpr int RXROWS = RBN + 64;             // staged rows per chunk (256 frames + halo <= 64)
constexpr int RXBUF = RXROWS * 128;
constexpr int RX_OFF = RNW * RWSLOT;
constexpr int RBIAS_OFF = RX_OFF + 2 * RXBUF;
constexpr int RRAG_OFF = RBIAS_OFF + 256 * 4;
constexpr int RLDS = RRAG_OFF + RAG_LDS;
static_assert(RLDS <= 160 * 1024, "LDS budget");
constexpr int RFN = 4, RWNC = 64;

// Staging by LW loader waves (waves 0 .. LW-1; with LW = 4 one per SIMD, so the other wave of each SIMD never
// stalls on DMA issue): per step WPW weight pieces each, per chunk XPW row pieces each, spread over the chunk's first
// TX steps (>= 2 steps before they are needed). Counted waits: VcSched (mt_vconv.h).
template <int LW>
struct RbStage {
  static constexpr int WPW = 16 / LW, XPW = 40 / LW;
};
template <int K, int LW>
constexpr int rb_tx() {
  const int t = K - 2 < 1 ? 1 : K - 2;
  return t < RbStage<LW>::XPW ? t : RbStage<LW>::XPW;
}
template <int EF>
constexpr int rb_nst() {  // the epilogue's stores per wave and tile
  return 2 * RFN * ((EF & VE_DUAL) && !(EF & VE_Y2ONLY) ? 2 : 1);
}

}  // namespace

__device__ __forceinline__ void rb_glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

__device__ __forceinline__ void rb_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

// compile-time loop: f(integral_constant<int, I>) for I in [0, N)
template <int I, int N, class F>
__device__ __forceinline__ void rb_for(F&& f) {
  if constexpr (I < N) {
    f(std::integral_constant<int, I>{});
    rb_for<I + 1, N>(f);
  }
}

template <int EF, int C, int K, int LW>
__global__ __launch_bounds__(RNT) void rbconv_kernel(VConvArgs a) {
  constexpr int WPW = RbStage<LW>::WPW, XPW = RbStage<LW>::XPW, TX = rb_tx<K, LW>();
  constexpr bool ACTIN = (EF & VE_ACTIN) != 0;
  using SCH = VcSched<C / 64, K, RNW, 2, TX, WPW, XPW, rb_nst<EF>(), ACTIN ? 2 : 1>;
  constexpr int NCH = C / 64, S = NCH * K;        // chunks, steps per tile
  static_assert(NCH % 2 == 0 && S % 2 == 0, "schedule period (row buffers alternate per chunk)");
  constexpr int NTM = C / RBM;                    // row tiles
  __shared__ __attribute__((aligned(1024))) char smem[RLDS];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int dil = a.dil, L = a.L;
  const int ntn = (L + RBN - 1) / RBN;
  const bool rag = a.lens != nullptr;
  int* rtc = reinterpret_cast<int*>(smem + RRAG_OFF);
  int* rlv = rtc + RAG_MAXB;
  if (rag) rag_build(rtc, rlv, a.lens, a.lmul, L, 0, L, a.B, RBN, tid);
  for (int i = tid; i < C; i += RNT) reinterpret_cast<float*>(smem + RBIAS_OFF)[i] = a.bias[i];
  __syncthreads();
  // (read once into a scalar: everything derived from it — the tile walk included — then stays scalar)
  const int ntiles = __builtin_amdgcn_readfirstlane(rag ? rtc[a.B - 1] * NTM : a.B * ntn * NTM);
  // tile ownership: mt_vconv's (XCD-major on grids of <= 3 rounds, else the XCD-grouped round-robin walk)
  const int G = gridDim.x, g = blockIdx.x;
  const int xcd = g & 7, lw = g >> 3;
  const int gx = (G - xcd + 7) >> 3;
  const int sx = xcd * (G >> 3) + min(xcd, G & 7);
  const int xt0 = (int)((long)ntiles * sx / G), xt1 = (int)((long)ntiles * (sx + gx) / G);
  const bool xmaj = a.xcd_tiles != 0;
  const int gl = xmaj ? xt0 + lw : (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int gstep = xmaj ? gx : G;
  const int nmine = xmaj ? (gl < xt1 ? (xt1 - gl + gx - 1) / gx : 0) : (gl < ntiles ? (ntiles - gl + G - 1) / G : 0);
  if (nmine == 0) return;

  struct Tile {
    int b, n0, m0, lx;  // lx: the utterance's valid frames (ragged), read from the LDS table once per tile
  };
  RagWalk walk;  // RB_RAGWALK: the workgroup's rows r only increase (tile_of(ti) is called for ti = 0, 1, 2, ...)
  auto tile_of = [&](int ti) __attribute__((always_inline)) {
    Tile tl;
    // past the last tile: the last one (phantom prefetches); a scalar, so the utterance walk below is a scalar loop
    const int tile = __builtin_amdgcn_readfirstlane(gl + min(ti, nmine - 1) * gstep);
    const int r = tile / NTM;
    tl.m0 = (tile - r * NTM) * RBM;
    if (rag) {
#if RB_RAGWALK
      const RagTile rt = walk.at(rtc, rlv, a.B, RBN, r);
      tl.b = rt.b, tl.n0 = rt.n0, tl.lx = rt.lv;
#else
      tl.b = rag_find(rtc, a.B, r);
      tl.n0 = (r - rag_first(rtc, tl.b)) * RBN;
      tl.lx = rlv[tl.b];
#endif
    } else {
      tl.b = r / ntn;
      tl.n0 = (r - tl.b * ntn) * RBN;
      tl.lx = L;
    }
    // wave-uniform by construction; said so, so that the buffer resources built from them stay scalar (a resource
    // the compiler thinks may vary per lane costs a readfirstlane loop per DMA)
    tl.b = __builtin_amdgcn_readfirstlane(tl.b);
    tl.n0 = __builtin_amdgcn_readfirstlane(tl.n0);
    tl.m0 = __builtin_amdgcn_readfirstlane(tl.m0);
    tl.lx = __builtin_amdgcn_readfirstlane(tl.lx);
    return tl;
  };

  const int lrow = lane >> 3, lp = lane & 7;
  const bool loader = wave < LW;
  // weight piece i of a loader wave: row r of the 128-row slot, 16-byte unit q (swizzled on the source address)
  int woff[WPW];
#pragma unroll
  for (int i = 0; i < WPW; ++i) {
    const int r = 8 * (wave * WPW + i) + lrow;
    woff[i] = r * 128 + ((lp ^ (r & 6)) * 16);
  }
  const char* wbase = reinterpret_cast<const char*>(a.w);
  const auto wrsrc = buf_rsrc(a.w, (unsigned)(C * C * K * 2));  // the whole [C/64][K][C][64] image
  auto issue_w = [&](const Tile& tl, int c, int t, int slot) __attribute__((always_inline)) {
    // the LDS destination goes through an opaque copy: with a known constant offset the compiler tracks the DMA's
    // LDS range and puts a vmcnt wait before every ds_read it cannot prove disjoint (all of them), draining the
    // prefetch each step; the ordering is ours (counted waits + barrier)
    int so = slot * RWSLOT + wave * WPW * 1024;
    asm volatile("" : "+s"(so));
    if constexpr ((RB_BUF & 1) != 0) {
      // the step's block (chunk c, tap t, rows m0 ..) as the scalar offset; each piece's lane offset is fixed
      const unsigned sof = (unsigned)(((c * K + t) * C + tl.m0) * 128);
#pragma unroll
      for (int i = 0; i < WPW; ++i) buf_lds16(wrsrc, (unsigned)woff[i], sof, smem + so + i * 1024);
    } else {
      const char* base = wbase + ((size_t)(c * K + t) * C + tl.m0) * 128;
#pragma unroll
      for (int i = 0; i < WPW; ++i) {
        int wo = woff[i];
        asm volatile("" : "+v"(wo));  // per-step address (see read_frag)
        rb_glds16(base + wo, smem + so + i * 1024);
      }
    }
  };
  const int R = RBN + (K - 1) * dil;
  // RB_BUF: this lane's byte offset within a row piece (row lrow, swizzled 16-byte unit lp ^ (row & 6); a piece's 8
  // rows start at a multiple of 8, so row & 6 = lrow & 6)
  const int xlane = lrow * C * 2 + ((lp ^ (lrow & 6)) * 16);
  // the row pieces i (of this loader wave's XPW) with i * TX / XPW == part, of chunk c of a tile
  auto issue_x = [&](const Tile& tl, int c, int buf, auto partc) __attribute__((always_inline)) {
    constexpr int part = decltype(partc)::value;
    const int f0 = tl.n0 - a.pad;
    const int Lx = tl.lx;
    const char* xb = reinterpret_cast<const char*>(a.x) + ((size_t)tl.b * L * C + c * 64) * 2;
    int xo = RX_OFF + buf * RXBUF;
    asm volatile("" : "+s"(xo));  // opaque LDS destination (see issue_w)
    char* dst = smem + xo;
    if constexpr ((RB_BUF & 2) != 0) {
      // the utterance's chunk-c columns as a buffer of its Lx valid frames: row r = frame f0 + r at byte offset
      // (f0 + r) * 2C + 16 q, where negative offsets (f < 0) wrap past num_records, so the range check reads the
      // conv's zero padding on both sides; rows past R are read too (in range or zero) and never used
      const auto xr = buf_rsrc(xb, (unsigned)Lx * (unsigned)(C * 2));
#pragma unroll
      for (int i = 0; i < XPW; ++i) {
        if (i * TX / XPW != part) continue;
        const int j = wave + LW * i;
        buf_lds16(xr, (unsigned)(xlane + (f0 + 8 * j) * C * 2), 0u, dst + j * 1024);
      }
    } else {
#pragma unroll
      for (int i = 0; i < XPW; ++i) {
        if (i * TX / XPW != part) continue;
        const int j = wave + LW * i;
        const int r = 8 * j + lrow;
        const int q = lp ^ (r & 6);
        const int f = f0 + r;
        const bool ok = r < R && f >= 0 && f < Lx;
        const char* src = ok ? xb + (size_t)f * C * 2 + q * 16 : reinterpret_cast<const char*>(a.zero) + q * 16;
        rb_glds16(src, dst + j * 1024);
      }
    }
  };

  f32x4 acc[4][RFN];  // a tile's first K-slice starts from the MFMA's zero C operand (no zeroing pass)

  const int g4 = lane >> 4, l16 = lane & 15;
  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  const int ch16 = wm * 64 + (g4 & 1) * 16 + (g4 >> 1) * 8;
  u32x4 rv[2][RFN], yv[2][RFN];
  // epilogue operand loads of a tile (issued at the start of its last step, consumed after its MFMAs)
  auto epi_loads = [&](const Tile& tl) __attribute__((always_inline)) {
    const size_t rowbase = (size_t)tl.b * L;
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < RFN; ++fn) {
        const int n = min(tl.n0 + wn * RWNC + fn * 16 + l16, L - 1);
        const size_t o = (rowbase + n) * C + tl.m0 + ch16 + fp * 32;
        if constexpr ((RB_EXP & 1) != 0) {  // timing experiment 1: no epilogue operand loads (wrong results)
          rv[fp][fn] = yv[fp][fn] = u32x4{(uint32_t)o, 0u, 0u, 0u};
          continue;
        }
        if constexpr ((EF & VE_RESID) != 0) rv[fp][fn] = *reinterpret_cast<const u32x4*>(a.resid + o);
        if constexpr ((EF & VE_ACCUM) != 0) yv[fp][fn] = *reinterpret_cast<const u32x4*>(a.y + o);
      }
  };
  // mt_vconv's packed epilogue (bias, + residual, + old accumulator, / div, then lrelu / dual outputs), the same
  // operations in the same order; every lane stores (frames past L go to the trash line): RNST per tile
  auto epilogue = [&](const Tile& tl, bool real) __attribute__((always_inline)) {
    // RB_BUF: the utterance's [L][C] rows of y / y2 from the tile's channel m0 on (in the base, not as a scalar
    // offset: the range check then drops exactly the frames n >= L)
    const unsigned ylim = (unsigned)L * (unsigned)(C * 2) - (unsigned)(tl.m0 * 2);
    const auto yr = buf_rsrc(a.y + (size_t)tl.b * L * C + tl.m0, ylim);
    const auto y2r = buf_rsrc(((EF & VE_DUAL) ? a.y2 : a.y) + (size_t)tl.b * L * C + tl.m0, ylim);
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < RFN; ++fn) {
        uint32_t rx0 = 0, rx1 = 0, ry0 = 0, ry1 = 0, yx0 = 0, yx1 = 0, yy0 = 0, yy1 = 0;
        if constexpr ((EF & VE_RESID) != 0) {
          rx0 = rv[fp][fn][0], rx1 = rv[fp][fn][1], ry0 = rv[fp][fn][2], ry1 = rv[fp][fn][3];
          swap16(rx0, ry0);
          swap16(rx1, ry1);
        }
        if constexpr ((EF & VE_ACCUM) != 0) {
          yx0 = yv[fp][fn][0], yx1 = yv[fp][fn][1], yy0 = yv[fp][fn][2], yy1 = yv[fp][fn][3];
          swap16(yx0, yy0);
          swap16(yx1, yy1);
        }
        uint32_t o1[2][2], o2[2][2];
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const int m = tl.m0 + wm * 64 + fm * 16 + 4 * g4;
          const f32x4 bias4 = *reinterpret_cast<const f32x4*>(smem + RBIAS_OFF + 4 * m);
          const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
          const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            f32x2 v = f32x2{acc[fm][fn][2 * u], acc[fm][fn][2 * u + 1]} + f32x2{bias4[2 * u], bias4[2 * u + 1]};
            if constexpr ((EF & VE_RESID) != 0) v = v + unpk_bf16(rr[u]);
            if constexpr ((EF & VE_ACCUM) != 0) v = unpk_bf16(yy[u]) + v;
            if constexpr ((EF & VE_DIV) != 0) v = f32x2{div_rn(v.x, a.div, 1.f / a.div), div_rn(v.y, a.div, 1.f / a.div)};
            const uint32_t rb = pk_bf16(v);
            uint32_t av = 0u;
            if constexpr (RB_LMAX) av = (EF & VE_ACT) ? lrelu_pk_f(v, a.slope) : (EF & VE_DUAL) ? lrelu_pk(rb, a.slope) : 0u;
            else av = (EF & VE_ACT) ? lrelu_pk_f_sel(v, a.slope) : (EF & VE_DUAL) ? lrelu_pk_sel(rb, a.slope) : 0u;
            o1[h][u] = (EF & VE_ACT) ? av : rb;
            o2[h][u] = av;
          }
        }
        swap16(o1[0][0], o1[1][0]);
        swap16(o1[0][1], o1[1][1]);
        const int n = tl.n0 + wn * RWNC + fn * 16 + l16;
        if constexpr ((RB_BUF & 4) != 0) {
          // the utterance's [L][C] output as a buffer: frames past L fall outside the range (store dropped); every
          // lane still issues its store, so the counted waits' NST is unchanged
          const unsigned vo = (unsigned)((n * C + ch16 + fp * 32) * 2);
          if constexpr ((EF & VE_Y2ONLY) == 0)
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]}, yr, vo, 0, 0);
          if constexpr ((EF & VE_DUAL) != 0 && (RB_EXP & 2) == 0) {
            swap16(o2[0][0], o2[1][0]);
            swap16(o2[0][1], o2[1][1]);
            __builtin_amdgcn_raw_buffer_store_b128(u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]}, y2r, vo, 0, 0);
          }
          continue;
        }
        const bool ok = real && n < L;
        const size_t o = ((size_t)tl.b * L + n) * C + tl.m0 + ch16 + fp * 32;
        if constexpr ((EF & VE_Y2ONLY) == 0)
          *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        if constexpr ((EF & VE_DUAL) != 0 && (RB_EXP & 2) == 0) {  // timing experiment 2: no y2 store
          swap16(o2[0][0], o2[1][0]);
          swap16(o2[0][1], o2[1][1]);
          *reinterpret_cast<u32x4*>(ok ? a.y2 + o : a.trash + 8 * lane) = u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]};
        }
      }
  };

  // fragments of one K-slice of a step: 4 A (weights) + 4 B (frames) x 16 bytes per lane
  struct Frag {
    bf16x8 A[4], B[RFN];
  };
  const int ha = l16 & 6;
  const char* pa0 = smem + (wm * 64 + l16) * 128;
  const int rbl = wn * RWNC + l16;  // this lane's B row before the tap shift
  // The per-lane fragment addresses of a step depend only on (slot, buffer, tap), so the compiler would compute
  // every step's once outside the tile loop and keep them all live (hundreds of VGPRs, scratch spills); the
  // opaque copies below make them per-step values (a handful of VALU each step).
  auto read_frag = [&](Frag& F, int ks, int slot, int xbuf, int tap) __attribute__((always_inline)) {
    int lb = rbl, la = 0;
    asm volatile("" : "+v"(lb), "+v"(la));
    const char* pa = pa0 + la + slot * RWSLOT;
    const int rb0 = lb + tap * dil;
    const int hb = rb0 & 6;
    const char* pb = smem + RX_OFF + xbuf * RXBUF + rb0 * 128;
    const int oa = ((ks * 4 + g4) ^ ha) * 16, ob = ((ks * 4 + g4) ^ hb) * 16;
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048 + oa);
#pragma unroll
    for (int f = 0; f < RFN; ++f) F.B[f] = *reinterpret_cast<const bf16x8*>(pb + f * 2048 + ob);
  };
  // VE_ACTIN: lrelu over a landed row buffer in place (the chain state as stored -> the conv's input), each thread
  // its own 16-byte units, so no wave waits for another; the next barrier publishes the result
  auto act_pass = [&](int buf) __attribute__((always_inline)) {
    int bo = RX_OFF + buf * RXBUF;
    asm volatile("" : "+v"(bo));
#pragma unroll
    for (int i = 0; i < RXBUF / 16 / RNT; ++i) {
      char* p = smem + bo + (tid + RNT * i) * 16;
      u32x4 v = *reinterpret_cast<const u32x4*>(p);
#pragma unroll
      for (int w = 0; w < 4; ++w) v[w] = lrelu_pk(v[w], a.slope);
      *reinterpret_cast<u32x4*>(p) = v;
    }
  };
  // NV > 0 (a VE_ACTIN pass step): NV VALU instructions placed after each MFMA, so the pass runs beside them
  auto mma_slice = [&](const Frag& F, auto nvc, auto firstc) {
    constexpr bool FIRST = decltype(firstc)::value;
    constexpr int NV = decltype(nvc)::value;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < RFN; ++fn) {
        if constexpr ((RB_EXP & 16) != 0) asm volatile("" : "+v"(acc[fm][fn]) : "v"(F.A[fm]), "v"(F.B[fn]));
        else acc[fm][fn] = mfma16(F.A[fm], F.B[fn], FIRST ? f32x4{0.f, 0.f, 0.f, 0.f} : acc[fm][fn]);
      }
    if constexpr (NV == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
        __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
      }
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    } else {
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);             // MFMA
        if (i < 8) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
        __builtin_amdgcn_sched_group_barrier(0x002, NV, 0);            // VALU
      }
    }
  };

  // ---- prologue: the virtual steps v0 .. -1 stage tile 0's chunk-0 rows (part t at tap t), weights of steps 0 .. 2
  // (phase stamps of the diagnostic build, tools/rblab: 0 wait, 1 barrier, 2 DMA issue, 3 MFMA block, 4 activation
  // pass, 5 epilogue, 6 tile head, 7 prologue, 11 drain)
  VP_TS_DECL
  Tile cur = tile_of(0), nxt = tile_of(1);
  if (loader) {
    vc_for<SCH::v0, 0>([&](auto vc) {
      constexpr int v = decltype(vc)::value;
      constexpr int t = SCH::md(v) % K;
      if constexpr (t < TX && SCH::vfloor(v) + 1 >= 0) issue_x(cur, 0, 0, std::integral_constant<int, t>{});
      if constexpr (v + RNW - 1 >= 0) issue_w(cur, (v + RNW - 1) / K, (v + RNW - 1) % K, v + RNW - 1);
    });
    if constexpr (ACTIN) vc_wait_vmcnt<0>();  // chunk 0's rows too (RL = 2: no step before step 0 publishes them)
    else vc_wait_vmcnt<SCH::wait_first(-1)>();
  }
  rb_barrier();
  if constexpr (ACTIN) {
    act_pass(0);
    rb_barrier();
  }
  Frag F0, F1;
  read_frag(F0, 0, 0, 0, 0);
  VP_TS(7);

  // ---- the tile loop: one unrolled tile per iteration. The ring slot of step s of tile ti is (ti * S + s) % 4: a
  // constant when S % 4 == 0 (C = 256), else (C = 128, S = 2K = 2 mod 4) the tile's parity adds 2 ----
  for (int ti = 0; ti < nmine; ++ti) {
    const int sb = (S % RNW == 0) ? 0 : (ti & 1) * 2;  // slot base of this tile
    rb_for<0, S>([&](auto uc) {
      constexpr int s = decltype(uc)::value;           // step in the tile
      constexpr int c = s / K, t = s % K;              // chunk, tap
      constexpr int xbuf = c % 2;
      constexpr int s1 = (s + 1) % S, c1 = s1 / K, t1 = s1 % K;  // step s + 1 (maybe the next tile's)
      constexpr int xbuf1 = c1 % 2;
      const int slot = (sb + s) & 3, slot1 = (sb + s + 1) & 3, slot3 = (sb + s + 3) & 3;
      // publish step s+1's data (its weights; its rows when it starts a chunk); every wave's reads of step s-1
      // are done, so its weight slot and (at a chunk's first step) the other row buffer may be restaged
      __builtin_amdgcn_sched_barrier(0);  // the waits stay after the previous step's MFMAs
      if constexpr (s > 0) VP_TS(3);
      if (loader) {
        if constexpr (SCH::wait_first(s) == SCH::wait(s)) {
          vc_wait_vmcnt<SCH::wait(s)>();
        } else {
          if (ti == 0) vc_wait_vmcnt<SCH::wait_first(s)>();
          else vc_wait_vmcnt<SCH::wait(s)>();
        }
      }
      // LDS reads still in flight here (the next step's first K-slice: its weight slot and row buffer) touch neither
      // what this step's DMAs overwrite (the slot of step s - 1, the row buffer of chunk c - 1) nor anything another
      // wave writes, so the barrier drains nothing; only the in-place activation pass (VE_ACTIN, at the step before)
      // writes LDS that other waves read after it
      if constexpr (ACTIN && t == K - 1) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      VP_TS(0);
      if constexpr ((RB_EXP & 8) == 0) rb_barrier();
      VP_TS(1);
      // the epilogue's residual / old-xs loads, RB_EPI_AT steps before the tile's last (compiler-visible loads: the
      // epilogue's use waits for them, the counted waits leave them out)
      if constexpr (s == S - RB_EPI_AT && (EF & (VE_RESID | VE_ACCUM)) != 0) epi_loads(cur);
      auto dma = [&]() __attribute__((always_inline)) {
        if (loader && (RB_EXP & 4) == 0) {
          if constexpr (t < TX) {  // rows of the next chunk (this tile's c + 1, or the next tile's chunk 0), part t
            if constexpr (c + 1 < NCH) issue_x(cur, c + 1, (c + 1) % 2, std::integral_constant<int, t>{});
            else issue_x(nxt, 0, 0, std::integral_constant<int, t>{});
          }
          // weights of step s + 3 (slot of step s - 1)
          constexpr int s3 = (s + 3) % S, c3 = s3 / K, t3 = s3 % K;
          if constexpr (s + 3 < S) issue_w(cur, c3, t3, slot3);
          else issue_w(nxt, c3, t3, slot3);
        }
      };
      if constexpr (RB_DMA_AT == 0) dma();
      VP_TS(2);
      read_frag(F1, 1, slot, xbuf, t);
      // VE_ACTIN: the next chunk's rows were published by this step's wait (RL = 2); activated here, published by the
      // next step's barrier, read from the step after it (or by this step's successor's prefetch)
      if constexpr (ACTIN && t == K - 2) {
        act_pass((c + 1) % 2);
        VP_TS(4);
      }
      using NVP = std::integral_constant<int, (ACTIN && t == K - 2) ? RB_ACTIN_NV : 0>;
      mma_slice(F0, NVP{}, std::integral_constant<bool, s == 0>{});
      if constexpr (RB_DMA_AT == 1) {
        __builtin_amdgcn_sched_barrier(0);
        dma();
        __builtin_amdgcn_sched_barrier(0);
      }
      read_frag(F0, 0, slot1, xbuf1, t1);
      mma_slice(F1, NVP{}, std::false_type{});
      if constexpr (RB_DMA_AT == 2) {
        __builtin_amdgcn_sched_barrier(0);
        dma();
      }
      if constexpr (s == S - 1) {
        // the epilogue after the MFMAs: nothing of it (e.g. a copy of a residual register, whose compiler wait is
        // vmcnt(0)) may be scheduled into the MFMA block
        __builtin_amdgcn_sched_barrier(0);
        VP_TS(3);
        epilogue(cur, true);
        VP_TS(5);
      }
    });
    cur = nxt;
    nxt = tile_of(ti + 2);
    VP_TS(6);
  }
  // the prefetches past the last tile (valid addresses, never read) must land before the workgroup's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  VP_TS(11);
  VP_TS_END(wave, lane);
}

namespace {
#ifndef RB_LOADERS
#define RB_LOADERS 4
#endif
template <int EF, int C, int K>
void rb_launch(int G, const VConvArgs& a, hipStream_t st) {
  // the kernel's schedule (as rbconv_kernel derives it), registered for the CPU schedule test; VE_ACTIN's prologue
  // waits for all of its staging (vmcnt(0))
  constexpr int LW = RB_LOADERS, WPW = RbStage<LW>::WPW, XPW = RbStage<LW>::XPW, TX = rb_tx<K, LW>();
  constexpr bool ACTIN = (EF & VE_ACTIN) != 0;
  using SCH = VcSched<C / 64, K, RNW, 2, TX, WPW, XPW, rb_nst<EF>(), ACTIN ? 2 : 1>;
  (void)SchedReg<1, C / 64, K, RNW, 2, TX, WPW, XPW, rb_nst<EF>(), ACTIN ? 2 : 1,
                 ACTIN ? 0 : SCH::wait_first(-1)>::reg;
  hipLaunchKernelGGL((rbconv_kernel<EF, C, K, RB_LOADERS>), dim3(G), dim3(RNT), 0, st, a);
}
// on by default; MT_RBCONV=0 in the environment or mt_vconv_set_rbconv(0): the generic mt_vconv kernel instead
int g_rb = -1;
int rb_knob() {
  if (g_rb < 0) {
    const char* e = getenv("MT_RBCONV");
    g_rb = e && e[0] == '0' ? 0 : 1;
  }
  return g_rb;
}
}  // namespace

namespace {
int g_actin = -1;
}
int rbconv_actin_on() {
  if (g_actin < 0) {
    const char* e = getenv("MT_ACTIN");
    g_actin = e && e[0] == '0' ? 0 : 1;
  }
  return g_actin && rb_knob();
}
int rbconv_actin_set(int enable) {
  const int prev = rbconv_actin_on() ? 1 : 0;
  g_actin = enable ? 1 : 0;
  return prev;
}

int rbconv_set(int enable) {
  const int prev = rb_knob();
  g_rb = enable ? 1 : 0;
  return prev;
}

// the HiFi-GAN wide-stage ResBlock convs: C_in = C_out in {128, 256}, K in {3, 7, 11}, stride 1, plain output
// (not placed), one source, the ResBlock epilogues, halo <= 64 rows
VP_TS_BINDER(rbconv_ts_bind)

// the RB_EXP value this file was built with (mt_build_experiments: nonzero = a timing-experiment build)
int rbconv_exp_flags() { return RB_EXP; }

bool rbconv_handles(int ef, const VConvArgs& a) {
  if (!rb_knob()) return false;
  const bool eps = ef == VE_ACT || ef == (VE_ACT | VE_ACTIN) || ef == (VE_RESID | VE_DUAL) || ef == VE_RESID || ef == (VE_RESID | VE_ACCUM) ||
                   ef == (VE_RESID | VE_ACCUM | VE_DIV) || ef == (VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL) ||
                   ef == (VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL | VE_Y2ONLY);
  return eps && !a.f32 && (a.cin == 128 || a.cin == 256) && a.M == a.cin && a.Mpad == a.M && a.c0 == a.cin &&
         (a.taps == 3 || a.taps == 7 || a.taps == 11) && a.dil >= 1 && RBN + (a.taps - 1) * a.dil <= RXROWS &&
         a.Lout == a.L && a.ldy == a.M && a.yshift == 0 && a.ylim == a.L * a.M && a.B <= RAG_MAXB;
}

int launch_rbconv(int ef, const VConvArgs& a, int G, hipStream_t st) {
#define MT_RB_K(E, C)                                   \
  switch (a.taps) {                                     \
    case 3: rb_launch<E, C, 3>(G, a, st); break;        \
    case 7: rb_launch<E, C, 7>(G, a, st); break;        \
    default: rb_launch<E, C, 11>(G, a, st); break;      \
  }
#define MT_RB_EF(E)                      \
  case E:                                \
    if (a.cin == 256) {                  \
      MT_RB_K(E, 256)                    \
    } else {                             \
      MT_RB_K(E, 128)                    \
    }                                    \
    break;
  switch (ef) {
    MT_RB_EF(VE_ACT)
    MT_RB_EF(VE_ACT | VE_ACTIN)
    MT_RB_EF(VE_RESID | VE_DUAL)
    MT_RB_EF(VE_RESID)
    MT_RB_EF(VE_RESID | VE_ACCUM)
    MT_RB_EF(VE_RESID | VE_ACCUM | VE_DIV)
    MT_RB_EF(VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL)
    MT_RB_EF(VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL | VE_Y2ONLY)
    default: set_error("rbconv: epilogue %d", ef); return -1;
  }
#undef MT_RB_EF
#undef MT_RB_K
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
