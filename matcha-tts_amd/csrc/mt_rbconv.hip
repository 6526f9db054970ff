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
// Counted waits: each wave issues, per step and in program order, [the epilogue's residual / accumulator loads on a
// tile's last step] [5 row pieces on a chunk's first step] [2 weight pieces] [the epilogue stores on a tile's last
// step]. The step-(q+1) data a wait needs was issued at step q-2 (weights) or at the previous chunk's first step
// (rows); the VMEM operations issued after it are a compile-time function of the step's position in the tile
// (rb_after), the same for every tile because the prologue issues the tail of a virtual previous tile (its residual
// loads, the third weight step and its stores, all to valid addresses) in the steady state's order.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "mt_probe.h"
#include "mt_ragged.h"
#include "mt_vconv.h"

namespace mt {

namespace {
constexpr int RBM = 128, RBN = 256, RNT = 512;
constexpr int RWSLOT = RBM * 128;           // 128 rows x 64 bf16 channels
constexpr int RNW = 4;                       // weight ring slots
constexpr int RXROWS = RBN + 64;             // staged rows per chunk (256 frames + halo <= 64)
constexpr int RXBUF = RXROWS * 128;
constexpr int RNXW = RXROWS / 64;            // row pieces per wave per chunk (8 waves x 1 KiB)
constexpr int RNWW = RBM / 64;               // weight pieces per wave per step
constexpr int RX_OFF = RNW * RWSLOT;
constexpr int RBIAS_OFF = RX_OFF + 2 * RXBUF;
constexpr int RRAG_OFF = RBIAS_OFF + 256 * 4;
constexpr int RLDS = RRAG_OFF + RAG_LDS;
static_assert(RLDS <= 160 * 1024, "LDS budget");
constexpr int RFN = 4, RWNC = 64;

// VMEM operations per wave: epilogue loads (residual, old accumulator: 8 x 16 B each) and stores (y, y2)
template <int EF>
constexpr int rb_nepi() { return 8 * (((EF & VE_RESID) ? 1 : 0) + ((EF & VE_ACCUM) ? 1 : 0)); }
template <int EF>
constexpr int rb_nst() { return 8 * ((EF & VE_DUAL) ? 2 : 1); }

// VMEM operations a wave issues in step s of a tile of S steps (K taps per chunk): everything in program order
template <int EF, int K>
constexpr int rb_ops(int s, int S) {
  return (s == S - 1 ? rb_nepi<EF>() : 0) + (s % K == 0 ? RNXW : 0) + RNWW + (s == S - 1 ? rb_nst<EF>() : 0);
}
// issued after the weight pieces of step s (its stores on a tile's last step)
template <int EF>
constexpr int rb_ops_after_w(int s, int S) { return s == S - 1 ? rb_nst<EF>() : 0; }
// issued after the row pieces of step s (its weights and stores)
template <int EF>
constexpr int rb_ops_after_x(int s, int S) { return RNWW + rb_ops_after_w<EF>(s, S); }

// the wait at the top of step s: the data of step s + 1 must have landed. Its weights were issued at step s - 2
// (tile-periodic: index mod S), its rows (when step s + 1 starts a chunk) at the previous chunk's first step.
// Returns the VMEM operations issued after the youngest of them.
template <int EF, int K>
constexpr int rb_after(int s, int S) {
  auto md = [S](int v) { return ((v % S) + S) % S; };
  int nw = rb_ops_after_w<EF>(md(s - 2), S) + rb_ops<EF, K>(md(s - 1), S);
  if ((s + 1) % K == 0) {  // step s + 1 starts a chunk: its rows came from step s + 1 - K (mod S)
    const int sx = md(s + 1 - K);
    int nx = rb_ops_after_x<EF>(sx, S);
    for (int v = sx + 1; v < sx + K; ++v) nx += rb_ops<EF, K>(md(v), S);  // steps sx+1 .. s-1 ... up to s - 1
    // sx + K - 1 == s: the loop above counted steps sx+1 .. s-1 plus step s itself; drop step s (not issued yet)
    nx -= rb_ops<EF, K>(md(s), S);
    nw = nw < nx ? nw : nx;
  }
  return nw;
}
}  // namespace

__device__ __forceinline__ void rb_glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

template <int N>
__device__ __forceinline__ void rb_wait_vmcnt() {
  static_assert(N >= 0 && N <= 63, "vmcnt range");
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
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

template <int EF, int C, int K>
__global__ __launch_bounds__(RNT) void rbconv_kernel(VConvArgs a) {
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
  const int ntiles = rag ? rtc[a.B - 1] * NTM : a.B * ntn * NTM;
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
    int b, n0, m0;
  };
  auto tile_of = [&](int ti) {
    Tile tl;
    const int tile = gl + min(ti, nmine - 1) * gstep;  // past the last tile: the last one (phantom prefetches)
    const int r = tile / NTM;
    tl.m0 = (tile - r * NTM) * RBM;
    if (rag) {
      tl.b = rag_find(rtc, a.B, r);
      tl.n0 = (r - rag_first(rtc, tl.b)) * RBN;
    } else {
      tl.b = r / ntn;
      tl.n0 = (r - tl.b * ntn) * RBN;
    }
    return tl;
  };

  const int lrow = lane >> 3, lp = lane & 7;
  // weight piece i of this wave: row r of the 128-row slot, 16-byte unit q (swizzled on the source address)
  int woff[RNWW];
#pragma unroll
  for (int i = 0; i < RNWW; ++i) {
    const int r = 8 * (wave * RNWW + i) + lrow;
    woff[i] = r * 128 + ((lp ^ (r & 6)) * 16);
  }
  const char* wbase = reinterpret_cast<const char*>(a.w);
  auto issue_w = [&](const Tile& tl, int c, int t, int slot) {
    const char* base = wbase + ((size_t)(c * K + t) * C + tl.m0) * 128;
    // the LDS destination goes through an opaque copy: with a known constant offset the compiler tracks the DMA's
    // LDS range and puts a vmcnt wait before every ds_read it cannot prove disjoint (all of them), draining the
    // prefetch each step; the ordering is ours (counted waits + barrier)
    int so = slot * RWSLOT + wave * RNWW * 1024;
    asm volatile("" : "+s"(so));
#pragma unroll
    for (int i = 0; i < RNWW; ++i) {
      int wo = woff[i];
      asm volatile("" : "+v"(wo));  // per-step address (see read_frag)
      rb_glds16(base + wo, smem + so + i * 1024);
    }
  };
  const int R = RBN + (K - 1) * dil;
  auto issue_x = [&](const Tile& tl, int c, int buf) {
    const int f0 = tl.n0 - a.pad;
    const int Lx = rag ? rlv[tl.b] : L;
    const char* xb = reinterpret_cast<const char*>(a.x) + ((size_t)tl.b * L * C + c * 64) * 2;
    int xo = RX_OFF + buf * RXBUF;
    asm volatile("" : "+s"(xo));  // opaque LDS destination (see issue_w)
    char* dst = smem + xo;
#pragma unroll
    for (int i = 0; i < RNXW; ++i) {
      const int j = wave + 8 * i;
      const int r = 8 * j + lrow;
      const int q = lp ^ (r & 6);
      const int f = f0 + r;
      const bool ok = r < R && f >= 0 && f < Lx;
      const char* src = ok ? xb + (size_t)f * C * 2 + q * 16 : reinterpret_cast<const char*>(a.zero) + q * 16;
      rb_glds16(src, dst + j * 1024);
    }
  };

  f32x4 acc[4][RFN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < RFN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, l16 = lane & 15;
  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  const int ch16 = wm * 64 + (g4 & 1) * 16 + (g4 >> 1) * 8;
  u32x4 rv[2][RFN], yv[2][RFN];
  // epilogue operand loads of a tile (issued at the start of its last step, consumed after its MFMAs)
  auto epi_loads = [&](const Tile& tl) {
    const size_t rowbase = (size_t)tl.b * L;
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < RFN; ++fn) {
        const int n = min(tl.n0 + wn * RWNC + fn * 16 + l16, L - 1);
        const size_t o = (rowbase + n) * C + tl.m0 + ch16 + fp * 32;
        if constexpr ((EF & VE_RESID) != 0) rv[fp][fn] = *reinterpret_cast<const u32x4*>(a.resid + o);
        if constexpr ((EF & VE_ACCUM) != 0) yv[fp][fn] = *reinterpret_cast<const u32x4*>(a.y + o);
      }
  };
  // mt_vconv's packed epilogue (bias, + residual, + old accumulator, / div, then lrelu / dual outputs), the same
  // operations in the same order; every lane stores (frames past L go to the trash line): RNST per tile
  auto epilogue = [&](const Tile& tl, bool real) {
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
            if constexpr ((EF & VE_DIV) != 0) v = f32x2{v.x / a.div, v.y / a.div};
            const uint32_t rb = pk_bf16(v);
            const uint32_t av = (EF & VE_ACT) ? lrelu_pk_f_sel(v, a.slope) : (EF & VE_DUAL) ? lrelu_pk_sel(rb, a.slope) : 0u;
            o1[h][u] = (EF & VE_ACT) ? av : rb;
            o2[h][u] = av;
          }
        }
        swap16(o1[0][0], o1[1][0]);
        swap16(o1[0][1], o1[1][1]);
        const int n = tl.n0 + wn * RWNC + fn * 16 + l16;
        const bool ok = real && n < L;
        const size_t o = ((size_t)tl.b * L + n) * C + tl.m0 + ch16 + fp * 32;
        *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        if constexpr ((EF & VE_DUAL) != 0) {
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
  auto read_frag = [&](Frag& F, int ks, int slot, int xbuf, int tap) {
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
  auto mma_slice = [&](const Frag& F) {
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < RFN; ++fn) acc[fm][fn] = mfma16(F.A[fm], F.B[fn], acc[fm][fn]);
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
  };

  // ---- prologue: tile 0's chunk-0 rows and weights of steps 0..2, with the virtual previous tile's tail ----
  Tile cur = tile_of(0), nxt = tile_of(1);
  issue_x(cur, 0, 0);
  issue_w(cur, 0, 0, 0);
  issue_w(cur, 1 / K, 1 % K, 1);
  // the virtual previous tile's epilogue loads and stores, as stores of zeros to the trash line (VMEM operations
  // count in vmcnt in issue order, loads and stores alike). Inline asm: the compiler neither removes them (dead
  // stores to one address) nor orders them with vmcnt(0) waits (volatile)
  auto dummy_stores = [&](int n) {
    const u32x4 z = {0u, 0u, 0u, 0u};
    char* tp = reinterpret_cast<char*>(a.trash) + 16 * lane;
    for (int i = 0; i < n; ++i) asm volatile("global_store_dwordx4 %0, %1, off" ::"v"(tp), "v"(z) : "memory");
  };
  dummy_stores(rb_nepi<EF>());
  issue_w(cur, 2 / K, 2 % K, 2);
  dummy_stores(rb_nst<EF>());
  // step 0's data: rows of chunk 0 and weights of step 0 (issued after them: w1, epi, w2, stores)
  rb_wait_vmcnt<RNWW + rb_nepi<EF>() + RNWW + rb_nst<EF>()>();
  rb_barrier();
  Frag F0, F1;
  read_frag(F0, 0, 0, 0, 0);

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
      rb_wait_vmcnt<rb_after<EF, K>(s, S)>();
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      rb_barrier();
      if constexpr (s == S - 1 && rb_nepi<EF>() > 0) epi_loads(cur);
      if constexpr (t == 0) {  // rows of the next chunk (this tile's c + 1, or the next tile's chunk 0)
        if constexpr (c + 1 < NCH) issue_x(cur, c + 1, (c + 1) % 2);
        else issue_x(nxt, 0, 0);
      }
      {  // weights of step s + 3 (slot of step s - 1)
        constexpr int s3 = (s + 3) % S, c3 = s3 / K, t3 = s3 % K;
        if constexpr (s + 3 < S) issue_w(cur, c3, t3, slot3);
        else issue_w(nxt, c3, t3, slot3);
      }
      read_frag(F1, 1, slot, xbuf, t);
      mma_slice(F0);
      read_frag(F0, 0, slot1, xbuf1, t1);
      mma_slice(F1);
      if constexpr (s == S - 1) {
        // the epilogue after the MFMAs: nothing of it (e.g. a copy of a residual register, whose compiler wait is
        // vmcnt(0)) may be scheduled into the MFMA block
        __builtin_amdgcn_sched_barrier(0);
        epilogue(cur, true);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < RFN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    });
    cur = nxt;
    nxt = tile_of(ti + 2);
  }
  // the prefetches past the last tile (valid addresses, never read) must land before the workgroup's LDS is freed
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

namespace {
template <int EF, int C, int K>
void rb_launch(int G, const VConvArgs& a, hipStream_t st) {
  hipLaunchKernelGGL((rbconv_kernel<EF, C, K>), dim3(G), dim3(RNT), 0, st, a);
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

int rbconv_set(int enable) {
  const int prev = rb_knob();
  g_rb = enable ? 1 : 0;
  return prev;
}

// the HiFi-GAN wide-stage ResBlock convs: C_in = C_out in {128, 256}, K in {3, 7, 11}, stride 1, plain output
// (not placed), one source, the ResBlock epilogues, halo <= 64 rows
bool rbconv_handles(int ef, const VConvArgs& a) {
  if (!rb_knob()) return false;
  const bool eps = ef == VE_ACT || ef == (VE_RESID | VE_DUAL) || ef == VE_RESID || ef == (VE_RESID | VE_ACCUM) ||
                   ef == (VE_RESID | VE_ACCUM | VE_DIV) || ef == (VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL);
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
    MT_RB_EF(VE_RESID | VE_DUAL)
    MT_RB_EF(VE_RESID)
    MT_RB_EF(VE_RESID | VE_ACCUM)
    MT_RB_EF(VE_RESID | VE_ACCUM | VE_DIV)
    MT_RB_EF(VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL)
    default: set_error("rbconv: epilogue %d", ef); return -1;
  }
#undef MT_RB_EF
#undef MT_RB_K
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

}  // namespace mt
