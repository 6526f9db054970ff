// Persistent LDS-DMA implicit-GEMM Conv1d for the wide HiFi-GAN ResBlock convs (gfx950, bf16).
//
// GEMM view (same as mt_conv.h): rows m = output channels, columns n = output frames of one
// utterance, K = taps x C_in. One workgroup = 8 waves (2 in M x 4 in N, 64x64 per wave,
// v_mfma_f32_16x16x32_bf16) owns a 128 x 256 output tile at a time and walks its tiles: on grids of up to
// three rounds the XCD that runs it owns a contiguous, frame-major range of the tiles (so a launch reads what
// the previous one wrote from its own L2), else gl, gl + G, gl + 2G, ... (G = one workgroup per CU; gl groups
// consecutive tiles on workgroups that share an XCD, so the tiles that read the same input rows / weights meet
// in one L2).
//
// K loop of a tile: for each 64-channel chunk c, for each tap t: one "step" =
//   A = W[c][t] (128 rows x 128 B, one 16 KiB slot of a 4-slot ring)
//   B = X rows n0 - pad + t*dil + [0, 256) of chunk c (one of two 40 KiB row buffers; the chunk's
//       rows are staged ONCE and every tap reads them shifted by t*dil rows)
//   32 MFMAs per wave (2 K-slices x 4 x 4 fragments).
// Every byte is staged by global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear LDS
// image); LDS rows are 128 B with the 16-byte chunk XOR-swizzled by (row & 6) on the SOURCE address and
// on the ds_read (cdna_hip_programming.md rule 21): every ds_read_b128 lane group of an MFMA fragment
// then hits 16 distinct bank slots for ANY row shift t*dil (exhaustively checked over the 16 shifts;
// a (row >> 1) & 7 swizzle is 2-way on half of them). Weights of step s+3 and the rows of chunk u+1 are
// in flight while step s computes: each wave counts the DMA instructions it issued and waits with a
// COUNTED `s_waitcnt vmcnt(N)` for exactly the ones the step needs, then one raw s_barrier per step
// publishes them (no __syncthreads: its fence would drain the prefetch). The loop runs across tile
// boundaries, so the next tile's first weights and rows land while this tile's epilogue stores.
// Zero padding (frames outside [0, L)) is read from a zero page instead of branching.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <type_traits>

#include "mt_misc.h"
#include "mt_probe.h"
#include "mt_ragged.h"
#include "mt_vconv.h"

namespace mt {

namespace {
constexpr int BN = 256, NT = 512;                // BN: frames per tile (128 for small 1x1 grids)
constexpr int MMAX = 1024;                        // largest C_out (per-channel epilogue tables in LDS)
constexpr int BMP = 64;                           // packed weight rows are padded to a multiple of this
// Tile geometry by output rows per workgroup: BM = 128 (waves 2 in M x 4 in N, 64x64 per wave) for
// C_out % 128 == 0, BM = 64 (1 x 8 waves, 64x32 per wave) for the 64-channel stage.
// K1: 1x1 convs (Linear): a chunk's rows are exactly the tile's 256 frames and every step starts a new
// chunk, so rows are staged two chunks ahead in three 32 KiB buffers and the weight ring is 3 deep.
template <int BM_, bool K1_, int NPAR_, int BN_ = BN>
struct VT {
  static constexpr int BM = BM_, TBN = BN_;
  static constexpr int WAVES_M = BM / 64, WAVES_N = 8 / WAVES_M;
  static constexpr int WNC = TBN / WAVES_N;       // frames per wave
  static constexpr int FN = WNC / 16;             // 16-frame fragments per wave
  static_assert(WNC % 16 == 0, "a wave covers whole 16-frame fragments");
  static constexpr int WSLOT = BM * 128;          // BM rows x 64 bf16 channels
  static constexpr int NWW = BM / 64;             // W wave-instructions per wave per step
  static constexpr int XROWS = K1_ ? TBN : TBN + 64;  // >= BN + (taps - 1) * dil (halo <= 64 rows)
  static constexpr int XBUF = XROWS * 128;
  static constexpr int NXW = XROWS / 64;          // X wave-instructions per wave per chunk
  static constexpr int PARB = NPAR_ * MMAX * 4 + (K1_ ? 0 : RAG_LDS);  // per-channel tables (+ the ragged tile map)
  static constexpr int LDSMAX = 160 * 1024;
  // Ring depths: as deep as LDS allows (the short decoder K loops are bound by the DMA latency the ring covers:
  // NWSLOT - 1 weight steps in flight). K1: weights and rows advance together (every step is a chunk), 3..5 deep.
  // k >= 2: row buffers hold chunks staged NXB-1 ahead (the 64-row tiles with 256 frames have one chunk per tile
  // and stage two tiles ahead; with 384 frames the buffers only fit twice); the weight ring 4..6 deep.
  static constexpr int K1D = (5 * (WSLOT + XBUF) + PARB <= LDSMAX) ? 5 : (4 * (WSLOT + XBUF) + PARB <= LDSMAX) ? 4 : 3;
  static constexpr int NXB = K1_ ? K1D : (BM == 64 && TBN <= 256) ? 3 : 2;
  static constexpr int NWSLOT = K1_ ? K1D
                                    : (6 * WSLOT + NXB * XBUF + PARB <= LDSMAX) ? 6
                                    : (5 * WSLOT + NXB * XBUF + PARB <= LDSMAX) ? 5 : 4;
  static constexpr int PAR_OFF = NWSLOT * WSLOT + NXB * XBUF;  // per-channel tables: bias, wsum, alpha, ibeta
  static constexpr int RAG_OFF = PAR_OFF + NPAR_ * MMAX * 4;
  static constexpr int LDS_BYTES = PAR_OFF + PARB;
  static_assert(LDS_BYTES <= LDSMAX, "LDS budget");
};
}  // namespace

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// s_waitcnt vmcnt(k) for a wave-uniform runtime bound n, with k the largest of {0,2,4,7,10,15,23,31} <= n:
// waiting for fewer outstanding operations than allowed is always correct (only stricter), and a
// three-level branch tree keeps the scalar cost per step small (a 64-way switch was ~40 SALU + branches)
__device__ __forceinline__ void wait_vmcnt(int n) {
#if defined(VCONV_EXP) && VCONV_EXP == 1  // timing experiment only: no DMA waits (wrong results)
  return;
#endif
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

__device__ __forceinline__ void raw_barrier() {
#if defined(VCONV_EXP) && VCONV_EXP == 2  // timing experiment only: no step barrier (wrong results)
  return;
#endif
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

#ifndef VC_CT_LOADERS
#define VC_CT_LOADERS 8
#endif

template <int EF>
constexpr int vc_npar() {  // per-channel LDS tables (MMAX floats each); VE_GNRES: gamma, beta + the GN table
  return 1 + ((EF & VE_LN) ? 1 : 0) + ((EF & VE_SNAKE) ? 2 : 0) + ((EF & VE_GNRES) ? 3 : 0);
}

// The compile-time K loop's staging split and schedule (bf16 vconv_kernel<EF, BMT, K1, BNT, false, CTN, CTT>): the
// kernel and its host launcher (which registers the schedule for the CPU schedule test) take them from here.
template <int EF, int BMT, bool K1, int BNT, int CTN, int CTT>
struct CtSched {
  using TT = VT<BMT, K1, vc_npar<EF>(), BNT>;
  static constexpr int TAPS = CTT, NCHC = CTN, LW = VC_CT_LOADERS;  // LW loader waves (one per SIMD when 4)
  static constexpr int WPW = (TT::WSLOT / 1024) / LW, XPW = (TT::XBUF / 1024) / LW;
  static_assert(WPW * LW * 1024 == TT::WSLOT && XPW * LW * 1024 == TT::XBUF, "pieces per loader wave");
  static constexpr int TXA = (TT::NXB - 1) * TAPS - 2 < 1 ? 1 : (TT::NXB - 1) * TAPS - 2;
  static constexpr int TX = TXA < TAPS ? (TXA < XPW ? TXA : XPW) : (TAPS < XPW ? TAPS : XPW);
  static constexpr int NST = 2 * TT::FN * ((EF & VE_DUAL) ? 2 : 1);  // the epilogue's stores (every lane stores)
  using SCH = VcSched<NCHC, TAPS, TT::NWSLOT, TT::NXB, TX, WPW, XPW, NST>;
  using REG = SchedReg<0, NCHC, TAPS, TT::NWSLOT, TT::NXB, TX, WPW, XPW, NST, 1, SCH::wait_first(-1)>;
};

// FM (operand mode) 1, fp32 operands (the text encoder, whose duration path must be the reference's fp32
// arithmetic): a 128-byte LDS row holds 32 channels, one 16-byte fragment per lane feeds 4 exact-fp32
// v_mfma_f32_16x16x4_f32 (mfma16), and the epilogue stores fp32 in the accumulator layout (bias, ReLU, residual, mask
// only). FM 2, split-bf16 (VConvArgs::f32 == 2): the bf16 K loop over the 6-plane operands with FM 1's fp32 epilogue
// (or, VE_SPLIT6, the 6-plane split of its result).
template <int EF, int BMT, bool K1, int BNT = BN, int FM = 0, int CTN = 0, int CTT = 0>
__global__ __launch_bounds__(NT) void vconv_kernel(VConvArgs a) {
  constexpr bool F32 = FM == 1;   // fp32 K loop (operands, fragments, MFMA)
  constexpr bool F32E = FM != 0;  // fp32 epilogue (fp32 residual; fp32 output unless VE_SPLIT6)
  using TT = VT<BMT, K1, vc_npar<EF>(), BNT>;
  constexpr int BN = TT::TBN;
  constexpr int BM = TT::BM, WSLOT = TT::WSLOT, NWW = TT::NWW, FN = TT::FN;
  constexpr int WNC = TT::WNC, NXB = TT::NXB, NWSLOT = TT::NWSLOT, XBUF = TT::XBUF, NXW = TT::NXW;
  constexpr int BIAS_OFF = TT::PAR_OFF;
  constexpr int WSUM_OFF = BIAS_OFF + MMAX * 4;
  constexpr int SNAKE_OFF = WSUM_OFF + ((EF & VE_LN) ? MMAX * 4 : 0);
  constexpr int GNP_OFF = SNAKE_OFF + ((EF & VE_SNAKE) ? 2 * MMAX * 4 : 0);  // gamma, beta, then per-wave GN table
  __shared__ __attribute__((aligned(1024))) char smem[TT::LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave % TT::WAVES_M, wn = wave / TT::WAVES_M;
  const int taps = a.taps, dil = a.dil, L = a.L, cin = a.cin;
  constexpr int ES = F32 ? 4 : 2, CHR = 128 / ES;  // element bytes, channels per 128-byte row
  const int nch = cin / CHR;
  const int S = nch * taps;
  const int ntn = (a.Lout + BN - 1) / BN, ntm = a.Mpad / BM;
  // ragged batch: the live column tiles of each utterance (mt_ragged.h)
  const bool rag = !K1 && a.lens != nullptr;
  int* rtc = reinterpret_cast<int*>(smem + TT::RAG_OFF);
  int* rlv = rtc + RAG_MAXB;
  if (rag) {
    rag_build(rtc, rlv, a.lens, a.lmul, L, a.Lout - L, a.Lout, a.B, BN, tid);
    __syncthreads();
  }
  const int ntiles = rag ? rtc[a.B - 1] * ntm : a.B * ntn * ntm;
  const int G = gridDim.x, g = blockIdx.x;
  // XCD-major tile ownership (MT_XCD_TILES, A/B knob; default on): workgroup g runs on XCD g % 8 (round-robin
  // dispatch; speed only, never correctness) and the 8 XCDs own CONTIGUOUS tile ranges in proportion to their
  // workgroup counts, walked round-robin by their workgroups. Tiles are frame-major, so every launch maps a frame
  // range to the same XCD: a conv reads what the previous launch wrote from that XCD's L2 (the decoder's
  // activations fit its 4 MiB). Off: the round-robin walk gl, gl + G, ... with consecutive gl on one XCD.
  const int xcd = g & 7, lw = g >> 3;
  const int gx = (G - xcd + 7) >> 3;                   // workgroups on this XCD
  const int sx = xcd * (G >> 3) + min(xcd, G & 7);     // workgroups on the XCDs before it
  const int xt0 = (int)((long)ntiles * sx / G), xt1 = (int)((long)ntiles * (sx + gx) / G);
  const bool xmaj = a.xcd_tiles != 0;
  const int gl = xmaj ? xt0 + lw : (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int gstep = xmaj ? gx : G;
  const int nmine = xmaj ? (gl < xt1 ? (xt1 - gl + gx - 1) / gx : 0) : (gl < ntiles ? (ntiles - gl + G - 1) / G : 0);
  const int Q = nmine * S;
  if (Q == 0) return;
#if defined(VCONV_TS)
  unsigned long long ts_v[4] = {__builtin_amdgcn_s_memrealtime(), 0, 0, 0};
#endif
  // per-channel epilogue tables in LDS (one array with the staging images: a second __shared__ object
  // costs vmcnt(0) waits). With 16-byte aligned tables (every packed weight blob) they arrive by LDS-DMA issued
  // ahead of the prologue's staging (below), so their latency overlaps it; else by VGPR loads and a barrier.
  const float* tabs[6];
  int toff[6], ntab = 0;
  tabs[ntab] = a.bias, toff[ntab++] = BIAS_OFF;
  if constexpr ((EF & VE_LN) != 0) tabs[ntab] = a.wsum, toff[ntab++] = WSUM_OFF;
  if constexpr ((EF & VE_SNAKE) != 0) {
    tabs[ntab] = a.snake_alpha, toff[ntab++] = SNAKE_OFF;
    tabs[ntab] = a.snake_ibeta, toff[ntab++] = SNAKE_OFF + MMAX * 4;
  }
  if constexpr ((EF & VE_GNRES) != 0) {
    tabs[ntab] = a.gn_gamma, toff[ntab++] = GNP_OFF;
    tabs[ntab] = a.gn_beta, toff[ntab++] = GNP_OFF + MMAX * 4;
  }
  uintptr_t tor = 0;
  for (int i = 0; i < ntab; ++i) tor |= reinterpret_cast<uintptr_t>(tabs[i]);
  const bool tab_dma = (tor & 15) == 0;
  if (!tab_dma) {
  for (int i = tid; i < a.M; i += NT) {
    reinterpret_cast<float*>(smem + BIAS_OFF)[i] = a.bias[i];
    if constexpr ((EF & VE_LN) != 0) reinterpret_cast<float*>(smem + WSUM_OFF)[i] = a.wsum[i];
    if constexpr ((EF & VE_SNAKE) != 0) {
      reinterpret_cast<float*>(smem + SNAKE_OFF)[i] = a.snake_alpha[i];
      reinterpret_cast<float*>(smem + SNAKE_OFF)[MMAX + i] = a.snake_ibeta[i];
    }
    if constexpr ((EF & VE_GNRES) != 0) {
      reinterpret_cast<float*>(smem + GNP_OFF)[i] = a.gn_gamma[i];
      reinterpret_cast<float*>(smem + GNP_OFF)[MMAX + i] = a.gn_beta[i];
    }
  }
  __syncthreads();
  }

  auto tile_of = [&](int ti, int& b, int& n0, int& m0) {
    const int tile = gl + ti * gstep;
    const int r = tile / ntm;
    m0 = (tile - r * ntm) * BM;
    if (rag) {
      b = rag_find(rtc, a.B, r);
      n0 = (r - rag_first(rtc, b)) * BN;
    } else {
      b = r / ntn;
      n0 = (r - b * ntn) * BN;
    }
  };

  const int lrow = lane >> 3, lp = lane & 7;
  // staging of one step's weights / one chunk's rows; (b, n0, m0) of the cursor's tile are kept
  // decoded by the caller (no integer division per step)
  auto issue_w = [&](int m0, int c, int t, int slot) {
    const char* base = reinterpret_cast<const char*>(a.w) + ((size_t)(c * taps + t) * a.Mpad + m0) * 128;
    char* dst = smem + slot * WSLOT;
#pragma unroll
    for (int i = 0; i < NWW; ++i) {
      const int j = wave * NWW + i;
      const int r = 8 * j + lrow;
      const int q = lp ^ (r & 6);
      glds16(base + r * 128 + q * 16, dst + j * 1024);
    }
  };
  const int R = BN + (taps - 1) * dil;
  const int c0 = a.c0;
  auto issue_x = [&](int b, int n0, int c, int buf) {
    const int f0 = n0 - a.pad;
    const int Lx = rag ? rlv[b] : L;  // frames at and past Lx are the utterance's zero padding
    const bool lo = c * CHR < c0;  // chunk from the first or the second source (skip concatenation)
    const int ldx = lo ? c0 : cin - c0;
    const char* xb = lo ? reinterpret_cast<const char*>(a.x) + ((size_t)b * L * c0 + c * CHR) * ES
                        : reinterpret_cast<const char*>(a.x1) + ((size_t)b * L * (cin - c0) + (c * CHR - c0)) * ES;
    char* dst = smem + NWSLOT * WSLOT + buf * XBUF;
#pragma unroll
    for (int i = 0; i < NXW; ++i) {
      const int j = wave + 8 * i;
      const int r = 8 * j + lrow;
      const int q = lp ^ (r & 6);
      const int f = f0 + r;
      const bool ok = r < R && f >= 0 && f < Lx;
      const char* src = ok ? xb + (size_t)f * ldx * ES + q * 16 : reinterpret_cast<const char*>(a.zero) + q * 16;
      glds16(src, dst + j * 1024);
    }
  };

  f32x4 acc[4][FN];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, l16 = lane & 15;
  // Epilogue I/O is 16 bytes per lane: blocks X = (fm, fn) and Y = (fm + 1, fn) hold, per lane, 4
  // channels of one frame each; v_permlane16_swap (odd 16-lane rows of X <-> even rows of Y) turns
  // them into 8 consecutive channels per lane (row g4: X or Y by g4 & 1, channels +8 by g4 >> 1), so a
  // wave moves 64 B contiguous per frame per instruction. The swap is an involution, so loaded
  // residuals are swapped back into the accumulator layout the same way.
  auto swap16 = [](uint32_t& x, uint32_t& y) {
    const auto r = __builtin_amdgcn_permlane16_swap(x, y, false, false);
    x = r[0];
    y = r[1];
  };
  const int ch16 = wm * 64 + (g4 & 1) * 16 + (g4 >> 1) * 8;  // + fm * 16 (fm even): this lane's 8 channels
  // residual / accumulator values of the tile, 16 B per lane: loaded at the start of the tile's last
  // step, consumed after its MFMAs
  u32x4 rv[2][FN], yv[2][FN];
  f32x4 rv32[F32E ? 4 : 1][FN];  // F32E: the fp32 residual of each accumulator block (4 channels of one frame)
  float2 lns[FN];  // (mean, rstd) of each fragment column's frame (VE_LN)
  f32x4 lnr[FN][2];  // VE_LNP: raw per-slab partials (s0, q0, s1, q1), (s2, q2, s3, q3)
  float mk[FN];    // frame mask of each fragment column (VE_MASK)
  auto epi_loads = [&](int ti) {
    int b, n0, m0;
    tile_of(ti, b, n0, m0);
    const size_t rowbase = (size_t)b * L;
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int n = min(n0 + wn * WNC + fn * 16 + l16, L - 1);  // clamped: no per-block branch
        const size_t o = (rowbase + n) * a.M + m0 + ch16 + fp * 32;
        if constexpr (F32E && (EF & VE_RESID) != 0) {
          const float* rp = reinterpret_cast<const float*>(a.resid) + (rowbase + n) * a.M + m0 + wm * 64 + 4 * g4;
          rv32[2 * fp][fn] = *reinterpret_cast<const f32x4*>(rp + (2 * fp) * 16);
          rv32[2 * fp + 1][fn] = *reinterpret_cast<const f32x4*>(rp + (2 * fp + 1) * 16);
        } else if constexpr ((EF & VE_RESID) != 0) {
          rv[fp][fn] = *reinterpret_cast<const u32x4*>(a.resid + o);
        }
        if constexpr ((EF & VE_ACCUM) != 0) yv[fp][fn] = *reinterpret_cast<const u32x4*>(a.y + o);
        if constexpr ((EF & VE_LN) != 0 && (EF & VE_LNP) == 0)
          if (fp == 0) lns[fn] = *reinterpret_cast<const float2*>(a.ln_stats + 2 * (rowbase + n));
        if constexpr ((EF & VE_LNP) != 0)
          if (fp == 0) {  // the producer's 4 per-slab (sum, sum of squares) of this frame; merged after the MFMAs
            const f32x4* pp = reinterpret_cast<const f32x4*>(a.ln_stats + 8 * (rowbase + n));
            lnr[fn][0] = pp[0];
            lnr[fn][1] = pp[1];
          }
        if constexpr ((EF & (VE_MASK | VE_GNRES)) != 0)
          if (fp == 0) mk[fn] = a.emask[rowbase + n];
      }
  };
  // Every lane stores (frames past L go to a trash line), so the store count per tile is a constant the
  // vmcnt bookkeeping can add: NST younger VMEM operations the next steps' waits may leave in flight.
  constexpr int NST = F32E ? ((EF & VE_SPLIT6) ? 12 * FN : 4 * FN) : 2 * FN * ((EF & VE_DUAL) ? 2 : 1);
  // epilogues without per-element transcendental / statistics work run as packed fp32 pairs
  constexpr bool PK = (EF & ~(VE_RESID | VE_ACCUM | VE_DIV | VE_ACT | VE_DUAL | VE_MASK | VE_PMASK)) == 0;
  constexpr bool PKS = (EF & VE_LN) != 0 && (EF & ~(VE_LN | VE_LNP | VE_SNAKE)) == 0;
  auto bf2 = [](uint32_t w, int i) -> float { return __uint_as_float(i ? (w & 0xffff0000u) : (w << 16)); };
  auto pack2 = [](bf16 lo, bf16 hi) -> uint32_t {
    return (uint32_t)__builtin_bit_cast(uint16_t, lo) | ((uint32_t)__builtin_bit_cast(uint16_t, hi) << 16);
  };
  auto epilogue = [&](int ti) {
    int b, n0, m0;
    tile_of(ti, b, n0, m0);
    if constexpr (F32E && (EF & VE_SPLIT6) != 0) {
      // split-bf16 output: v as the fp32 epilogue below computes it, then its 3-way split h1 + h2 + h3 (split3_bf16)
      // stored as the 6 planes (h1, h1, h1, h2, h2, h3) of [frames][6 M]: blocks (2 fp, fn) and (2 fp + 1, fn)
      // packed per part and permlane16-swapped into 8 consecutive channels per lane (the bf16 epilogue's layout),
      // one 16-byte store per plane
      const size_t ld6 = (size_t)6 * a.M;
#pragma unroll
      for (int fp = 0; fp < 2; ++fp)
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          uint32_t pt[3][2][2];  // part, block (X / Y), word (channels 4 g4 + 0,1 / 2,3)
#pragma unroll
          for (int h = 0; h < 2; ++h) {
            const int fm = 2 * fp + h;
            const int m = m0 + wm * 64 + fm * 16 + 4 * g4;
            const f32x4 bias4 = *reinterpret_cast<const f32x4*>(smem + BIAS_OFF + 4 * m);
            f32x4 v = acc[fm][fn] + bias4;
            if constexpr ((EF & VE_RELU) != 0)
              v = f32x4{fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
            if constexpr ((EF & VE_RESID) != 0) v = v + rv32[fm][fn];
            if constexpr ((EF & VE_MASK) != 0) v = v * mk[fn];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              bf16 p1[2], p2[2], p3[2];
              split3_bf16(v[2 * u], p1[0], p2[0], p3[0]);
              split3_bf16(v[2 * u + 1], p1[1], p2[1], p3[1]);
              pt[0][h][u] = pack2(p1[0], p1[1]);
              pt[1][h][u] = pack2(p2[0], p2[1]);
              pt[2][h][u] = pack2(p3[0], p3[1]);
            }
          }
#pragma unroll
          for (int q = 0; q < 3; ++q) {
            swap16(pt[q][0][0], pt[q][1][0]);
            swap16(pt[q][0][1], pt[q][1][1]);
          }
          const int n = n0 + wn * WNC + fn * 16 + l16;
          const size_t o = ((size_t)b * L + n) * ld6 + m0 + ch16 + fp * 32;
#pragma unroll
          for (int pl = 0; pl < 6; ++pl) {
            const int q = pl < 3 ? 0 : pl < 5 ? 1 : 2;
            *reinterpret_cast<u32x4*>(n < L ? a.y + o + (size_t)pl * a.M : a.trash + 8 * lane) =
                u32x4{pt[q][0][0], pt[q][0][1], pt[q][1][0], pt[q][1][1]};
          }
        }
      return;
    }
    if constexpr (F32E) {
      // fp32 out in the accumulator layout: lane (g4, l16) of block (fm, fn) holds channels m..m+3 of frame n, one
      // 16-byte store (frames past L go to the trash line, so the store count stays the constant NST)
#pragma unroll
      for (int fm = 0; fm < 4; ++fm) {
        const int m = m0 + wm * 64 + fm * 16 + 4 * g4;
        const f32x4 bias4 = *reinterpret_cast<const f32x4*>(smem + BIAS_OFF + 4 * m);
#pragma unroll
        for (int fn = 0; fn < FN; ++fn) {
          const int n = n0 + wn * WNC + fn * 16 + l16;
          f32x4 v = acc[fm][fn] + bias4;
          if constexpr ((EF & VE_RELU) != 0)
            v = f32x4{fmaxf(v[0], 0.f), fmaxf(v[1], 0.f), fmaxf(v[2], 0.f), fmaxf(v[3], 0.f)};
          if constexpr ((EF & VE_RESID) != 0) v = v + rv32[fm][fn];
          if constexpr ((EF & VE_MASK) != 0) v = v * mk[fn];
          float* yp = reinterpret_cast<float*>(a.y) + ((size_t)b * L + n) * a.M + m;
          *reinterpret_cast<f32x4*>(n < L ? yp : reinterpret_cast<float*>(a.trash) + 4 * lane) = v;
        }
      }
      return;
    }
    double gs[2] = {0.0, 0.0}, gq[2] = {0.0, 0.0};  // VE_GNSTATS: this lane's sums per 32-channel group
    float rmean[FN], rm2[FN];  // VE_ROWSTATS: Welford (mean, M2) of this lane's 16 channels of frame fn
#pragma unroll
    for (int fn = 0; fn < FN; ++fn) rmean[fn] = rm2[fn] = 0.f;
    if constexpr ((EF & VE_LNP) != 0) {
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) lns[fn] = ln_merge4(lnr[fn][0], lnr[fn][1], a.ln_eps);
    }
    // VE_GNRES: (mean, rstd) of the residual's GroupNorm for the utterances this wave's frames span and its
    // two 32-channel groups, merged from the producer's partials into a wave-private LDS table (4 lanes per
    // (utterance, group) pair, fp64 as gn_apply merges them); read back by the same wave, no barrier
    int gu0 = 0;
    int gun[FN];
    const float* gtab = reinterpret_cast<const float*>(smem + GNP_OFF + 2 * MMAX * 4) + wave * 32;
    if constexpr ((EF & VE_GNRES) != 0) {
      const int nlo = n0 + wn * WNC, nhi = min(nlo + WNC, L) - 1;
      gu0 = nlo / a.gn_T;
      const int nu = min(nhi / a.gn_T, a.gn_B - 1) - gu0 + 1;  // <= 8 (host check)
      const int pair = lane >> 2, sub = lane & 3, pu = pair >> 1;
      const int G = a.M >> 5, grp = ((m0 + wm * 64) >> 5) + (pair & 1);
      double s1 = 0.0, s2 = 0.0;
      if (pu < nu) {
        const double* p = a.gn_in + ((size_t)(gu0 + pu) * G + grp) * a.gn_in_parts * 2;
        for (int k = sub; k < a.gn_in_parts; k += 4) {
          s1 += p[2 * k];
          s2 += p[2 * k + 1];
        }
      }
      s1 += __shfl_xor(s1, 1, 64);
      s2 += __shfl_xor(s2, 1, 64);
      s1 += __shfl_xor(s1, 2, 64);
      s2 += __shfl_xor(s2, 2, 64);
      if (sub == 0 && pu < nu) {
        const double cnt = 32.0 * (double)a.gn_T, mean = s1 / cnt;
        double var = s2 / cnt - mean * mean;
        var = var < 0.0 ? 0.0 : var;
        float* wt = reinterpret_cast<float*>(smem + GNP_OFF + 2 * MMAX * 4) + wave * 32;
        wt[2 * pair] = (float)mean;
        wt[2 * pair + 1] = (float)(1.0 / sqrt(var + (double)a.gn_eps));
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        const int n = min(n0 + wn * WNC + fn * 16 + l16, L - 1);
        gun[fn] = min(n / a.gn_T, a.gn_B - 1) - gu0;
      }
    }
#pragma unroll
    for (int fp = 0; fp < 2; ++fp)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        // residual / old accumulator of blocks X (fm = 2fp) and Y (fm = 2fp+1) back in accumulator layout
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
        uint32_t o1[2][2], o2[2][2];  // [X|Y][dword]
        float pmk = 1.f;  // VE_PMASK: the mask of the output frame this lane's 32-row group lands in
        if constexpr ((EF & VE_PMASK) != 0) {
          const int n = n0 + wn * WNC + fn * 16 + l16;
          const int e = n * a.ldy + m0 + wm * 64 + fp * 32 - a.yshift;
          const bool ok = n < a.Lout && e >= 0 && e < a.ylim;
          pmk = ok ? a.emask[(size_t)b * (a.ylim / a.mask_div) + e / a.mask_div] : 0.f;
        }
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const int fm = 2 * fp + h;
          const int m = m0 + wm * 64 + fm * 16 + 4 * g4;
          const f32x4 bias4 = *reinterpret_cast<const f32x4*>(smem + BIAS_OFF + 4 * m);
          f32x4 ws4, al4, ib4;
          if constexpr ((EF & VE_LN) != 0) ws4 = *reinterpret_cast<const f32x4*>(smem + WSUM_OFF + 4 * m);
          if constexpr ((EF & VE_SNAKE) != 0) {
            al4 = *reinterpret_cast<const f32x4*>(smem + SNAKE_OFF + 4 * m);
            ib4 = *reinterpret_cast<const f32x4*>(smem + SNAKE_OFF + 4 * (MMAX + m));
          }
          const uint32_t rr[2] = {h ? ry0 : rx0, h ? ry1 : rx1};
          float gga = 0.f, ggs = 0.f;  // VE_GNRES: this (utterance, group)'s mean and rstd
          f32x4 gam4, bet4;
          if constexpr ((EF & VE_GNRES) != 0) {
            const float2 mr = *reinterpret_cast<const float2*>(gtab + 2 * (2 * gun[fn] + fp));
            gga = mr.x;
            ggs = mr.y;
            gam4 = *reinterpret_cast<const f32x4*>(smem + GNP_OFF + 4 * m);
            bet4 = *reinterpret_cast<const f32x4*>(smem + GNP_OFF + 4 * (MMAX + m));
          }
          const uint32_t yy[2] = {h ? yy0 : yx0, h ? yy1 : yx1};
          if constexpr (PK) {
            // the HiFi-GAN / plain epilogues as packed fp32 pairs (same operations and order as the scalar path)
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              f32x2 v = f32x2{acc[fm][fn][2 * u], acc[fm][fn][2 * u + 1]} + f32x2{bias4[2 * u], bias4[2 * u + 1]};
              if constexpr ((EF & VE_RESID) != 0) v = v + unpk_bf16(rr[u]);
              if constexpr ((EF & VE_ACCUM) != 0) v = unpk_bf16(yy[u]) + v;
              if constexpr ((EF & VE_DIV) != 0) v = f32x2{div_rn(v.x, a.div, 1.f / a.div), div_rn(v.y, a.div, 1.f / a.div)};
              if constexpr ((EF & VE_MASK) != 0) v = v * mk[fn];
              if constexpr ((EF & VE_PMASK) != 0) v = v * pmk;
              const uint32_t rb = pk_bf16(v);
              // VE_ACT (conv1's only output): lrelu(t) rounded once from fp32; VE_DUAL: the activated copy of the STORED
              // chain state, lrelu(round(v)) — what a consumer activating the stored tensor itself (the fused pairs'
              // in-place pass) computes
              const uint32_t av = (EF & VE_ACT) ? lrelu_pk_f_sel(v, a.slope)
                                  : (EF & VE_DUAL) ? lrelu_pk_sel(rb, a.slope) : 0u;
              o1[h][u] = (EF & VE_ACT) ? av : rb;
              o2[h][u] = av;
            }
            continue;
          }
          if constexpr (PKS) {
            // LayerNorm-folded (+ SnakeBeta) epilogues (the transformer FF1 / QKV GEMMs) as packed fp32 pairs, the
            // same operations in the same order as the scalar path below
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              // (v - mean * wsum) * rstd + bias [+ ibeta * sin(alpha * v)^2], multiply-adds spelled out (fma2: mt_ffn
              // computes the same bits)
              f32x2 v = f32x2{acc[fm][fn][2 * u], acc[fm][fn][2 * u + 1]};
              v = fma2(f32x2{-lns[fn].x, -lns[fn].x}, f32x2{ws4[2 * u], ws4[2 * u + 1]}, v);
              v = fma2(v, f32x2{lns[fn].y, lns[fn].y}, f32x2{bias4[2 * u], bias4[2 * u + 1]});
              if constexpr ((EF & VE_SNAKE) != 0) {
                const f32x2 arg = v * f32x2{al4[2 * u], al4[2 * u + 1]};
                const f32x2 sn = f32x2{__sinf(arg.x), __sinf(arg.y)};
                v = fma2(f32x2{ib4[2 * u], ib4[2 * u + 1]}, sn * sn, v);
              }
              o1[h][u] = pk_bf16(v);
              o2[h][u] = 0u;
            }
            continue;
          }
          bf16 ob[4], ab[4];
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float v = acc[fm][fn][r];
            if constexpr ((EF & VE_LN) != 0) v = lns[fn].y * (v - lns[fn].x * ws4[r]);
            v = v + bias4[r];
            if constexpr ((EF & VE_SNAKE) != 0) {
              const float sn = __sinf(v * al4[r]);
              v = v + ib4[r] * (sn * sn);
            }
            if constexpr ((EF & VE_RELU) != 0) v = fmaxf(v, 0.f);
            if constexpr ((EF & VE_GNRES) != 0) {
              // gn_apply's arithmetic: scale = rstd * gamma, shift = -scale * mean + beta, mish, * mask; the block
              // output h stays fp32 into h + res(x) (as under the reference's autocast: GroupNorm / Mish run in
              // fp32 and the sum rounds once)
              const float sc = ggs * gam4[r], sh = -sc * gga + bet4[r];
              const float hv = mish_f(bf2(rr[r >> 1], r & 1) * sc + sh) * mk[fn];
              v = v + hv;
            } else if constexpr ((EF & VE_RESID) != 0) {
              v = v + bf2(rr[r >> 1], r & 1);
            }
            if constexpr ((EF & VE_ACCUM) != 0) v = bf2(yy[r >> 1], r & 1) + v;
            if constexpr ((EF & VE_DIV) != 0) v = div_rn(v, a.div, 1.f / a.div);
            if constexpr ((EF & VE_GNSTATS) != 0) {
              if (n0 + wn * WNC + fn * 16 + l16 < L) {
                gs[fp] += (double)v;
                gq[fp] += (double)v * (double)v;
              }
            }
            if constexpr ((EF & VE_MASK) != 0 && (EF & VE_GNRES) == 0) v = v * mk[fn];
            if constexpr ((EF & VE_PMASK) != 0) v = v * pmk;
            const bf16 rb = (bf16)v;
            if constexpr ((EF & VE_ROWSTATS) != 0) {  // Welford over the lane's values (k-th value: 1/k)
              const float fr = (float)rb, dl = fr - rmean[fn];
              rmean[fn] += dl * (1.f / (float)(fp * 8 + h * 4 + r + 1));
              rm2[fn] += dl * (fr - rmean[fn]);
            }
            const bf16 av = (bf16)lrelu_f((EF & VE_ACT) ? v : (float)rb, a.slope);
            ob[r] = (EF & VE_ACT) ? av : rb;
            ab[r] = av;
          }
          o1[h][0] = pack2(ob[0], ob[1]);
          o1[h][1] = pack2(ob[2], ob[3]);
          o2[h][0] = pack2(ab[0], ab[1]);
          o2[h][1] = pack2(ab[2], ab[3]);
        }
        swap16(o1[0][0], o1[1][0]);
        swap16(o1[0][1], o1[1][1]);
        const int n = n0 + wn * WNC + fn * 16 + l16;
        const int e = n * a.ldy + m0 + ch16 + fp * 32 - a.yshift;  // element of this utterance's output
        const bool ok = n < a.Lout && e >= 0 && e < a.ylim;
        const size_t o = (size_t)b * a.ystride + e;
        *reinterpret_cast<u32x4*>(ok ? a.y + o : a.trash + 8 * lane) = u32x4{o1[0][0], o1[0][1], o1[1][0], o1[1][1]};
        if constexpr ((EF & VE_DUAL) != 0) {
          swap16(o2[0][0], o2[1][0]);
          swap16(o2[0][1], o2[1][1]);
          *reinterpret_cast<u32x4*>(ok ? a.y2 + o : a.trash + 8 * lane) = u32x4{o2[0][0], o2[0][1], o2[1][0], o2[1][1]};
        }
      }
    if constexpr ((EF & VE_ROWSTATS) != 0) {
      // lanes l16 + 16*g4 hold the wave's 64-channel slab of one frame: reduce over g4, lanes 0-15 store
      const int ns = a.M >> 6, slab = (m0 >> 6) + wm;
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) {
        // Chan's merge of equal-count (16, then 32) groups across the 4 lane rows: the slab's (mean, M2)
        float mu = rmean[fn], m2 = rm2[fn];
#pragma unroll
        for (int o = 16; o <= 32; o <<= 1) {
          const float mo = __shfl_xor(mu, o, 64), qo = __shfl_xor(m2, o, 64);
          const float dl = mo - mu;
          const float nh = (float)(o == 16 ? 16 : 32);  // count of each half
          m2 = m2 + qo + dl * dl * (nh * 0.5f);
          mu = 0.5f * (mu + mo);
        }
        const int n = n0 + wn * WNC + fn * 16 + l16;
        if (g4 == 0 && n < L)
          *reinterpret_cast<float2*>(a.row_out + 2 * (((size_t)b * L + n) * ns + slab)) = float2{mu, m2};
      }
    }
    if constexpr ((EF & VE_GNSTATS) != 0) {
      // fm pair fp covers channels m0 + wm*64 + 32*fp .. +31: one GroupNorm(8) group of the 256 channels
      const int nparts = ntn * TT::WAVES_N, part = (n0 / BN) * TT::WAVES_N + wn;
      const int G = a.M / 32;
#pragma unroll
      for (int fp = 0; fp < 2; ++fp) {
        const double s1 = wave_sum_d(gs[fp]), s2 = wave_sum_d(gq[fp]);
        if (lane == 0) {
          const int g = (m0 + wm * 64) / 32 + fp;
          double* o = a.gn_out + (((size_t)b * G + g) * nparts + part) * 2;
          o[0] = s1;
          o[1] = s2;
        }
      }
    }
  };

  // ---- staging cursors and DMA bookkeeping (all wave-uniform) ----
  int issued = 0;                      // global_load_lds (+ epilogue store) instructions this wave issued
  // FIFO of the marks (`issued` right after each staged chunk's rows) not yet waited for: <= NXB-1
  constexpr int NXM = NXB - 1;
  int nX = 0, mX[NXM];
#pragma unroll
  for (int i = 0; i < NXM; ++i) mX[i] = 0;
  int xti = 0, xc = 0, xub = 0;        // next chunk to stage and its row buffer
  int wti = 0, wc = 0, wt = 0, wq = 0, wsl = 0; // next weight step to stage and its ring slot
  int wb, wn0, wm0, xb_, xn0, xm0;  // decoded tiles of the weight / row cursors
  tile_of(0, wb, wn0, wm0);
  tile_of(0, xb_, xn0, xm0);
  auto stage_w = [&]() -> int {
    if (wq < Q) {
      issue_w(wm0, wc, wt, wsl);
      issued += NWW;
      if (++wsl == NWSLOT) wsl = 0;
      if (++wt == taps) {
        wt = 0;
        if (++wc == nch) {
          wc = 0;
          if (++wti < nmine) tile_of(wti, wb, wn0, wm0);
        }
      }
      ++wq;
    }
    return issued;
  };
  auto stage_x = [&]() {
    if (xti < nmine) {
      issue_x(xb_, xn0, xc, xub);
      issued += NXW;
#pragma unroll
      for (int i = 0; i < NXM; ++i)
        if (i == nX) mX[i] = issued;  // constant register index, wave-uniform select
      ++nX;
      if (++xc == nch) {
        xc = 0;
        if (++xti < nmine) tile_of(xti, xb_, xn0, xm0);
      }
      if (++xub == NXB) xub = 0;
    }
  };
  auto pop_x = [&]() -> int {  // mark of the oldest staged chunk not yet waited for
    const int m = nX > 0 ? mX[0] : issued;
#pragma unroll
    for (int i = 0; i + 1 < NXM; ++i) mX[i] = mX[i + 1];
    if (nX > 0) --nX;
    return m;
  };

  // Fragments of one K-slice (ks) of a step: 4 A (weights) + 4 B (frames) x 16 bytes per lane.
  using FT = typename std::conditional<F32, f32x4, bf16x8>::type;  // one 16-byte fragment per lane
  struct Frag {
    FT A[4], B[FN];
  };
  const int ha = l16 & 6;
  auto read_frag = [&](Frag& F, int ks, int slot, int xbuf, int tap) {
    const char* pa = smem + slot * WSLOT + (wm * 64 + l16) * 128;
    const int rb0 = wn * WNC + l16 + tap * dil;
    const int hb = rb0 & 6;
    const char* pb = smem + NWSLOT * WSLOT + xbuf * XBUF + rb0 * 128;
    const int oa = ((ks * 4 + g4) ^ ha) * 16, ob = ((ks * 4 + g4) ^ hb) * 16;
#pragma unroll
    for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const FT*>(pa + f * 2048 + oa);
#pragma unroll
    for (int f = 0; f < FN; ++f) F.B[f] = *reinterpret_cast<const FT*>(pb + f * 2048 + ob);
  };
  // 16 MFMAs of one K-slice with the 8 reads of another slice interleaved, one per MFMA issue slot
  auto mma_slice = [&](const Frag& F) {
#pragma unroll
    for (int fm = 0; fm < 4; ++fm)
#pragma unroll
      for (int fn = 0; fn < FN; ++fn) acc[fm][fn] = mfma16(F.A[fm], F.B[fn], acc[fm][fn]);
    constexpr int NR = 4 + FN, NMF = (F32 ? 16 : 4) * FN;  // reads of the other slice, MFMAs of this one
#pragma unroll
    for (int i = 0; i < NR; ++i) {
      __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);  // MFMA
      __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);  // DS read
    }
    __builtin_amdgcn_sched_group_barrier(0x008, NMF - NR, 0);
  };

  // compile-time K loop (CTN > 0): tiles ti + 0 .. 2 of this workgroup, decoded once (past the last: the last, for
  // the phantom prefetches), before any LDS-DMA is in flight (the compiler would wait for it before the LDS reads)
  struct Tl { int b, n0, m0; };
  auto dec = [&](int ti) {
    Tl r;
    tile_of(min(ti, nmine - 1), r.b, r.n0, r.m0);
    return r;
  };
  Tl tq[3];
  if constexpr (CTN > 0) {
    tq[0] = dec(0);
    tq[1] = dec(1);
    tq[2] = dec(2);
  }
  // ---- prologue: (the tables,) rows of chunks 0 .. NXB-2, weights of steps 0..2, K-slice 0 of step 0 ----
  if (tab_dma) {
    // 1 KiB per wave-instruction (lane-linear), instructions dealt round-robin over the waves; lanes past the
    // table's end read the zero page. Loads retire in order, so the first counted wait covers them.
    const int per = (a.M * 4 + 1023) >> 10;
    for (int j = wave; j < ntab * per; j += 8) {
      const int ti = j / per, part = j - ti * per;
      const int byte = part * 1024 + lane * 16;
      const char* src = byte < a.M * 4 ? reinterpret_cast<const char*>(tabs[ti]) + byte
                                       : reinterpret_cast<const char*>(a.zero) + (lane & 7) * 16;
      glds16(src, smem + toff[ti] + part * 1024);
      ++issued;
    }
  }
  if constexpr (CTN > 0) {
    // ================= compile-time K loop (CTN chunks x CTT taps per tile; see VcSched) =================
    using CS = CtSched<EF, BMT, K1, BNT, CTN, CTT>;
    constexpr int TAPS = CTT, NCHC = CTN, SC = CTN * CTT;
    constexpr int LW = CS::LW, WPW = CS::WPW, XPW = CS::XPW, TX = CS::TX;
    static_assert(CS::NST == NST && FM == 0, "CtSched matches the kernel");
    using SCH = typename CS::SCH;
    const bool loader = wave < LW;
    if (nch != NCHC || taps != TAPS) __builtin_trap();  // the host dispatches on (cin / 64, taps)
    // tiles ti + 0 .. 2 of this workgroup, decoded once (past the last: the last, for the phantom prefetches)
    int sb = 0, xbb = 0;  // ring slot / row buffer of the tile's step 0 / chunk 0 (0 when the period divides)
    auto wslot = [&](int d) {  // ring slot of step d of the tile (d may pass the tile)
      const int r = ((d % NWSLOT) + NWSLOT) % NWSLOT;
      if constexpr (SC % NWSLOT == 0) return r;
      const int v = sb + r;
      return v >= NWSLOT ? v - NWSLOT : v;
    };
    auto xbuf_of = [&](int e) {  // row buffer of chunk e of the tile (e may pass the tile)
      const int r = ((e % NXB) + NXB) % NXB;
      if constexpr (NCHC % NXB == 0) return r;
      const int v = xbb + r;
      return v >= NXB ? v - NXB : v;
    };
    auto ct_w = [&](const Tl& tl, int c, int t, int slot) {  // a loader wave's WPW weight pieces of (c, t)
      const char* base = reinterpret_cast<const char*>(a.w) + ((size_t)(c * TAPS + t) * a.Mpad + tl.m0) * 128;
      // opaque LDS offset and per-step source offsets: a constant destination lets the compiler track the DMA and
      // wait on it before every ds_read; hoisted per-step addresses would take hundreds of VGPRs
      int so = slot * WSLOT + wave * WPW * 1024;
      asm volatile("" : "+s"(so));
#pragma unroll
      for (int i = 0; i < WPW; ++i) {
        const int r = 8 * (wave * WPW + i) + lrow;
        int off = r * 128 + (lp ^ (r & 6)) * 16;
        asm volatile("" : "+v"(off));
        glds16(base + off, smem + so + i * 1024);
      }
    };
    auto ct_x = [&](const Tl& tl, int c, int buf, int part) {  // a loader wave's row pieces `part` of chunk c
      const int f0 = tl.n0 - a.pad;
      const int Lx = rag ? rlv[tl.b] : L;
      const bool lo = c * CHR < c0;
      const int ldx = lo ? c0 : cin - c0;
      const char* xb = lo ? reinterpret_cast<const char*>(a.x) + ((size_t)tl.b * L * c0 + c * CHR) * ES
                          : reinterpret_cast<const char*>(a.x1) + ((size_t)tl.b * L * (cin - c0) + (c * CHR - c0)) * ES;
      int xo = NWSLOT * WSLOT + buf * XBUF;
      asm volatile("" : "+s"(xo));
#pragma unroll
      for (int i = 0; i < XPW; ++i) {
        if (i * TX / XPW != part) continue;
        const int j = wave + LW * i;
        const int r = 8 * j + lrow;
        const int q = lp ^ (r & 6);
        const int f = f0 + r;
        const bool ok = r < R && f >= 0 && f < Lx;
        const char* src = ok ? xb + (size_t)f * ldx * ES + q * 16 : reinterpret_cast<const char*>(a.zero) + q * 16;
        glds16(src, smem + xo + j * 1024);
      }
    };
    auto rd = [&](Frag& F, int ks, int slot, int xbuf, int tap) {  // read_frag with per-step (opaque) bases
      int lb = 0;
      asm volatile("" : "+v"(lb));
      const char* pa = smem + lb + slot * WSLOT + (wm * 64 + l16) * 128;
      const int rb0 = lb + wn * WNC + l16 + tap * dil;
      const int hb = rb0 & 6;
      const char* pb = smem + NWSLOT * WSLOT + xbuf * XBUF + rb0 * 128;
      const int oa = ((ks * 4 + g4) ^ ha) * 16, ob = ((ks * 4 + g4) ^ hb) * 16;
#pragma unroll
      for (int f = 0; f < 4; ++f) F.A[f] = *reinterpret_cast<const FT*>(pa + f * 2048 + oa);
#pragma unroll
      for (int f = 0; f < FN; ++f) F.B[f] = *reinterpret_cast<const FT*>(pb + f * 2048 + ob);
    };
    // the staging ops of (relative) step v of the tile (v < 0: the prologue's virtual steps, which stage only the
    // targets at or past tile 0)
    auto stage_step = [&](auto vc, const Tl* tls) {
      constexpr int v = decltype(vc)::value;
      constexpr int sv = SCH::md(v), t = sv % TAPS;
      if constexpr (t < TX) {
        constexpr int g = SCH::vfloor(v) + NXB - 1;  // target chunk, relative to the tile of step 0
        if constexpr (g >= 0) ct_x(tls[g / NCHC], g % NCHC, xbuf_of(g), t);
      }
      constexpr int q = v + NWSLOT - 1;  // the weight step staged at step v
      if constexpr (q >= 0) ct_w(tls[q / SC], (q % SC) / TAPS, (q % SC) % TAPS, wslot(q));
    };
    static_assert((NCHC + NXB - 2) / NCHC <= 2 && (SC + NWSLOT - 2) / SC <= 2, "stage targets within 2 tiles ahead");
    if (loader) {
      vc_for<SCH::v0, 0>([&](auto vc) { stage_step(vc, tq); });
      vc_wait_vmcnt<SCH::wait_first(-1)>();
    }
    raw_barrier();
    Frag F0, F1;
    rd(F0, 0, wslot(0), xbuf_of(0), 0);
    for (int ti = 0; ti < nmine; ++ti) {
      vc_for<0, SC>([&](auto sc) {
        constexpr int s = decltype(sc)::value;
        constexpr int c = s / TAPS, t = s % TAPS;
        constexpr int s1 = s + 1, c1 = s1 / TAPS, t1 = s1 % TAPS;  // step s + 1 (chunk c1 may be the next tile's)
        __builtin_amdgcn_sched_barrier(0);
        if (loader) {
          if constexpr (SCH::wait_first(s) == SCH::wait(s)) {
            vc_wait_vmcnt<SCH::wait(s)>();
          } else {
            if (ti == 0) vc_wait_vmcnt<SCH::wait_first(s)>();
            else vc_wait_vmcnt<SCH::wait(s)>();
          }
        }
        // no lgkmcnt drain: the LDS reads in flight (the next step's first K-slice) touch neither what this step's
        // DMAs overwrite nor anything another wave writes (the GNRES table is wave-private), mt_rbconv.hip
        raw_barrier();
        if constexpr (s == SC - 1 && (EF & (VE_RESID | VE_ACCUM | VE_LN | VE_MASK | VE_GNRES)) != 0) epi_loads(ti);
        if (loader) stage_step(sc, tq);
        rd(F1, 1, wslot(s), xbuf_of(c), t);
        mma_slice(F0);
        rd(F0, 0, wslot(s1), xbuf_of(c1), t1);
        mma_slice(F1);
        if constexpr (s == SC - 1) {
          __builtin_amdgcn_sched_barrier(0);
          epilogue(ti);
#pragma unroll
          for (int i = 0; i < 4; ++i)
#pragma unroll
            for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        }
      });
      if constexpr (SC % NWSLOT != 0) sb = wslot(SC);
      if constexpr (NCHC % NXB != 0) xbb = xbuf_of(NCHC);
      tq[0] = tq[1];
      tq[1] = tq[2];
      tq[2] = dec(ti + 3);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // phantom prefetches land before the LDS is released
    return;
  }
#pragma unroll
  for (int i = 0; i < NXB - 1; ++i) stage_x();
  const int m0w = stage_w();
  int mW[NWSLOT - 2];  // `issued` after the weights of steps qq+1 .. qq+NWSLOT-2
#pragma unroll
  for (int i = 0; i < NWSLOT - 2; ++i) mW[i] = stage_w();
  wait_vmcnt(issued - max(m0w, pop_x()));
  raw_barrier();
#if defined(VCONV_TS)
  ts_v[1] = __builtin_amdgcn_s_memrealtime();
#endif
  Frag F0, F1;  // F0: slice 0 of the step being computed (read one step ahead), F1: its slice 1
  read_frag(F0, 0, 0, 0, 0);

  int ti = 0, c = 0, t = 0, ub = 0, cs = 0;  // step qq (ub: its row buffer, cs: its weight slot)
  int rt = 0, rub = 0, rs = 0;               // step qq + 1
  for (int qq = 0; qq < Q; ++qq) {
    if (++rs == NWSLOT) rs = 0;
    if (++rt == taps) {
      rt = 0;
      if (++rub == NXB) rub = 0;
    }
    // publish step qq+1's weights (and rows, on a chunk's first tap); every wave's reads of step qq-1
    // are done (lgkmcnt), so its weight slot and, on a chunk change, the old row buffer may be restaged
    if (qq + 1 < Q) wait_vmcnt(issued - (rt == 0 ? max(mW[0], pop_x()) : mW[0]));
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    raw_barrier();
    const bool tile_end = t == taps - 1 && c == nch - 1;
    if constexpr ((EF & (VE_RESID | VE_ACCUM | VE_LN | VE_MASK)) != 0)
      if (tile_end) epi_loads(ti);
    if (t == 0) stage_x();  // rows of chunk u+NXB-1 into the buffer chunk u-1 used
    // weights of step qq + NWSLOT - 1 into the slot step qq-1 used
#pragma unroll
    for (int i = 0; i + 1 < NWSLOT - 2; ++i) mW[i] = mW[i + 1];
    mW[NWSLOT - 3] = stage_w();
    // slice 0 of step qq (registers) || reads of slice 1 of step qq; slice 1 || slice 0 of step qq+1
    read_frag(F1, 1, cs, ub, t);
    mma_slice(F0);
    read_frag(F0, 0, rs, rub, rt);
    mma_slice(F1);
    if (++cs == NWSLOT) cs = 0;
    if (++t == taps) {
      t = 0;
      if (++ub == NXB) ub = 0;
      if (++c == nch) {
        c = 0;
#if defined(VCONV_TS)
        if (ti == 0) ts_v[2] = __builtin_amdgcn_s_memrealtime();
#endif
        epilogue(ti);
        issued += NST;  // its stores join the counted VMEM stream
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < FN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ++ti;
      }
    }
  }
#if defined(VCONV_EXP)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
#endif
#if defined(VCONV_TS)
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the stores have landed
  __syncthreads();
  ts_v[3] = __builtin_amdgcn_s_memrealtime();
  if (a.ts && tid < 4) a.ts[((size_t)a.ts_slot * 256 + blockIdx.x) * 4 + tid] = ts_v[tid];
#endif
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
__global__ void vconv_repack_kernel(const bf16* __restrict__ src, int Mpad0, int taps, int cin_pad, int cin_src,
                                    int cout, int Mpad, size_t total, bf16* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cl = (int)(i & 63);
    size_t r = i >> 6;
    const int m = (int)(r % Mpad);
    r /= Mpad;
    const int t = (int)(r % taps);
    const int c = (int)(r / taps);
    const int ci = c * 64 + cl;
    dst[i] = m < cout && m < Mpad0 && ci < cin_src ? src[((size_t)m * taps + t) * cin_pad + ci] : (bf16)0.f;
  }
}

// k = 3, stride 2, pad 1 conv as a stride-1 conv over frame PAIRS ([T][C] == [T/2][2C] in memory): output j
// = W0 x[2j-1] + W1 x[2j] + W2 x[2j+1] = W'_0 . pair[j-1] + W'_1 . pair[j] with W'_0 = (0 | W0) and
// W'_1 = (W1 | W2) over the pair's (even | odd) channel halves. Source: the generic [Mpad0][3][cin_pad] image.
__global__ void vconv_repack_s2_kernel(const bf16* __restrict__ src, int cin_pad, int C, int cout, int Mpad,
                                       size_t total, bf16* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cl = (int)(i & 63);
    size_t r = i >> 6;
    const int m = (int)(r % Mpad);
    r /= Mpad;
    const int t = (int)(r % 2);
    const int cp = (int)(r / 2) * 64 + cl;  // channel of the pair
    const int odd = cp >= C, ci = odd ? cp - C : cp;
    const int k = t == 0 ? (odd ? 0 : -1) : (odd ? 2 : 1);
    dst[i] = (m < cout && k >= 0) ? src[((size_t)m * 3 + k) * cin_pad + ci] : (bf16)0.f;
  }
}

int vconv_repack_s2(const void* src, int cin_pad, int C, int cout, void* dst, hipStream_t st) {
  MT_REQUIRE(C % 32 == 0 && cin_pad >= C, "vconv_repack_s2: C %d", C);
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  const size_t total = (size_t)(2 * C / 64) * 2 * Mpad * 64;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(vconv_repack_s2_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)src, cin_pad, C, cout, Mpad,
                     total, (bf16*)dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// the VCONV_EXP value this file was built with, or 1 << 8 for the -DVCONV_TS diagnostic build (mt_build_experiments)
int vconv_exp_flags() {
  int f = 0;
#if defined(VCONV_EXP)
  f |= VCONV_EXP == 0 ? 0 : (VCONV_EXP & 0xff) | 1;
#endif
#if defined(VCONV_TS)
  f |= 1 << 8;
#endif
  return f;
}

bool vconv_supported(int cin, int cout, int k, int dil, int stride) {
  // k >= 2 convs stage a chunk's rows during its predecessor's first step and read them a step later;
  // 1x1 convs use the K1 pipeline (rows staged two chunks ahead)
  return stride == 1 && cin % 64 == 0 && cout % 64 == 0 && cout <= MMAX && (k == 1 || BN + (k - 1) * dil <= 320);
}

size_t vconv_packed_bytes(int cin, int cout, int k) {
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  return (size_t)(cin / 64) * k * Mpad * 64 * sizeof(bf16);
}

int vconv_repack(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st,
                 int cin_src) {
  if (cin_src < 0) cin_src = cin;
  MT_REQUIRE(cin % 64 == 0 && cin_pad >= cin_src && cin_src <= cin, "vconv_repack: cin %d (source %d)", cin, cin_src);
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  const size_t total = (size_t)(cin / 64) * taps * Mpad * 64;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(vconv_repack_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)src, Mpad0, taps, cin_pad,
                     cin_src, cout, Mpad, total, (bf16*)dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// fp32 image [cin/32][taps][Mpad][32] (128-byte rows of 32 channels) from the generic fp32 [Mpad0][taps][cin_pad]
__global__ void vconv_repack_f32_kernel(const float* __restrict__ src, int Mpad0, int taps, int cin_pad, int cout,
                                        int Mpad, size_t total, float* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cl = (int)(i & 31);
    size_t r = i >> 5;
    const int m = (int)(r % Mpad);
    r /= Mpad;
    const int t = (int)(r % taps);
    const int c = (int)(r / taps);
    const int ci = c * 32 + cl;
    dst[i] = m < cout && m < Mpad0 && ci < cin_pad ? src[((size_t)m * taps + t) * cin_pad + ci] : 0.f;
  }
}

size_t vconv_packed_bytes_f32(int cin, int cout, int k) {
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  return (size_t)(cin / 32) * k * Mpad * 32 * sizeof(float);
}

int vconv_repack_f32(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st) {
  MT_REQUIRE(cin % 32 == 0 && cin_pad >= cin, "vconv_repack_f32: cin %d", cin);
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  const size_t total = (size_t)(cin / 32) * taps * Mpad * 32;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(vconv_repack_f32_kernel, dim3(blocks), dim3(256), 0, st, (const float*)src, Mpad0, taps, cin_pad,
                     cout, Mpad, total, (float*)dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// split-bf16 image [6 cin / 64][taps][Mpad][64] bf16: input channel cc = p cin + c of plane p holds part
// (0, 1, 2, 0, 1, 0)[p] of the 3-way split of W[m][t][c] (the planes W1 W2 W3 W1 W2 W1 that meet the activation planes
// x1 x1 x1 x2 x2 x3)
__global__ void vconv_repack_split6_kernel(const float* __restrict__ src, int Mpad0, int taps, int cin_pad, int cin,
                                           int cout, int Mpad, size_t total, bf16* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cl = (int)(i & 63);
    size_t r = i >> 6;
    const int m = (int)(r % Mpad);
    r /= Mpad;
    const int t = (int)(r % taps);
    const int cc = (int)(r / taps) * 64 + cl;
    const int p = cc / cin, c = cc - p * cin;
    const float w = m < cout && m < Mpad0 && c < cin_pad ? src[((size_t)m * taps + t) * cin_pad + c] : 0.f;
    bf16 h[3];
    split3_bf16(w, h[0], h[1], h[2]);
    dst[i] = h[p < 3 ? p : p - 3 < 2 ? p - 3 : 0];
  }
}

size_t vconv_packed_bytes_split6(int cin, int cout, int k) { return vconv_packed_bytes(6 * cin, cout, k); }

int vconv_repack_split6(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st) {
  MT_REQUIRE((6 * cin) % 64 == 0 && cin_pad >= cin, "vconv_repack_split6: cin %d", cin);
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  const size_t total = (size_t)(6 * cin / 64) * taps * Mpad * 64;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(vconv_repack_split6_kernel, dim3(blocks), dim3(256), 0, st, (const float*)src, Mpad0, taps, cin_pad,
                     cin, cout, Mpad, total, (bf16*)dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

bool vconv_supported_f32(int cin, int cout, int k, int stride) {
  return stride == 1 && cin % 32 == 0 && cout % 64 == 0 && cout <= MMAX && (k == 1 || BN + (k - 1) <= 320);
}

// MT_XCD_TILES=0 (A/B knob, read once): the round-robin tile walk instead of XCD-major ownership
static int xcd_tiles_knob() {
  static const int v = [] {
    const char* e = getenv("MT_XCD_TILES");
    return e && e[0] == '0' ? 0 : 1;
  }();
  return v;
}

int xcd_remap_enabled() { return xcd_tiles_knob(); }

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

__global__ void vconv_wsum_kernel(const bf16* __restrict__ img, int nk, int Mpad, int cout, float* __restrict__ out) {
  const int m = blockIdx.x * blockDim.x + threadIdx.x;
  if (m >= cout) return;
  float s = 0.f;
  for (int i = 0; i < nk; ++i) {  // (chunk, tap) blocks of [Mpad][64]
    const bf16* r = img + ((size_t)i * Mpad + m) * 64;
    for (int c = 0; c < 64; ++c) s += (float)r[c];
  }
  out[m] = s;
}

int vconv_wsum(const void* img, int cin, int taps, int cout, float* wsum, hipStream_t st) {
  const int Mpad = (cout + BMP - 1) / BMP * BMP;
  hipLaunchKernelGGL(vconv_wsum_kernel, dim3((cout + 255) / 256), dim3(256), 0, st, (const bf16*)img,
                     (cin / 64) * taps, Mpad, cout, wsum);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// Frames per tile of the decoder's k >= 2 GroupNorm-stat / masked convs (128-row tiles): 256, or 192 / 128 when
// the 256-frame grid leaves CUs idle and a finer grid finishes sooner (B = 32: L = 728 gives 192 tiles of 256
// frames but exactly 256 of 192; L = 364 gives 128 tiles of 256 but 192 of 128). A smaller tile carries the same
// per-step barrier and staging overhead for fewer MFMAs: priced as 1.125x (192) / 1.25x (128) its frames.
static int vconv_tile_frames(int B, int L, int Mpad, int ef) {
  if (Mpad % 128 != 0 || (ef != VE_GNSTATS && ef != VE_MASK)) return BN;
  const long cu = cu_count(), ntm = Mpad / 128;
  auto cost = [&](long f, long w) { return ((long)B * ((L + f - 1) / f) * ntm + cu - 1) / cu * f * w; };
  const long c256 = cost(256, 8), c192 = cost(192, 9), c128 = cost(128, 10);
  if (c128 < c256 && c128 <= c192) return 128;
  return c192 < c256 ? 192 : BN;
}

int vconv_gn_parts(int B, int L, int M) {
  const int BM = M % 128 == 0 ? 128 : 64;
  const int bn = vconv_tile_frames(B, L, M, VE_GNSTATS);
  return (L + bn - 1) / bn * (8 / (BM / 64));
}

int vconv_gn_parts_max(int L) { return (L + 127) / 128 * 4; }

// VE_GNRES: a wave's 64 (or 32) frames must span at most 8 utterances (its GN table holds 16 pairs)
int vconv_gnres_min_frames() { return 10; }

#if defined(VCONV_TS)
// diagnostic: phase timestamps of the last TS_SLOTS launches (see VConvArgs::ts); meta per slot = the vclog record
constexpr int TS_SLOTS = 4096;
static unsigned long long* g_ts = nullptr;
static int g_ts_next = 0;
static int g_ts_meta[TS_SLOTS][VCLOG_FIELDS];
static void ts_assign(VConvArgs& a, const int* rec) {
  if (!g_ts && hipMalloc(&g_ts, sizeof(unsigned long long) * TS_SLOTS * 256 * 4) != hipSuccess) g_ts = nullptr;
  a.ts = g_ts;
  a.ts_slot = g_ts_next % TS_SLOTS;
  for (int i = 0; i < VCLOG_FIELDS; ++i) g_ts_meta[a.ts_slot][i] = rec[i];
  ++g_ts_next;
}
#endif

// fp32 operands (mt_encoder): one launch of the F32 kernel; tiles of BM = 128 rows when C_out % 128 == 0, else 64,
// and 128 frames (k >= 2: 64-row tiles hold 384 / 128 frames as in bf16; 1x1: the cost model's 128 / 192 / 256)
static int launch_vconv_split(int ef, const VConvArgs& a0, hipStream_t st);
static int launch_vconv_f32(int ef, const VConvArgs& a0, hipStream_t st) {
  if (a0.f32 == 2) return launch_vconv_split(ef, a0, st);
  MT_REQUIRE(a0.cin % 32 == 0 && a0.M % 64 == 0 && a0.Mpad == a0.M && a0.M <= MMAX && a0.c0 == 0 && !a0.Lout &&
                 !a0.ldy && (a0.taps == 1 || BN + (a0.taps - 1) * a0.dil <= 320),
             "vconv f32: geometry (cin %d, M %d, taps %d)", a0.cin, a0.M, a0.taps);
  MT_REQUIRE(!(ef & VE_SPLIT6), "vconv f32: VE_SPLIT6 is a split-bf16 (f32 = 2) epilogue");
  MT_REQUIRE(!(ef & VE_RESID) || a0.resid, "vconv f32: resid");
  MT_REQUIRE(!(ef & VE_MASK) || a0.emask, "vconv f32: mask");
  VConvArgs a = a0;
  a.c0 = a.cin;
  a.xcd_tiles = xcd_tiles_knob();
  const bool k1 = a.taps == 1;
  if (k1) {
    MT_REQUIRE(a0.pad == 0, "vconv f32: 1x1 conv with padding");
    a.L = a0.B * a0.L;
    a.B = 1;
  }
  a.Lout = a.L;
  a.ldy = a.M;
  a.ylim = a.L * a.M;
  a.ystride = (long long)a.L * a.M;
  // tile (rows x frames) by rounds of tiles over the CUs x tile size (an fp32 tile is MFMA-bound: no fixed-cost
  // weight): 128 x 128 / 128 x 256 / 64 x 128, ties to the larger tile (the text encoder's FFN conv1, 768 rows at
  // B = 32: 384 tiles of 128 x 128 = 2 rounds of 256 CUs, 768 tiles of 64 x 128 = 3 rounds of half the work)
  const long cu = cu_count();
  auto rounds = [&](long bm, long f) {
    return ((long)a.B * ((a.L + f - 1) / f) * (a.Mpad / bm) + cu - 1) / cu * bm * f;
  };
  int BM = a.M % 128 == 0 ? 128 : 64, bn = 128;
  if (BM == 128) {
    if (rounds(128, 256) < rounds(128, 128)) bn = 256;
    if (rounds(64, 128) < rounds(128, bn)) BM = 64, bn = 128;
  }
  const long ntiles = (long)a.B * ((a.L + bn - 1) / bn) * (a.Mpad / BM);
  const int G = (int)std::min<long>(ntiles, cu);
  {
    const int rec[VCLOG_FIELDS] = {ef | (1 << 20), BM, bn, (int)k1, (int)ntiles, G, a.taps, a.M, a.cin, a.B, a.L};
    vclog_record(rec);
#if defined(VCONV_TS)
    ts_assign(a, rec);
#endif
  }
#define MT_F32CASE(E)                                                                                              \
  case E:                                                                                                          \
    if (k1) {                                                                                                      \
      if (BM == 128 && bn == 256) hipLaunchKernelGGL((vconv_kernel<E, 128, true, 256, 1>), dim3(G), dim3(NT), 0, st, a); \
      else if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, true, 128, 1>), dim3(G), dim3(NT), 0, st, a); \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, true, 128, 1>), dim3(G), dim3(NT), 0, st, a);                \
    } else {                                                                                                       \
      if (BM == 128 && bn == 256) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 256, 1>), dim3(G), dim3(NT), 0, st, a); \
      else if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 128, 1>), dim3(G), dim3(NT), 0, st, a); \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, false, 128, 1>), dim3(G), dim3(NT), 0, st, a);               \
    }                                                                                                              \
    break;
  switch (ef) {
    MT_F32CASE(0)
    MT_F32CASE(VE_RELU)
    MT_F32CASE(VE_RELU | VE_MASK)
    MT_F32CASE(VE_MASK)
    MT_F32CASE(VE_RESID)
    MT_F32CASE(VE_RESID | VE_MASK)
    default: set_error("vconv f32: epilogue %d not compiled in", ef); return -1;
  }
#undef MT_F32CASE
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

// split-bf16 mode (VConvArgs::f32 == 2; the text encoder's FFN convs): the bf16 K loop over cin = 6 cin0 channels
// (the operands' six planes), the fp32 epilogue; k >= 2 tiles of 128 x 256 frames (C_out % 128 == 0) or 64 x 128,
// chosen by rounds of tiles as the fp32 launcher does (the K loop is MFMA-bound: 6 bf16 products per fp32 product)
static int launch_vconv_split(int ef, const VConvArgs& a0, hipStream_t st) {
  MT_REQUIRE(a0.cin % 384 == 0 && a0.M % 64 == 0 && a0.Mpad == a0.M && a0.M <= MMAX && a0.c0 == 0 && !a0.Lout &&
                 !a0.ldy && a0.taps >= 2 && BN + (a0.taps - 1) * a0.dil <= 320 && !a0.lens,
             "vconv split: geometry (cin %d = 6 x a multiple of 64, M %d, taps %d >= 2)", a0.cin, a0.M, a0.taps);
  MT_REQUIRE(!(ef & VE_RESID) || a0.resid, "vconv split: resid");
  MT_REQUIRE(!(ef & VE_MASK) || a0.emask, "vconv split: mask");
  VConvArgs a = a0;
  a.c0 = a.cin;
  a.xcd_tiles = xcd_tiles_knob();
  a.Lout = a.L;
  a.ldy = a.M;
  a.ylim = a.L * a.M;
  a.ystride = (long long)a.L * a.M;
  const long cu = cu_count();
  auto rounds = [&](long bm, long f) {
    return ((long)a.B * ((a.L + f - 1) / f) * (a.Mpad / bm) + cu - 1) / cu * bm * f;
  };
  // 64-row tiles (C_out = 192: conv 2) span 384 frames (24 MFMAs per wave per step: the 216-step K loop is bound by
  // its per-step cost at 128 frames, 776 vs 580 us for the fp32 kernel at B = 256)
  int BM = a.M % 128 == 0 ? 128 : 64, bn = BM == 128 ? 256 : 384;
  if (BM == 128 && rounds(128, 128) < rounds(128, 256)) bn = 128;
  if (BM == 64 && rounds(64, 128) < rounds(64, 384)) bn = 128;  // small batches: fill the CUs first
  const long ntiles = (long)a.B * ((a.L + bn - 1) / bn) * (a.Mpad / BM);
  const int G = (int)std::min<long>(ntiles, cu);
  {
    const int rec[VCLOG_FIELDS] = {ef | (2 << 20), BM, bn, 0, (int)ntiles, G, a.taps, a.M, a.cin, a.B, a.L};
    vclog_record(rec);
#if defined(VCONV_TS)
    ts_assign(a, rec);
#endif
  }
#define MT_SPLCASE(E)                                                                                            \
  case E:                                                                                                        \
    if (BM == 128 && bn == 256) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 256, 2>), dim3(G), dim3(NT), 0, st, a); \
    else if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 128, 2>), dim3(G), dim3(NT), 0, st, a); \
    else hipLaunchKernelGGL((vconv_kernel<E, 64, false, 384, 2>), dim3(G), dim3(NT), 0, st, a);               \
    break;
  switch (ef) {
    MT_SPLCASE(VE_RELU | VE_MASK | VE_SPLIT6)
    MT_SPLCASE(VE_RESID | VE_MASK)
    default: set_error("vconv split: epilogue %d not compiled in", ef); return -1;
  }
#undef MT_SPLCASE
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}


// Compile-time K-loop variants (CTN chunks x CTT taps; VcSched): the decoder's convs and the upsamplers, each
// (epilogue, tile) with the (C_in / 64, taps) pairs its launches have; other shapes run the runtime-cursor loop.
// MT_VCONV_CT=0 in the environment or mt_vconv_set_ct(0): the runtime-cursor loop everywhere (A/B, tests: the two
// are bit-identical, same tiles and MFMA order).
static int g_ct = -1;
static bool ct_on() {
  if (g_ct < 0) {
    const char* e = getenv("MT_VCONV_CT");
    g_ct = e && e[0] == '0' ? 0 : 1;
  }
  return g_ct != 0;
}
int vconv_set_ct(int enable) {
  const int prev = ct_on() ? 1 : 0;
  g_ct = enable ? 1 : 0;
  return prev;
}
int vconv_path_id() {
  const int rb = rbconv_set(1);  // read the rbconv setting (and restore it)
  rbconv_set(rb);
  return (ct_on() ? 2 : 0) | rb;
}
template <int E, int BMV, bool K1V, int BNV>
static void ct_try(const VConvArgs&, int, hipStream_t, bool&) {}
template <int E, int BMV, bool K1V, int BNV, int N, int T, int... R>
static void ct_try(const VConvArgs& a, int G, hipStream_t st, bool& done) {
  (void)CtSched<E, BMV, K1V, BNV, N, T>::REG::reg;  // the schedule, for the CPU schedule test
  if (a.cin / 64 == N && a.taps == T) {
    hipLaunchKernelGGL((vconv_kernel<E, BMV, K1V, BNV, 0, N, T>), dim3(G), dim3(NT), 0, st, a);
    done = true;
    return;
  }
  ct_try<E, BMV, K1V, BNV, R...>(a, G, st, done);
}
// launch vconv_kernel<E, BMV, K1V, BNV>, on its compile-time K loop when (C_in / 64, taps) is one of the pairs P
template <int E, int BMV, bool K1V, int BNV, int... P>
static void vlaunch(const VConvArgs& a, int G, hipStream_t st) {
  bool done = false;
  if (ct_on()) ct_try<E, BMV, K1V, BNV, P...>(a, G, st, done);
  if (!done) hipLaunchKernelGGL((vconv_kernel<E, BMV, K1V, BNV>), dim3(G), dim3(NT), 0, st, a);
}

int launch_vconv(int ef, const VConvArgs& a0, hipStream_t st) {
  MT_REQUIRE(a0.x && a0.w && a0.bias && a0.y && a0.zero && a0.trash, "vconv: null pointer");
  MT_REQUIRE(!(ef & VE_DIV) || div_rn_ok(a0.div), "vconv: VE_DIV divisor %g outside the exactly-checked set (div_rn)", (double)a0.div);
  if (a0.f32) return launch_vconv_f32(ef, a0, st);
  MT_REQUIRE(a0.B > 0 && a0.L > 0 && a0.cin % 64 == 0 && a0.M % 64 == 0 && a0.Mpad == a0.M && a0.M <= MMAX,
             "vconv: geometry");
  MT_REQUIRE(a0.taps >= 1 && a0.dil >= 1 && (a0.taps == 1 || BN + (a0.taps - 1) * a0.dil <= 320),
             "vconv: taps %d dil %d", a0.taps, a0.dil);
  MT_REQUIRE(!(ef & VE_RESID) || a0.resid, "vconv: resid");
  MT_REQUIRE(!(ef & VE_DUAL) || a0.y2, "vconv: y2");
  MT_REQUIRE(!(ef & VE_LN) || (a0.ln_stats && a0.wsum), "vconv: LN stats / weight sums");
  MT_REQUIRE(!(ef & VE_LNP) || ((ef & VE_LN) && a0.ln_eps > 0.f && a0.cin == 256),
             "vconv: LN partials need VE_LN, eps and 256 input channels (4 slabs)");
  MT_REQUIRE(!(ef & VE_ROWSTATS) || a0.row_out, "vconv: row statistics output");
  MT_REQUIRE(!(ef & VE_SNAKE) || (a0.snake_alpha && a0.snake_ibeta), "vconv: snake params");
  MT_REQUIRE(!(ef & VE_MASK) || a0.emask, "vconv: mask");
  MT_REQUIRE(!(ef & VE_GNSTATS) || (a0.gn_out && a0.taps > 1 && a0.M % 32 == 0), "vconv: GN statistics");
  MT_REQUIRE(!(ef & VE_GNRES) || ((ef & VE_RESID) && !(ef & VE_MASK) && a0.taps == 1 && a0.gn_in && a0.gn_gamma &&
                                  a0.gn_beta && a0.emask && a0.gn_in_parts > 0 && a0.gn_B == a0.B &&
                                  a0.gn_T == a0.L && a0.gn_T >= vconv_gnres_min_frames() && a0.M % 64 == 0),
             "vconv: residual GroupNorm (1x1, resid, partials, gamma / beta, mask, T >= %d)", vconv_gnres_min_frames());
  VConvArgs a = a0;
  a.xcd_tiles = xcd_tiles_knob();
  if (a.c0 == 0) a.c0 = a.cin;  // one source
  MT_REQUIRE(a.c0 == a.cin || (a.x1 && a.c0 % 64 == 0 && a.c0 > 0 && a.c0 < a.cin), "vconv: channel split %d/%d",
             a.c0, a.cin);
  const bool k1 = a0.taps == 1;
  const bool placed = a0.Lout || a0.ldy || a0.yshift || a0.ylim || a0.ystride;
  MT_REQUIRE(!(ef & VE_PMASK) || (a0.emask && a0.mask_div > 0 && a0.ylim % a0.mask_div == 0 && a0.mask_div % 32 == 0),
             "vconv: placed-output mask");
  MT_REQUIRE(!placed || (!k1 && (ef & ~(VE_DUAL | VE_PMASK)) == 0 && a0.Lout > 0 && a0.ldy >= a0.M && a0.ylim > 0 &&
                         a0.ystride >= a0.ylim && a0.yshift % 8 == 0 && a0.ldy % 8 == 0),
             "vconv: placed output (ConvTranspose) geometry / epilogue %d", ef);
  if (k1) {  // no halo: the utterances' frames are one contiguous sequence of B*L columns
    MT_REQUIRE(a0.pad == 0, "vconv: 1x1 conv with padding");
    a.L = a0.B * a0.L;
    a.B = 1;
  }
  if (!placed) {
    MT_REQUIRE((long long)a.L * a.M < (1ll << 31), "vconv: %d frames x %d channels", a.L, a.M);
    a.Lout = a.L;
    a.ldy = a.M;
    a.ylim = a.L * a.M;
    a.ystride = (long long)a.L * a.M;
  }
  const int BM = a.M % 128 == 0 ? 128 : 64;
  long ntiles = (long)a.B * ((a.Lout + BN - 1) / BN) * (a.Mpad / BM);
  // 1x1 GEMMs whose 256-frame tiles would leave CUs idle (the decoder's half-resolution blocks):
  // 128-frame tiles double the parallelism
#ifndef VCONV_SMALL_MULT
#define VCONV_SMALL_MULT 1
#endif
  // tile width by the k >= 2 convs' cost model (rounds of tiles x frames x per-frame weight 8 / 9 / 10 for 256 /
  // 192 / 128 frames: a smaller tile amortises its fixed per-tile work over fewer frames);
  // MT_K1_TILES=0 (A/B knob, read once): the round-2 rule (128 only when 256-frame tiles leave CUs idle)
  static const int k1_model = [] {
    const char* e = getenv("MT_K1_TILES");
    return e && e[0] == '0' ? 0 : 1;
  }();
  bool small = k1 && ntiles < (long)VCONV_SMALL_MULT * cu_count();
  int tf1 = k1 ? (small ? 128 : BN) : 0;  // 1x1 tile frames: 256, 192 or 128
  if (k1 && k1_model) {
    const long cu = cu_count(), ntm = a.Mpad / BM;
    auto cost = [&](long f, long w) { return (((long)a.L + f - 1) / f * ntm + cu - 1) / cu * f * w; };
    const long c256 = cost(256, 8), c192 = BM == 128 ? cost(192, 9) : LONG_MAX, c128 = cost(128, 10);
    tf1 = (c128 < c256 && c128 <= c192) ? 128 : c192 < c256 ? 192 : BN;
    small = tf1 == 128;
  }
  if (k1 && tf1 != BN) ntiles = (long)((a.L + tf1 - 1) / tf1) * (a.Mpad / BM);
  // k >= 2 convs with 64-row tiles take 384 frames per tile: 1.5x the MFMAs per step barrier
  constexpr int BN64 = 384;
  if (!k1 && BM == 64) ntiles = (long)a.B * ((a.Lout + BN64 - 1) / BN64) * (a.Mpad / BM);
  // the text encoder's FFN conv2 (k = 3, 192 rows -> 64-row tiles) on short utterances: 128-frame tiles when the
  // 384-frame grid leaves CUs idle (same cost model, 384-frame tiles weighted 7.5 per frame); 64-row tiles of
  // 128 frames run one fragment per wave
  bool bm64_128 = false;
  if (!k1 && BM == 64 && !placed && ef == (VE_RESID | VE_MASK)) {
    const long cu = cu_count(), ntm = a.Mpad / BM;
    const long t384 = (long)a.B * ((a.L + 383) / 384) * ntm, t128 = (long)a.B * ((a.L + 127) / 128) * ntm;
    bm64_128 = (t128 + cu - 1) / cu * 128 * 10 < (t384 + cu - 1) / cu * 384 * 15 / 2;
    if (bm64_128) ntiles = t128;
  }
  MT_REQUIRE(!(ef & VE_GNSTATS) || BM == 128, "vconv: GroupNorm partials need 128-row tiles");
  const int tf = (!k1 && !placed) ? vconv_tile_frames(a.B, a.L, a.Mpad, ef) : BN;  // 256, 192 or 128
  if (tf != BN) ntiles = (long)a.B * ((a.L + tf - 1) / tf) * (a.Mpad / BM);
  const int G = (int)std::min<long>(ntiles, cu_count());
  // XCD-major ownership pays where a launch's activations fit the XCDs' L2 (the decoder at B = 32: CFM solve
  // 8.71 -> 8.61 ms); on larger grids (B = 256: 40.2 vs 40.5 ms) the round-robin walk's weight reuse wins
  a.xcd_tiles = a.xcd_tiles && ntiles <= 3L * G;
  MT_REQUIRE(!(ef & VE_GNSTATS) || a0.gn_parts == 0 || a0.gn_parts == ((a.L + tf - 1) / tf) * (8 / (BM / 64)),
             "vconv: caller expects %d GroupNorm partial slots, the launch writes a different count", a0.gn_parts);
  {
    const int bn = k1 ? tf1 : (BM == 64 ? (bm64_128 ? 128 : 384) : tf);
    const int rec[VCLOG_FIELDS] = {ef, BM, bn, (int)k1, (int)ntiles, G, a.taps, a.M, a.cin, a.B, a.L};
    vclog_record(rec);
#if defined(VCONV_TS)
    ts_assign(a, rec);
#endif
  }
  const double flops = 2.0 * a.M * a.cin * a.taps * (double)a.B * a.Lout;
  // algorithmic bytes by SURVEY.md §8d's layer-boundary definition: the conv reads its input once and writes
  // its output once (bf16), + its weights; the residual / accumulator / activated-copy traffic this
  // implementation adds is NOT counted (it shows up as the PMC traffic ratio instead)
  const double bytes = 2.0 * a.B * ((double)a.L * a.cin + (double)a.Lout * a.M) + 2.0 * a.M * a.cin * a.taps;
  // the probe site covers the HiFi-GAN ResBlock convs (k >= 3), the bench's roofline family
  const int site = a.probe ? a.probe : PROBE_VCONV;
  const bool probed = !k1 && site > 0;
  // VE_Y2ONLY: only mt_rbconv honours it; the generic kernels store y as well (correct either way)
  if ((ef & VE_Y2ONLY) && !(!k1 && !placed && BM == 128 && rbconv_handles(ef, a))) ef &= ~VE_Y2ONLY;
  // VE_ACTIN exists only on mt_rbconv; its producers store no activated copy, so a launch it does not take must fail
  // here by name (the vocoder's stage_actin predicts acceptance from the same shape fields)
  MT_REQUIRE(!(ef & VE_ACTIN) || (!k1 && !placed && BM == 128 && rbconv_handles(ef, a)),
             "vconv: VE_ACTIN launch not taken by mt_rbconv (cin %d M %d k %d d %d B %d): stage_actin and the launch "
             "arguments disagree", a.cin, a.M, a.taps, a.dil, a.B);
  if (!k1 && !placed && BM == 128 && rbconv_handles(ef, a)) {  // the HiFi-GAN wide-stage ResBlock convs (mt_rbconv)
    if (probed) probe_begin(site, st);
    const int rc = launch_rbconv(ef, a, G, st);
    if (rc) return rc;
    if (probed) probe_end(site, st, flops, bytes, PROBE_TAG_RBCONV);
    return 0;
  }
  if (probed) probe_begin(site, st);
#define MT_VCASE(E)                                                                                \
  case E:                                                                                          \
    if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, false>), dim3(G), dim3(NT), 0, st, a); \
    else hipLaunchKernelGGL((vconv_kernel<E, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);     \
    break;
#define MT_VCASE_H(E)                                                                                  \
  case E:                                                                                              \
    if (tf == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 128>), dim3(G), dim3(NT), 0, st, a); \
    else if (tf == 192) hipLaunchKernelGGL((vconv_kernel<E, 128, false, 192>), dim3(G), dim3(NT), 0, st, a); \
    else if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, false>), dim3(G), dim3(NT), 0, st, a); \
    else hipLaunchKernelGGL((vconv_kernel<E, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);          \
    break;
#define MT_VCASE1(E)                                                                                    \
  case E:                                                                                               \
    if (tf1 == 128) {                                                                                   \
      if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, true, 128>), dim3(G), dim3(NT), 0, st, a); \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, true, 128>), dim3(G), dim3(NT), 0, st, a);           \
    } else if (tf1 == 192) { /* BM = 128 only (64-row tiles would give 24-frame waves) */               \
      hipLaunchKernelGGL((vconv_kernel<E, 128, true, 192>), dim3(G), dim3(NT), 0, st, a);               \
    } else {                                                                                            \
      if (BM == 128) hipLaunchKernelGGL((vconv_kernel<E, 128, true>), dim3(G), dim3(NT), 0, st, a);     \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, true>), dim3(G), dim3(NT), 0, st, a);                \
    }                                                                                                   \
    break;
#define MT_VCASE_HCT(E)                                                                                \
  case E:                                                                                              \
    if (tf == 128) vlaunch<E, 128, false, 128, 3, 3, 4, 3, 8, 3, 8, 2>(a, G, st);                        \
    else if (tf == 192) vlaunch<E, 128, false, 192, 3, 3, 4, 3, 8, 3, 8, 2>(a, G, st);                   \
    else if (BM == 128) vlaunch<E, 128, false, BN, 3, 3, 4, 3, 8, 3, 8, 2>(a, G, st);                    \
    else hipLaunchKernelGGL((vconv_kernel<E, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);          \
    break;
#define MT_VCASE1CT(E, ...)                                                                             \
  case E:                                                                                               \
    if (tf1 == 128) {                                                                                   \
      if (BM == 128) vlaunch<E, 128, true, 128, __VA_ARGS__>(a, G, st);                                 \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, true, 128>), dim3(G), dim3(NT), 0, st, a);           \
    } else if (tf1 == 192) {                                                                            \
      vlaunch<E, 128, true, 192, __VA_ARGS__>(a, G, st);                                                \
    } else {                                                                                            \
      if (BM == 128) vlaunch<E, 128, true, BN, __VA_ARGS__>(a, G, st);                                  \
      else hipLaunchKernelGGL((vconv_kernel<E, 64, true>), dim3(G), dim3(NT), 0, st, a);                \
    }                                                                                                   \
    break;
  if (!k1) {
    switch (ef) {
      MT_VCASE(VE_ACT)
      MT_VCASE(VE_RESID | VE_DUAL)
      MT_VCASE(VE_RESID)
      MT_VCASE(VE_RESID | VE_ACCUM)
      MT_VCASE(VE_RESID | VE_DIV)
      MT_VCASE(VE_RESID | VE_ACCUM | VE_DIV)
      MT_VCASE_HCT(VE_GNSTATS)
      MT_VCASE_HCT(VE_MASK)
      case VE_DUAL:  // the upsamplers (placed polyphase output)
        if (BM == 128) vlaunch<VE_DUAL, 128, false, BN, 8, 2, 4, 2, 2, 2>(a, G, st);
        else hipLaunchKernelGGL((vconv_kernel<VE_DUAL, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);
        break;
      MT_VCASE(VE_RELU | VE_MASK)
      case VE_PMASK:  // the decoder's ConvTranspose up conv
        if (BM == 128) vlaunch<VE_PMASK, 128, false, BN, 4, 2>(a, G, st);
        else hipLaunchKernelGGL((vconv_kernel<VE_PMASK, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);
        break;
      case VE_RESID | VE_MASK:
        if (bm64_128) hipLaunchKernelGGL((vconv_kernel<VE_RESID | VE_MASK, 64, false, 128>), dim3(G), dim3(NT), 0, st, a);
        else if (BM == 128) hipLaunchKernelGGL((vconv_kernel<VE_RESID | VE_MASK, 128, false>), dim3(G), dim3(NT), 0, st, a);
        else hipLaunchKernelGGL((vconv_kernel<VE_RESID | VE_MASK, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);
        break;
      MT_VCASE(VE_RESID | VE_DIV | VE_DUAL)
      MT_VCASE(VE_RESID | VE_ACCUM | VE_DIV | VE_DUAL)
      case 0:  // plain: the upsamplers whose stage activates its input itself (VE_ACTIN), compile-time K loops
#if defined(VCONV_UP_NOCT)  // A/B build: the runtime-cursor loop
        if (BM == 128) hipLaunchKernelGGL((vconv_kernel<0, 128, false>), dim3(G), dim3(NT), 0, st, a);
#else
        if (BM == 128) vlaunch<0, 128, false, BN, 8, 2, 4, 2, 2, 2>(a, G, st);
#endif
        else hipLaunchKernelGGL((vconv_kernel<0, 64, false, BN64>), dim3(G), dim3(NT), 0, st, a);
        break;
      default: set_error("vconv: epilogue %d not compiled in", ef); return -1;
    }
  } else {
    switch (ef) {
      MT_VCASE1(VE_LN)
      MT_VCASE1(VE_LN | VE_SNAKE)
      MT_VCASE1(VE_RESID)
      MT_VCASE1CT(VE_RESID | VE_MASK, 16, 1, 2, 1)
      MT_VCASE1CT(VE_RESID | VE_ROWSTATS, 2, 1, 16, 1)
      MT_VCASE1CT(VE_RESID | VE_ROWSTATS | VE_GNRES, 3, 1, 4, 1, 8, 1)
      MT_VCASE1CT(VE_LN | VE_LNP, 4, 1)
      MT_VCASE1CT(VE_LN | VE_LNP | VE_SNAKE, 4, 1)
      MT_VCASE1(0)
      default: set_error("vconv: 1x1 epilogue %d not compiled in", ef); return -1;
    }
  }
#undef MT_VCASE
#undef MT_VCASE_H
#undef MT_VCASE_HCT
#undef MT_VCASE1
#undef MT_VCASE1CT
  MT_CHECK_HIP(hipGetLastError());
  if (probed) probe_end(site, st, flops, bytes);
  return 0;
}

}  // namespace mt

#if defined(VCONV_TS)
// diagnostic export (not in include/matcha_hip.h; only the -DVCONV_TS build has it): copies the timestamps and the
// per-launch records of the launches since the last call (at most TS_SLOTS); returns their count
extern "C" int mt_vconv_ts_dump(unsigned long long* ts, int* meta, int max_slots) {
  const int n = std::min(std::min(mt::g_ts_next, mt::TS_SLOTS), max_slots);
  if (n > 0 && mt::g_ts) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpy(ts, mt::g_ts, sizeof(unsigned long long) * n * 256 * 4, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    for (int i = 0; i < n; ++i)
      for (int j = 0; j < mt::VCLOG_FIELDS; ++j) meta[i * mt::VCLOG_FIELDS + j] = mt::g_ts_meta[i][j];
  }
  mt::g_ts_next = 0;
  return n;
}
#endif
