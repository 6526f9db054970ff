// Fused HiFi-GAN ResBlock1 stage for the small-channel stages (C = 32, 64) on gfx950.
//
//   y = ( rb_0(x) + rb_1(x) + ... ) / nk,   rb_j(x): 3 x [ t = conv_{k_j, d}(lrelu x);
//                                                       x = conv_{k_j, 1}(lrelu t) + x ]
// (hifigan/models.py:90-97, 187-192). One workgroup = 8 waves = one (utterance, tile of N output
// frames). The input tile with its receptive-field halo H = max_j (k_j-1)/2 * (sum d + 3) is read
// from HBM (and re-read from L2 per resblock); every intermediate lives in LDS:
//   S   chain state x_i    (residual), SL = lrelu(S) (first-conv input)
//   T   lrelu(conv1 out)   (conv2 input)
// Weights are not staged: each wave streams the A fragments of its 32 output channels straight
// from L1/L2 into registers one K chunk (4 taps x 64 bytes) ahead, across conv boundaries too.
// Each conv computes exactly the rows the rest of the chain needs (ranges shrink towards the N
// output rows). Rows whose frame lies outside [0, L) are forced to 0 — that is the zero padding the
// per-layer convs apply — so results match the per-layer path. Rounding points are the same as the
// per-layer bf16 path (every intermediate stored in the element type, the resblock sum rounded after
// each add), and the MFMA accumulation order per output equals the per-layer TConv tile's (taps in
// groups of 4, 64-byte channel slices inside), so the two paths agree bit for bit.
#include "mt_rbfuse.h"
#include "mt_probe.h"

#include <algorithm>
#include <type_traits>

namespace mt {

template <class E, int C, int N>
struct RBTile {
  static constexpr int NT = 512, NW = 8;
  static constexpr int HMAX = 60;
  static constexpr int W0 = N + 2 * HMAX;
  // rows padded by 32 bytes: the MFMA fragment reads (16 rows x 4 16-byte columns, ds_read_b128 lane
  // groups {0-3,12-15,20-27}, ...) then hit 16 distinct 16-byte bank slots per group
  static constexpr int ROW = C * (int)sizeof(E) + 32;
  static constexpr int KC = C * (int)sizeof(E) / 64;   // 64-byte K slices per row
  static constexpr int VPR = C * (int)sizeof(E) / 16;  // 16-byte vectors per row
  static constexpr int FMJ = 2;                        // job = 32 output channels x 16 frames
  static constexpr int CB = C / 32;                    // channel blocks (a wave keeps one)
  static constexpr int WPC = NW / CB;                  // waves per channel block
  static constexpr int JPW = ((W0 + 15) / 16 + WPC - 1) / WPC;  // frame blocks per wave (widest conv)
  static constexpr int OJ = N / 16 / WPC;              // frame blocks per wave in the last conv
  // +16 spare rows: a partial last frame block reads up to 15 rows past the conv's input rows
  // (those columns are discarded), which must stay inside the buffer set
  static constexpr int BUF = (W0 + 16) * ROW;
  static constexpr int LDS = 3 * BUF;
  static_assert(LDS <= 160 * 1024, "LDS budget");
  static_assert(N % (16 * WPC) == 0, "output frame blocks must split evenly over the waves");
};

// A fragments of one K chunk = (4-tap group g, 64-byte slice kc): [tap in group][row block].
// Taps past the kernel are clamped (loaded, never used) so every chunk issues the same loads.
template <class E, int C, int FMJ>
__device__ __forceinline__ void rb_load_chunk(const E* wl, int kk, int g, int kc, Vec16<E> (&A)[4][FMJ]) {
  constexpr int EPS = 64 / (int)sizeof(E);
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int t = min(4 * g + i, kk - 1);
#pragma unroll
    for (int x = 0; x < FMJ; ++x) A[i][x] = load16(wl + ((size_t)x * 16 * kk + t) * C + kc * EPS);
  }
}

// NG taps x NJ frame blocks of one chunk: all B fragments first, then the MFMAs (tap-major, the
// per-layer tile's accumulation order).
template <class E, int NG, int NJ, int JPW, int FMJ, int ROW, int WPC>
__device__ __forceinline__ void rb_chunk(const char* bsrc, int row0, int g, int d, const Vec16<E> (&A)[4][FMJ],
                                         f32x4 (&acc)[JPW][FMJ]) {
  Vec16<E> Bf[NG][NJ];
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj)
      Bf[i][jj] = load16(reinterpret_cast<const E*>(bsrc + (row0 + jj * WPC * 16 + (4 * g + i) * d) * ROW));
#pragma unroll
  for (int i = 0; i < NG; ++i)
#pragma unroll
    for (int jj = 0; jj < NJ; ++jj)
#pragma unroll
      for (int x = 0; x < FMJ; ++x) acc[jj][x] = mfma16(A[i][x].v, Bf[i][jj].v, acc[jj][x]);
}

template <class E, int NJ, int JPW, int FMJ, int ROW, int WPC>
__device__ __forceinline__ void rb_chunk_ng(int ng, const char* bsrc, int row0, int g, int d,
                                            const Vec16<E> (&A)[4][FMJ], f32x4 (&acc)[JPW][FMJ]) {
  switch (ng) {
    case 4: rb_chunk<E, 4, NJ, JPW, FMJ, ROW, WPC>(bsrc, row0, g, d, A, acc); break;
    case 3: rb_chunk<E, 3, NJ, JPW, FMJ, ROW, WPC>(bsrc, row0, g, d, A, acc); break;
    case 2: rb_chunk<E, 2, NJ, JPW, FMJ, ROW, WPC>(bsrc, row0, g, d, A, acc); break;
    default: rb_chunk<E, 1, NJ, JPW, FMJ, ROW, WPC>(bsrc, row0, g, d, A, acc); break;
  }
}

template <class E, int JPW, int FMJ, int ROW, int WPC>
__device__ __forceinline__ void rb_chunk_dispatch(int nj, int ng, const char* bsrc, int row0, int g, int d,
                                                  const Vec16<E> (&A)[4][FMJ], f32x4 (&acc)[JPW][FMJ]) {
  static_assert(JPW <= 5, "frame blocks per wave");
  switch (nj) {
    case 1: rb_chunk_ng<E, 1, JPW, FMJ, ROW, WPC>(ng, bsrc, row0, g, d, A, acc); break;
    case 2: rb_chunk_ng<E, 2, JPW, FMJ, ROW, WPC>(ng, bsrc, row0, g, d, A, acc); break;
    case 3: rb_chunk_ng<E, 3, JPW, FMJ, ROW, WPC>(ng, bsrc, row0, g, d, A, acc); break;
    case 4:
      if constexpr (JPW >= 4) rb_chunk_ng<E, 4, JPW, FMJ, ROW, WPC>(ng, bsrc, row0, g, d, A, acc);
      break;
    case 5:
      if constexpr (JPW >= 5) rb_chunk_ng<E, 5, JPW, FMJ, ROW, WPC>(ng, bsrc, row0, g, d, A, acc);
      break;
    default: break;
  }
}

// bf16 epilogue helpers (mt_common.h): packed fp32 pairs, one v_cvt_pk_bf16_f32 per pair, max-form lrelu
__device__ __forceinline__ uint32_t rb_pack(f32x2 v) { return pk_bf16(v); }
__device__ __forceinline__ f32x2 rb_unpack(uint32_t w) { return unpk_bf16(w); }
__device__ __forceinline__ f32x2 rb_lrelu(f32x2 t, float slope) { return lrelu2(t, slope); }

template <class E, int C, int N>
__global__ __launch_bounds__(512) void rbfuse_kernel(RBArgs a) {
  using TL = RBTile<E, C, N>;
  constexpr int ROW = TL::ROW, KC = TL::KC, FMJ = TL::FMJ, JPW = TL::JPW, OJ = TL::OJ, WPC = TL::WPC;
  constexpr int VN = Vec16<E>::N;
  __shared__ __attribute__((aligned(16))) char smem[TL::LDS];
  char* S = smem;            // chain state (residual)
  char* SL = S + TL::BUF;    // lrelu(S): first-conv input
  char* T = SL + TL::BUF;    // lrelu(first-conv output): second-conv input

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cbk = wave % TL::CB;   // this wave's 32 output channels
  const int fw = wave / TL::CB;    // this wave's frame-block phase (0 .. WPC-1)
  const int ntile = (a.L + N - 1) / N;
  const int b = blockIdx.x / ntile, f0 = (blockIdx.x % ntile) * N;
  const int hm = a.hmax;
  const int fbase = f0 - hm;  // frame of local row 0
  const int W0 = N + 2 * hm;
  const E* X = reinterpret_cast<const E*>(a.x) + (size_t)b * a.L * C;
  E* Y = reinterpret_cast<E*>(a.y) + (size_t)b * a.L * C;
  const int np2 = 2 * a.npair, ncv = a.nk * np2;

  // per-lane base of this wave's weight rows for a conv: rows cbk*32 + x*16 + (lane & 15),
  // K elements (lane >> 4) * 8 .. +7 of each 64-byte slice
  auto wlane = [&](int c) -> const E* {
    const int j = c / np2, i = (c % np2) >> 1;
    const RBConv& cv = (c & 1) ? a.c2[j][i] : a.c1[j][i];
    return reinterpret_cast<const E*>(cv.w) + ((size_t)(cbk * 32 + (lane & 15)) * a.k[j]) * C + (lane >> 4) * VN;
  };

  // running resblock sum of this wave's output blocks (E-rounded values; bf16: packed pairs)
  constexpr bool BF = std::is_same<E, bf16>::value;
  float out[BF ? 1 : OJ][FMJ][4];
  uint32_t outp[BF ? OJ : 1][FMJ][2];
#pragma unroll
  for (int o = 0; o < (BF ? OJ : 1); ++o)
#pragma unroll
    for (int x = 0; x < FMJ; ++x) outp[o][x][0] = outp[o][x][1] = 0u;
#pragma unroll
  for (int o = 0; o < (BF ? 1 : OJ); ++o)
#pragma unroll
    for (int x = 0; x < FMJ; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) out[o][x][r] = 0.f;

  // The stage input tile (+ halo) stays in registers for the whole kernel: every resblock restarts its
  // chain from it without another trip to L2 / HBM (and without a load stall behind a barrier).
  // (C = 32 only: at C = 64 the tile would push the kernel past its register budget)
  constexpr bool XREG = C == 32;
  constexpr int XV = XREG ? (TL::W0 * TL::VPR + TL::NT - 1) / TL::NT : 1;
  Vec16<E> xr[XV];
  if constexpr (XREG) {
#pragma unroll
    for (int k = 0; k < XV; ++k) {
      const int v = tid + k * TL::NT;
      const int r = v / TL::VPR, sl = v % TL::VPR;
      const int f = fbase + r;
      xr[k] = zero16<E>();
      if (r < W0 && f >= 0 && f < a.L) xr[k] = load16(X + (size_t)f * C + sl * VN);
    }
  }

  // A fragments ping-pong between A0 / A1 (no register copies); A0 holds the next conv's first chunk
  Vec16<E> A0[4][FMJ], A1[4][FMJ];
  rb_load_chunk<E, C, FMJ>(wlane(0), a.k[0], 0, 0, A0);
  const bool interior = fbase >= 0 && fbase + W0 <= a.L;  // no tile row outside the sequence

  for (int c = 0; c < ncv; ++c) {
    const int j = c / np2, i = (c % np2) >> 1, half = c & 1;
    const int kk = a.k[j], q = (kk - 1) / 2;
    const bool last = i == a.npair - 1;
    const RBConv& cv = half == 0 ? a.c1[j][i] : a.c2[j][i];
    const int d = half == 0 ? a.dil[j][i] : 1;
    const int qd = q * d;
    const int ra = half == 0 ? a.r1a[j][i] : a.r2a[j][i];
    const int rb = half == 0 ? a.r1b[j][i] : a.r2b[j][i];
    const int nfb = (rb - ra + 15) / 16;
    const int nj = nfb > fw ? min(JPW, (nfb - fw + WPC - 1) / WPC) : 0;  // wave-uniform
    float bias[FMJ][4];
#pragma unroll
    for (int x = 0; x < FMJ; ++x)
#pragma unroll
      for (int r = 0; r < 4; ++r) bias[x][r] = cv.bias[cbk * 32 + x * 16 + 4 * (lane >> 4) + r];

    if (half == 0 && (c % np2) == 0) {
      // ---- new resblock: S = x, SL = lrelu(x) over tile + halo (0 outside [0, L)). The previous conv's
      // closing barrier already ordered every read of S / SL before these writes.
      if constexpr (XREG) {
#pragma unroll
        for (int k = 0; k < XV; ++k) {
          const int v = tid + k * TL::NT;
          const int r = v / TL::VPR, sl = v % TL::VPR;
          if (r >= W0) break;
          Vec16<E> act;
#pragma unroll
          for (int e = 0; e < VN; ++e) act.set(e, lrelu_f(xr[k].get(e), a.slope));
          store16(reinterpret_cast<E*>(S + r * ROW + sl * 16), xr[k]);
          store16(reinterpret_cast<E*>(SL + r * ROW + sl * 16), act);
        }
      } else {
        // x is L2-resident: re-read it per resblock
        for (int v = tid; v < W0 * TL::VPR; v += TL::NT) {
          const int r = v / TL::VPR, sl = v % TL::VPR;
          const int f = fbase + r;
          Vec16<E> raw = zero16<E>(), act = zero16<E>();
          if (f >= 0 && f < a.L) {
            raw = load16(X + (size_t)f * C + sl * VN);
#pragma unroll
            for (int e = 0; e < VN; ++e) act.set(e, lrelu_f(raw.get(e), a.slope));
          }
          store16(reinterpret_cast<E*>(S + r * ROW + sl * 16), raw);
          store16(reinterpret_cast<E*>(SL + r * ROW + sl * 16), act);
        }
      }
      __syncthreads();
    }

    // ---- MFMA phase: K chunks (g, kc) in the per-layer tile's order; the next chunk (or the next
    // conv's first chunk) is in flight while this one computes ----
    const char* src = half == 0 ? SL : T;
    f32x4 acc[JPW][FMJ];
#pragma unroll
    for (int jj = 0; jj < JPW; ++jj)
#pragma unroll
      for (int x = 0; x < FMJ; ++x) acc[jj][x] = f32x4{0.f, 0.f, 0.f, 0.f};
    const E* wl = wlane(c);
    const int ngroups = (kk + 3) / 4, nchunks = ngroups * KC;
    const int cn = c + 1 < ncv ? c + 1 : c;
    const int row0 = ra + fw * 16 + (lane & 15) - qd;
    const char* bsrc = src + (lane >> 4) * 16;
    for (int ch = 0;;) {
      if (ch + 1 < nchunks) rb_load_chunk<E, C, FMJ>(wl, kk, (ch + 1) / KC, (ch + 1) % KC, A1);
      rb_chunk_dispatch<E, JPW, FMJ, ROW, WPC>(nj, min(4, kk - 4 * (ch / KC)), bsrc + (ch % KC) * 64, row0, ch / KC,
                                               d, A0, acc);
      if (++ch == nchunks) break;
      if (ch + 1 < nchunks) rb_load_chunk<E, C, FMJ>(wl, kk, (ch + 1) / KC, (ch + 1) % KC, A0);
      rb_chunk_dispatch<E, JPW, FMJ, ROW, WPC>(nj, min(4, kk - 4 * (ch / KC)), bsrc + (ch % KC) * 64, row0, ch / KC,
                                               d, A1, acc);
      if (++ch == nchunks) break;
    }
    // the next conv's first chunk is in flight during this conv's epilogue
    rb_load_chunk<E, C, FMJ>(wlane(cn), a.k[cn / np2], 0, 0, A0);
    // No barrier here: this conv's epilogue writes T (conv1) or S / SL (conv2), none of which its own MFMA
    // phase reads (src is SL for conv1, T for conv2); the writes only race with the NEXT conv's reads,
    // which the barrier after the epilogue orders.

    // ---- epilogue ----
#pragma unroll
    for (int jj = 0; jj < JPW; ++jj) {
      if (jj >= nj) break;
      const int row = ra + (fw + jj * WPC) * 16 + (lane & 15);
      if (row >= rb) continue;
      const int f = fbase + row;
      const bool inseq = interior || (f >= 0 && f < a.L);
#pragma unroll
      for (int x = 0; x < FMJ; ++x) {
        const int ch = cbk * 32 + x * 16 + 4 * (lane >> 4);
        if constexpr (BF) {
          // 4 consecutive channels of one frame per lane: one 8-byte LDS access instead of four 2-byte ones
          f32x2 v01 = f32x2{acc[jj][x][0], acc[jj][x][1]} + f32x2{bias[x][0], bias[x][1]};
          f32x2 v23 = f32x2{acc[jj][x][2], acc[jj][x][3]} + f32x2{bias[x][2], bias[x][3]};
          if (half == 0) {
            uint2 w = make_uint2(rb_pack(rb_lrelu(rb_unpack(rb_pack(v01)), a.slope)),
                                 rb_pack(rb_lrelu(rb_unpack(rb_pack(v23)), a.slope)));
            if (!inseq) w = make_uint2(0u, 0u);
            *reinterpret_cast<uint2*>(T + row * ROW + ch * 2) = w;
            continue;
          }
          const uint2 sr = *reinterpret_cast<const uint2*>(S + row * ROW + ch * 2);
          v01 += rb_unpack(sr.x);
          v23 += rb_unpack(sr.y);
          if (!last) {
            uint2 ws = make_uint2(rb_pack(v01), rb_pack(v23));
            if (!inseq) ws = make_uint2(0u, 0u);
            *reinterpret_cast<uint2*>(S + row * ROW + ch * 2) = ws;
            *reinterpret_cast<uint2*>(SL + row * ROW + ch * 2) =
                make_uint2(rb_pack(rb_lrelu(rb_unpack(ws.x), a.slope)), rb_pack(rb_lrelu(rb_unpack(ws.y), a.slope)));
            continue;
          }
          if (jj < OJ) {
            // xs = rb_0; xs += rb_j (rounded to bf16 after every add, as the per-layer path stores xs);
            // the last add is followed by / nk before rounding
            if (j != 0) {
              v01 += rb_unpack(outp[jj][x][0]);
              v23 += rb_unpack(outp[jj][x][1]);
            }
            if (j == a.nk - 1) {
              v01 = f32x2{v01.x / a.div, v01.y / a.div};
              v23 = f32x2{v23.x / a.div, v23.y / a.div};
            }
            outp[jj][x][0] = rb_pack(v01);
            outp[jj][x][1] = rb_pack(v23);
          }
          continue;
        } else {
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[jj][x][r] + bias[x][r];
        if (half == 0) {
          E* tp = reinterpret_cast<E*>(T + row * ROW) + ch;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float tv = to_f(from_f<E>(v[r]));
            tp[r] = from_f<E>(inseq ? lrelu_f(tv, a.slope) : 0.f);
          }
          continue;
        }
        const E* sp = reinterpret_cast<const E*>(S + row * ROW) + ch;
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = v[r] + to_f(sp[r]);
        if (!last) {
          E* sw = reinterpret_cast<E*>(S + row * ROW) + ch;
          E* lw = reinterpret_cast<E*>(SL + row * ROW) + ch;
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            const float sv = inseq ? to_f(from_f<E>(v[r])) : 0.f;
            sw[r] = from_f<E>(sv);
            lw[r] = from_f<E>(lrelu_f(sv, a.slope));
          }
          continue;
        }
        if (jj < OJ) {
          // xs = rb_0; xs += rb_j (rounded to E after every add, as the per-layer path
          // stores xs); the last add is followed by / nk before rounding
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            float o = j == 0 ? v[r] : out[jj][x][r] + v[r];
            if (j == a.nk - 1) o = o / a.div;
            out[jj][x][r] = to_f(from_f<E>(o));
          }
        }
        }
      }
    }
    __syncthreads();  // dst complete before the next conv reads it
  }

  // ---- write the stage output (rows hm .. hm+N-1 = frames f0 .. f0+N-1) ----
#pragma unroll
  for (int o = 0; o < OJ; ++o) {
    const int f = f0 + (fw + o * WPC) * 16 + (lane & 15);
    if (f >= a.L) continue;
#pragma unroll
    for (int x = 0; x < FMJ; ++x) {
      E* yp = Y + (size_t)f * C + cbk * 32 + x * 16 + 4 * (lane >> 4);
      if constexpr (BF) {
        *reinterpret_cast<uint2*>(yp) = make_uint2(outp[o][x][0], outp[o][x][1]);
      } else {
#pragma unroll
        for (int r = 0; r < 4; ++r) yp[r] = from_f<E>(out[o][x][r]);
      }
    }
  }
}

int launch_rbfuse(int dtype, int C, const RBArgs& a, hipStream_t st) {
  MT_REQUIRE(a.hmax <= 60 && a.nk >= 1 && a.nk <= 3 && a.npair >= 1 && a.npair <= 3,
             "rbfuse: unsupported resblock configuration");
  // algorithmic work: 2*npair convs of C x C x k per resblock on B*L frames; the stage reads x
  // and writes y once, plus its weights
  double flops = 0, wbytes = 0;
  const int es = dtype == BF16 ? 2 : 4;
  for (int j = 0; j < a.nk; ++j) {
    flops += 2.0 * a.npair * 2.0 * C * C * a.k[j] * (double)a.B * a.L;
    wbytes += 2.0 * a.npair * ((double)C * C * a.k[j] * es + C * 4.0);
  }
  const double bytes = 2.0 * a.B * a.L * C * es + wbytes;
  const int site = C == 64 ? PROBE_RBFUSE_C64 : PROBE_RBFUSE_C32;
  probe_begin(site, st);
  if (dtype == BF16 && C == 32) {
    constexpr int N = 384;
    dim3 grid((unsigned)(a.B * ((a.L + N - 1) / N)));
    hipLaunchKernelGGL((rbfuse_kernel<bf16, 32, N>), grid, dim3(512), 0, st, a);
  } else if (dtype == BF16 && C == 64) {
    constexpr int N = 192;
    dim3 grid((unsigned)(a.B * ((a.L + N - 1) / N)));
    hipLaunchKernelGGL((rbfuse_kernel<bf16, 64, N>), grid, dim3(512), 0, st, a);
  } else {
    set_error("rbfuse: no fused kernel for dtype %d C %d", dtype, C);
    return -1;
  }
  MT_CHECK_HIP(hipGetLastError());
  probe_end(site, st, flops, bytes, PROBE_TAG_RBFUSE);
  return 0;
}

bool rbfuse_supported(int dtype, int C) { return dtype == BF16 && (C == 32 || C == 64); }

int rbfuse_tile_n(int C) { return C == 32 ? 384 : 192; }

}  // namespace mt
