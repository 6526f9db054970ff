// Persistent LDS-DMA implicit-GEMM Conv1d for the wide HiFi-GAN ResBlock convs (gfx950, bf16).
//
// GEMM view (same as mt_conv.h): rows m = output channels, columns n = output frames of one
// utterance, K = taps x C_in. One workgroup = 8 waves (2 in M x 4 in N, 64x64 per wave,
// v_mfma_f32_16x16x32_bf16) owns a 128 x 256 output tile at a time and walks the tiles
// gl, gl + G, gl + 2G, ... (G = one workgroup per CU; gl groups consecutive tiles on workgroups that
// share an XCD, so the tiles that read the same input rows / weights meet in one L2).
//
// K loop of a tile: for each 64-channel chunk c, for each tap t: one "step" =
//   A = W[c][t] (128 rows x 128 B, one 16 KiB slot of a 4-slot ring)
//   B = X rows n0 - pad + t*dil + [0, 256) of chunk c (one of two 40 KiB row buffers; the chunk's
//       rows are staged ONCE and every tap reads them shifted by t*dil rows)
//   32 MFMAs per wave (2 K-slices x 4 x 4 fragments).
// Every byte is staged by global_load_lds_dwordx4 (1 KiB per wave-instruction, lane-linear LDS
// image); LDS rows are 128 B with the 16-byte chunk XOR-swizzled by (row >> 1) & 7 on the SOURCE
// address and on the ds_read (cdna_hip_programming.md rule 21), so the 16-lane ds_read_b128 groups
// of an MFMA fragment hit 16 distinct bank slots. Weights of step s+3 and the rows of chunk u+1 are
// in flight while step s computes: each wave counts the DMA instructions it issued and waits with a
// COUNTED `s_waitcnt vmcnt(N)` for exactly the ones the step needs, then one raw s_barrier per step
// publishes them (no __syncthreads: its fence would drain the prefetch). The loop runs across tile
// boundaries, so the next tile's first weights and rows land while this tile's epilogue stores.
// Zero padding (frames outside [0, L)) is read from a zero page instead of branching.
#include <algorithm>

#include "mt_probe.h"
#include "mt_vconv.h"

namespace mt {

namespace {
constexpr int BM = 128, BN = 256, NT = 512;
constexpr int WSLOT = BM * 128;                   // 16 KiB: 128 rows x 64 bf16 channels
constexpr int NWSLOT = 4;                         // weight ring depth (3 steps in flight)
constexpr int XROWS = 320;                        // >= BN + (taps - 1) * dil
constexpr int XBUF = XROWS * 128;                 // 40 KiB per chunk buffer
constexpr int LDS_BYTES = NWSLOT * WSLOT + 2 * XBUF;  // 144 KiB
constexpr int NXW = XROWS / 8 / 8;                // X wave-instructions per wave per chunk
constexpr int NWW = BM / 8 / 8;                   // W wave-instructions per wave per step
static_assert(LDS_BYTES <= 160 * 1024, "LDS budget");
}  // namespace

__device__ __forceinline__ void glds16(const void* src, char* lds_wave_base) {
  __builtin_amdgcn_global_load_lds(src, (__attribute__((address_space(3))) void*)lds_wave_base, 16, 0, 0);
}

// s_waitcnt vmcnt(n) for a wave-uniform runtime n (n > 15 waits for 15: stricter, still correct)
__device__ __forceinline__ void wait_vmcnt(int n) {
#define MT_VMW(k) \
  case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
  switch (n) {
    MT_VMW(0) MT_VMW(1) MT_VMW(2) MT_VMW(3) MT_VMW(4) MT_VMW(5) MT_VMW(6) MT_VMW(7)
    MT_VMW(8) MT_VMW(9) MT_VMW(10) MT_VMW(11) MT_VMW(12) MT_VMW(13) MT_VMW(14)
    default: asm volatile("s_waitcnt vmcnt(15)" ::: "memory"); break;
  }
#undef MT_VMW
}

__device__ __forceinline__ void raw_barrier() {
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
  __builtin_amdgcn_sched_barrier(0);
}

template <int EF>
__global__ __launch_bounds__(NT) void vconv_kernel(VConvArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[LDS_BYTES];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave & 1, wn = wave >> 1;
  const int taps = a.taps, dil = a.dil, L = a.L, cin = a.cin;
  const int nch = cin >> 6;
  const int S = nch * taps;
  const int ntn = (L + BN - 1) / BN, ntm = a.Mpad / BM;
  const int ntiles = a.B * ntn * ntm;
  const int G = gridDim.x, g = blockIdx.x;
  const int gl = (G % 8 == 0) ? (g % 8) * (G / 8) + g / 8 : g;
  const int nmine = gl < ntiles ? (ntiles - gl + G - 1) / G : 0;
  const int Q = nmine * S;
  if (Q == 0) return;

  auto tile_of = [&](int ti, int& b, int& n0, int& m0) {
    const int tile = gl + ti * G;
    const int r = tile / ntm;
    m0 = (tile - r * ntm) * BM;
    b = r / ntn;
    n0 = (r - b * ntn) * BN;
  };

  const int lrow = lane >> 3, lp = lane & 7;
  auto issue_w = [&](int ti, int c, int t, int slot) {
    int b, n0, m0;
    tile_of(ti, b, n0, m0);
    const bf16* base = a.w + ((size_t)(c * taps + t) * a.Mpad + m0) * 64;
    char* dst = smem + slot * WSLOT;
#pragma unroll
    for (int i = 0; i < NWW; ++i) {
      const int j = wave * NWW + i;
      const int r = 8 * j + lrow;
      const int q = lp ^ ((r >> 1) & 7);
      glds16(base + r * 64 + q * 8, dst + j * 1024);
    }
  };
  auto issue_x = [&](int ti, int c, int buf) {
    int b, n0, m0;
    tile_of(ti, b, n0, m0);
    const int R = BN + (taps - 1) * dil;
    const int f0 = n0 - a.pad;
    const bf16* xb = a.x + (size_t)b * L * cin + c * 64;
    char* dst = smem + NWSLOT * WSLOT + buf * XBUF;
#pragma unroll
    for (int i = 0; i < NXW; ++i) {
      const int j = wave + 8 * i;
      const int r = 8 * j + lrow;
      const int q = lp ^ ((r >> 1) & 7);
      const int f = f0 + r;
      const bool ok = r < R && f >= 0 && f < L;
      const bf16* src = ok ? xb + (size_t)f * cin + q * 8 : a.zero + q * 8;
      glds16(src, dst + j * 1024);
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g4 = lane >> 4, l16 = lane & 15;
  auto epilogue = [&](int ti) {
    int b, n0, m0;
    tile_of(ti, b, n0, m0);
    const size_t rowbase = (size_t)b * L;
#pragma unroll
    for (int fm = 0; fm < 4; ++fm) {
      const int m = m0 + wm * 64 + fm * 16 + 4 * g4;
      if (m >= a.M) continue;
      const f32x4 bias4 = *reinterpret_cast<const f32x4*>(a.bias + m);
#pragma unroll
      for (int fn = 0; fn < 4; ++fn) {
        const int n = n0 + wn * 64 + fn * 16 + l16;
        if (n >= L) continue;
        const size_t o = (rowbase + n) * a.M + m;
        float v[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[fm][fn][r] + bias4[r];
        if constexpr ((EF & VE_RESID) != 0) {
          const bf16x4 rv = *reinterpret_cast<const bf16x4*>(a.resid + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] + (float)rv[r];
        }
        if constexpr ((EF & VE_ACCUM) != 0) {
          const bf16x4 yv = *reinterpret_cast<const bf16x4*>(a.y + o);
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = (float)yv[r] + v[r];
        }
        if constexpr ((EF & VE_DIV) != 0) {
#pragma unroll
          for (int r = 0; r < 4; ++r) v[r] = v[r] / a.div;
        }
        bf16x4 o1, o2;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const bf16 rv = (bf16)v[r];
          const bf16 av = (bf16)lrelu_f((float)rv, a.slope);
          o1[r] = (EF & VE_ACT) ? av : rv;
          o2[r] = av;
        }
        *reinterpret_cast<bf16x4*>(a.y + o) = o1;
        if constexpr ((EF & VE_DUAL) != 0) *reinterpret_cast<bf16x4*>(a.y2 + o) = o2;
      }
    }
  };

  // ---- prologue: rows of chunk 0, weights of steps 0..2 ----
  int issued = 0, mX = 0, mW0 = 0, mW1 = 0, mW2 = 0;
  int xti = 0, xc = 0, xu = 0;  // next chunk to stage
  int wti = 0, wc = 0, wt = 0, wq = 0;  // next weight step to stage
  auto adv_x = [&]() {
    if (++xc == nch) {
      xc = 0;
      ++xti;
    }
    ++xu;
  };
  auto adv_w = [&]() {
    if (++wt == taps) {
      wt = 0;
      if (++wc == nch) {
        wc = 0;
        ++wti;
      }
    }
    ++wq;
  };
  issue_x(0, 0, 0);
  issued += NXW;
  mX = issued;
  adv_x();
#pragma unroll
  for (int i = 0; i < 3; ++i) {
    int mk = issued;
    if (wq < Q) {
      issue_w(wti, wc, wt, wq & 3);
      issued += NWW;
      mk = issued;
      adv_w();
    }
    if (i == 0) mW0 = mk;
    else if (i == 1) mW1 = mk;
    else mW2 = mk;
  }

  int ti = 0, c = 0, t = 0, u = 0;
  for (int qq = 0; qq < Q; ++qq) {
    // ---- wait for this step's weights (and, on a chunk's first tap, its rows); publish ----
    const int need = t == 0 ? max(mW0, mX) : mW0;
    wait_vmcnt(issued - need);
    raw_barrier();
    // ---- stage ahead: rows of the next chunk (on its predecessor's first tap), weights of step qq+3 ----
    if (t == 0 && xti < nmine) {
      issue_x(xti, xc, xu & 1);
      issued += NXW;
      mX = issued;
      adv_x();
    }
    int mk = issued;
    if (wq < Q) {
      issue_w(wti, wc, wt, wq & 3);
      issued += NWW;
      mk = issued;
      adv_w();
    }
    mW0 = mW1;
    mW1 = mW2;
    mW2 = mk;

    // ---- MFMAs of step qq ----
    const char* Ws = smem + (qq & 3) * WSLOT;
    const char* Xs = smem + NWSLOT * WSLOT + (u & 1) * XBUF;
    const int ha = (l16 >> 1) & 7;
    const char* pa = Ws + (wm * 64 + l16) * 128;
    const int rb0 = wn * 64 + l16 + t * dil;
    const int hb = (rb0 >> 1) & 7;
    const char* pb = Xs + rb0 * 128;
    bf16x8 A[2][4], Bf[2][4];
#pragma unroll
    for (int ks = 0; ks < 2; ++ks) {
      const int oa = ((ks * 4 + g4) ^ ha) * 16, ob = ((ks * 4 + g4) ^ hb) * 16;
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        A[ks][f] = *reinterpret_cast<const bf16x8*>(pa + f * 2048 + oa);
        Bf[ks][f] = *reinterpret_cast<const bf16x8*>(pb + f * 2048 + ob);
      }
    }
#pragma unroll
    for (int ks = 0; ks < 2; ++ks)
#pragma unroll
      for (int fm = 0; fm < 4; ++fm)
#pragma unroll
        for (int fn = 0; fn < 4; ++fn) acc[fm][fn] = mfma16(A[ks][fm], Bf[ks][fn], acc[fm][fn]);

    // ---- tile done: epilogue, reset ----
    if (++t == taps) {
      t = 0;
      ++u;
      if (++c == nch) {
        c = 0;
        epilogue(ti);
#pragma unroll
        for (int i = 0; i < 4; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        ++ti;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// host side
// ------------------------------------------------------------------------------------
__global__ void vconv_repack_kernel(const bf16* __restrict__ src, int Mpad0, int taps, int cin_pad, int cout,
                                    int Mpad, size_t total, bf16* __restrict__ dst) {
  for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < total; i += (size_t)gridDim.x * blockDim.x) {
    const int cl = (int)(i & 63);
    size_t r = i >> 6;
    const int m = (int)(r % Mpad);
    r /= Mpad;
    const int t = (int)(r % taps);
    const int c = (int)(r / taps);
    const int ci = c * 64 + cl;
    dst[i] = m < cout && m < Mpad0 ? src[((size_t)m * taps + t) * cin_pad + ci] : (bf16)0.f;
  }
}

bool vconv_supported(int cin, int cout, int k, int dil, int stride) {
  return stride == 1 && cin % 64 == 0 && cout % BM == 0 && BN + (k - 1) * dil <= XROWS;
}

size_t vconv_packed_bytes(int cin, int cout, int k) {
  const int Mpad = (cout + BM - 1) / BM * BM;
  return (size_t)(cin / 64) * k * Mpad * 64 * sizeof(bf16);
}

int vconv_repack(const void* src, int Mpad0, int taps, int cin_pad, int cin, int cout, void* dst, hipStream_t st) {
  MT_REQUIRE(cin % 64 == 0 && cin_pad >= cin, "vconv_repack: cin %d", cin);
  const int Mpad = (cout + BM - 1) / BM * BM;
  const size_t total = (size_t)(cin / 64) * taps * Mpad * 64;
  const int blocks = (int)std::min<size_t>((total + 255) / 256, 65535);
  hipLaunchKernelGGL(vconv_repack_kernel, dim3(blocks), dim3(256), 0, st, (const bf16*)src, Mpad0, taps, cin_pad,
                     cout, Mpad, total, (bf16*)dst);
  MT_CHECK_HIP(hipGetLastError());
  return 0;
}

static int cu_count() {
  static int n = 0;
  if (n == 0) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0)
      n = 256;
  }
  return n;
}

int launch_vconv(int ef, const VConvArgs& a, hipStream_t st) {
  MT_REQUIRE(a.x && a.w && a.bias && a.y && a.zero, "vconv: null pointer");
  MT_REQUIRE(a.B > 0 && a.L > 0 && a.cin % 64 == 0 && a.M % BM == 0 && a.Mpad == a.M, "vconv: geometry");
  MT_REQUIRE(a.taps >= 1 && a.dil >= 1 && BN + (a.taps - 1) * a.dil <= XROWS, "vconv: taps %d dil %d", a.taps, a.dil);
  MT_REQUIRE(!(ef & VE_RESID) || a.resid, "vconv: resid");
  MT_REQUIRE(!(ef & VE_DUAL) || a.y2, "vconv: y2");
  const long ntiles = (long)a.B * ((a.L + BN - 1) / BN) * (a.Mpad / BM);
  const int G = (int)std::min<long>(ntiles, cu_count());
  const double flops = 2.0 * a.M * a.cin * a.taps * (double)a.B * a.L;
  const int touts = 1 + ((ef & VE_RESID) ? 1 : 0) + ((ef & VE_ACCUM) ? 1 : 0) + ((ef & VE_DUAL) ? 1 : 0);
  const double bytes = 2.0 * a.B * a.L * ((double)a.cin + (double)a.M * touts) + 2.0 * a.M * a.cin * a.taps;
  probe_begin(PROBE_VCONV, st);
#define MT_VCASE(E)                                                                  \
  case E: hipLaunchKernelGGL(vconv_kernel<E>, dim3(G), dim3(NT), 0, st, a); break;
  switch (ef) {
    MT_VCASE(VE_ACT)
    MT_VCASE(VE_RESID | VE_DUAL)
    MT_VCASE(VE_RESID)
    MT_VCASE(VE_RESID | VE_ACCUM)
    MT_VCASE(VE_RESID | VE_DIV)
    MT_VCASE(VE_RESID | VE_ACCUM | VE_DIV)
    MT_VCASE(0)
    default: set_error("vconv: epilogue %d not compiled in", ef); return -1;
  }
#undef MT_VCASE
  MT_CHECK_HIP(hipGetLastError());
  probe_end(PROBE_VCONV, st, flops, bytes);
  return 0;
}

}  // namespace mt
