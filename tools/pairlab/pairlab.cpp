// pairlab: standalone timing, bit-identity and phase-stamp harness for the HiFi-GAN ResBlock pair kernels (no torch).
// tools/pairlab/build.sh compiles the kernel sources several times into namespaces: mt_base (a git revision, the
// reference), mt (the working tree), mt_ts (the working tree with -DVPAIR_TS phase stamps, mt_ts.h) and one mt_<v> per
// experiment variant. Inputs are synthetic (random bf16 rows and weights; timing does not depend on the values).
// Every build is timed against mt_base in alternating blocks of launches, and compared with it bit for bit.
// Usage: pairlab KIND K D B L [EF] [REPS] [RAGGED]
//   KIND 32 | 64 | 128 (mt_vpair32 / mt_vpair (+ vpair3 for k = 3) / mt_vpair128), EF the epilogue flags (VE_*),
//   RAGGED 1: utterance lengths drawn in [0.6 L, L] (the bench's ragged vocoder), 0: every utterance has L frames.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mt_vpair.h"

namespace mt {
const char* last_error();
}  // namespace mt
namespace mt_ts {
struct VPairArgs;
int launch_vpair(int ef, const VPairArgs& a, hipStream_t st);
int launch_vpair32(int ef, const VPairArgs& a, hipStream_t st);
int launch_vpair128(int ef, const VPairArgs& a, hipStream_t st);
int vpair_ts_bind(unsigned long long* p);
int vpair32_ts_bind(unsigned long long* p);
int vpair128_ts_bind(unsigned long long* p);
}  // namespace mt_ts
namespace mt_base {
struct VPairArgs;
int launch_vpair(int ef, const VPairArgs& a, hipStream_t st);
int launch_vpair32(int ef, const VPairArgs& a, hipStream_t st);
int launch_vpair128(int ef, const VPairArgs& a, hipStream_t st);
}  // namespace mt_base

using Launch = int (*)(int, const void*, hipStream_t);
struct Build {
  std::string name;
  Launch l32, l64, l128;
};
#define LAUNCHERS(ns)                                                                             \
  reinterpret_cast<Launch>(static_cast<int (*)(int, const ns::VPairArgs&, hipStream_t)>(ns::launch_vpair32)), \
  reinterpret_cast<Launch>(static_cast<int (*)(int, const ns::VPairArgs&, hipStream_t)>(ns::launch_vpair)),   \
  reinterpret_cast<Launch>(static_cast<int (*)(int, const ns::VPairArgs&, hipStream_t)>(ns::launch_vpair128))
#include "variants_decl.inc"

#define CK(x)                                                                               \
  do {                                                                                      \
    hipError_t e_ = (x);                                                                    \
    if (e_ != hipSuccess) {                                                                 \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_));     \
      exit(1);                                                                              \
    }                                                                                       \
  } while (0)

static uint16_t to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static const char* PHASES[12] = {"x-wait", "x-barrier", "resid+bar", "lrelu+bar", "conv1", "epi1",
                                 "T-bar/steps", "conv2", "accum-wait", "epi2", "tile-head", "drain"};
// the split-phase 32-channel kernel's stamps (mt_vpair32.hip vpair32s_kernel)
static const char* PHASES32S[12] = {"A:resid+lrelu", "A-bar", "B:conv1", "B-bar", "C:epi1", "C-bar",
                                    "D:conv2", "D:epi2", "D:x-wait", "D-bar", "idle", "C:dma"};
static const char** PH = PHASES;

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: pairlab KIND K D B L [EF] [REPS] [RAGGED]\n");
    return 2;
  }
  const int kind = atoi(argv[1]), k = atoi(argv[2]), d = atoi(argv[3]), B = atoi(argv[4]), L = atoi(argv[5]);
  const int ef = argc > 6 ? atoi(argv[6]) : 0, reps = argc > 7 ? atoi(argv[7]) : 20;
  const int ragged = argc > 8 ? atoi(argv[8]) : 1;
  const int C = kind;
  using namespace mt;
  std::vector<Build> builds = {{"base", LAUNCHERS(mt_base)}, {"new", LAUNCHERS(mt)}};
#define VARIANT(name, ns) builds.push_back({#name, LAUNCHERS(ns)});
#include "variants.inc"
#undef VARIANT
  auto pick = [&](const Build& b) { return kind == 32 ? b.l32 : kind == 64 ? b.l64 : b.l128; };
  auto launch_ts = kind == 32 ? mt_ts::launch_vpair32 : kind == 64 ? mt_ts::launch_vpair : mt_ts::launch_vpair128;
  auto bind = kind == 32 ? mt_ts::vpair32_ts_bind : kind == 64 ? mt_ts::vpair_ts_bind : mt_ts::vpair128_ts_bind;

  srand(1234);
  auto rnd = [] { return (float)((double)rand() / RAND_MAX * 2.0 - 1.0); };
  const size_t nx = (size_t)B * L * C, nw = (size_t)C * C * k;
  std::vector<uint16_t> hx(nx), hw1(nw), hw2(nw);
  for (auto& v : hx) v = to_bf16(rnd());
  const float ws = 1.f / std::sqrt((float)C * k);
  for (auto& v : hw1) v = to_bf16(rnd() * ws);
  for (auto& v : hw2) v = to_bf16(rnd() * ws);
  std::vector<float> hb(2 * C);
  for (auto& v : hb) v = rnd() * 0.1f;
  std::vector<int> lens(B);
  for (int b = 0; b < B; ++b) lens[b] = ragged ? (int)(L * (0.6 + 0.4 * (double)rand() / RAND_MAX)) : L;
  if (ragged) lens[0] = L;

  bf16 *x, *w1, *w2, *y, *y2, *zero, *trash;
  float* bias;
  int* dl;
  CK(hipMalloc(&x, nx * 2));
  CK(hipMalloc(&y, nx * 2));
  CK(hipMalloc(&y2, nx * 2));
  CK(hipMalloc(&w1, nw * 2));
  CK(hipMalloc(&w2, nw * 2));
  CK(hipMalloc(&zero, 4096));
  CK(hipMalloc(&trash, 65536));
  CK(hipMalloc(&bias, 2 * C * 4));
  CK(hipMalloc(&dl, B * 4));
  CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w1, hw1.data(), nw * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w2, hw2.data(), nw * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), 2 * C * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, lens.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemset(zero, 0, 4096));
  CK(hipMemset(y, 0, nx * 2));

  VPairArgs a{};
  a.x = x;
  a.B = B;
  a.L = L;
  a.w1 = w1;
  a.b1 = bias;
  a.w2 = w2;
  a.b2 = bias + C;
  a.taps = k;
  a.dil = d;
  a.y = y;
  a.y2 = y2;
  a.div = 3.f;
  a.slope = 0.1f;
  a.zero = zero;
  a.trash = trash;
  a.lens = ragged ? dl : nullptr;
  a.lmul = 1;

  // warm-up, then every build in alternating blocks of `reps` launches (VE_ACCUM reads y: only the first launch sees
  // the initial y; fine for timing)
  for (auto& bd : builds)
    for (int i = 0; i < 2; ++i)
      if (pick(bd)(ef, &a, 0) != 0) {
        fprintf(stderr, "%s launch: %s\n", bd.name.c_str(), last_error());
        return 1;
      }
  CK(hipDeviceSynchronize());
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  std::vector<double> t(builds.size(), 0.0);
  const int rounds = 2 * (int)builds.size();
  // each round starts at another build: the first block of a round runs measurably slower (clock ramp after the
  // host sync), a bias that would otherwise always fall on the base build
  for (int r = 0; r < rounds; ++r)
    for (size_t jj = 0; jj < builds.size(); ++jj) {
      const size_t j = (jj + r) % builds.size();
      CK(hipEventRecord(e0, 0));
      for (int i = 0; i < reps; ++i) pick(builds[j])(ef, &a, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[j] += ms / reps / rounds;
    }
  long frames = 0;
  for (int b = 0; b < B; ++b) frames += ragged ? lens[b] : L;
  const double flops = 2.0 * 2.0 * C * C * k * (double)frames;
  const double bytes = 2.0 * 2.0 * C * (double)frames;
  // bit comparison against the base build: one launch each on zeroed y
  std::vector<uint16_t> ref(nx), out(nx);
  for (size_t j = 0; j < builds.size(); ++j) {
    CK(hipMemset(y, 0, nx * 2));
    pick(builds[j])(ef, &a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(j == 0 ? ref.data() : out.data(), y, nx * 2, hipMemcpyDeviceToHost));
    // frames at and past a row's valid length are don't-care (never read downstream: mt_ragged.h); kernels with
    // different tile widths leave different values there
    size_t nd = 0;
    if (j > 0)
      for (int b = 0; b < B; ++b)
        for (size_t i = (size_t)b * L * C; i < ((size_t)b * L + (ragged ? lens[b] : L)) * C; ++i) nd += ref[i] != out[i];
    printf("pairlab C=%d k=%d d=%d B=%d L=%d ef=%d ragged=%d  %-6s %.4f ms  x%.3f vs base  %6.1f TFLOP/s %5.2f TB/s%s\n",
           C, k, d, B, L, ef, ragged, builds[j].name.c_str(), t[j], t[j] / t[0], flops / t[j] * 1e-9,
           bytes / t[j] * 1e-9, j == 0 ? "" : nd ? "  <-- DIFFERS FROM BASE" : "  bit-identical");
  }

  // batch invariance: the first 8 utterances as a batch of their own (same rows, same lengths) must give the same
  // valid frames as inside the full batch (rows are independent; mt_ragged.h)
  if (B > 8) {
    CK(hipMemset(y, 0, nx * 2));
    pick(builds[1])(ef, &a, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(ref.data(), y, nx * 2, hipMemcpyDeviceToHost));
    CK(hipMemset(y, 0, nx * 2));
    VPairArgs a8 = a;
    a8.B = 8;
    pick(builds[1])(ef, &a8, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(out.data(), y, nx * 2, hipMemcpyDeviceToHost));
    size_t nb = 0, first = (size_t)-1;
    for (int b = 0; b < 8; ++b)
      for (size_t i = (size_t)b * L * C; i < ((size_t)b * L + (ragged ? lens[b] : L)) * C; ++i)
        if (ref[i] != out[i]) {
          if (first == (size_t)-1) first = i;
          ++nb;
        }
    printf("batch invariance (rows 0-7 alone vs in the B = %d batch): %zu valid outputs differ", B, nb);
    if (nb) printf(" (first: row %zu frame %zu channel %zu)", first / ((size_t)L * C), first / C % L, first % C);
    printf("\n");
  }

  // phase stamps (the working tree with -DVPAIR_TS)
  unsigned long long* ts;
  const int G = 256;
  CK(hipMalloc(&ts, (size_t)G * 2 * 12 * 8));
  CK(hipMemset(ts, 0, (size_t)G * 2 * 12 * 8));
  if (bind(ts) != 0) {
    fprintf(stderr, "ts bind failed\n");
    return 1;
  }
  CK(hipMemset(y, 0, nx * 2));
  launch_ts(ef, *reinterpret_cast<const mt_ts::VPairArgs*>(&a), 0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), y, nx * 2, hipMemcpyDeviceToHost));
  CK(hipMemset(y, 0, nx * 2));
  pick(builds[1])(ef, &a, 0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(ref.data(), y, nx * 2, hipMemcpyDeviceToHost));
  size_t nd = 0;
  for (size_t i = 0; i < nx; ++i) nd += ref[i] != out[i];
  if (kind == 32) PH = PHASES32S;
  printf("stamped build vs new: %zu of %zu outputs differ\n", nd, nx);
  std::vector<unsigned long long> h(G * 2 * 12);
  CK(hipMemcpy(h.data(), ts, h.size() * 8, hipMemcpyDeviceToHost));
  for (int half = 0; half < 2; ++half) {
    double sum[12] = {}, tot = 0;
    int n = 0;
    for (int g = 0; g < G; ++g) {
      double tt = 0;
      for (int i = 0; i < 12; ++i) tt += (double)h[(g * 2 + half) * 12 + i];
      if (tt == 0) continue;
      ++n;
      for (int i = 0; i < 12; ++i) sum[i] += (double)h[(g * 2 + half) * 12 + i];
      tot += tt;
    }
    if (!n) continue;
    printf("  wave %d stamps (mean over %d workgroups, cycles per launch, total %.0f):", half * 4, n, tot / n);
    for (int i = 0; i < 12; ++i)
      if (sum[i] > 0) printf(" %s %.1f%%", PH[i], 100.0 * sum[i] / tot);
    printf("\n");
  }
  return 0;
}
