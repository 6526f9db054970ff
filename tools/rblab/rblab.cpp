// rblab: standalone timing, bit-identity and phase-stamp harness for the stage 1-2 ResBlock conv kernel (mt_rbconv,
// no torch). tools/rblab/build.sh compiles mt_rbconv.hip into namespaces: mt_base (a git revision, the reference),
// mt (the working tree), mt_ts (-DVPAIR_TS phase stamps, mt_ts.h) and one mt_<v> per experiment variant. Inputs are
// synthetic (random bf16 rows and weights). Every build is timed against mt_base in alternating blocks of launches
// and compared with it bit for bit (y and, with VE_DUAL, y2; frames < each utterance's length).
// Usage: rblab C K D B L [EF] [REPS] [RAGGED]   (C 128 | 256, K 3 | 7 | 11, EF the VE_* epilogue flags, e.g.
// 16392 = VE_ACT | VE_ACTIN (conv1), 1 = VE_RESID (conv2), 23 = RESID | ACCUM | DIV | DUAL)
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "mt_vconv.h"

namespace mt {
const char* last_error();
}  // namespace mt
namespace mt_ts {
struct VConvArgs;
int launch_rbconv(int ef, const VConvArgs& a, int G, hipStream_t st);
int rbconv_ts_bind(unsigned long long* p);
}  // namespace mt_ts
namespace mt_base {
struct VConvArgs;
int launch_rbconv(int ef, const VConvArgs& a, int G, hipStream_t st);
}  // namespace mt_base

using Launch = int (*)(int, const void*, int, hipStream_t);
struct Build {
  std::string name;
  Launch l;
};
#define LAUNCHER(ns) \
  reinterpret_cast<Launch>(static_cast<int (*)(int, const ns::VConvArgs&, int, hipStream_t)>(ns::launch_rbconv))
#include "variants_decl.inc"

#define CK(x)                                                                           \
  do {                                                                                  \
    hipError_t e_ = (x);                                                                \
    if (e_ != hipSuccess) {                                                             \
      fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      exit(1);                                                                          \
    }                                                                                   \
  } while (0)

static uint16_t to_bf16(float f) {
  uint32_t u;
  memcpy(&u, &f, 4);
  return (uint16_t)((u + 0x7fff + ((u >> 16) & 1)) >> 16);
}

static const char* PHASES[12] = {"wait", "barrier", "dma-issue", "mfma", "act-pass", "epilogue",
                                 "tile-head", "prologue", "-", "-", "-", "drain"};

int main(int argc, char** argv) {
  if (argc < 6) {
    fprintf(stderr, "usage: rblab C K D B L [EF] [REPS] [RAGGED]\n");
    return 2;
  }
  const int C = atoi(argv[1]), k = atoi(argv[2]), d = atoi(argv[3]), B = atoi(argv[4]), L = atoi(argv[5]);
  const int ef = argc > 6 ? atoi(argv[6]) : mt::VE_ACT, reps = argc > 7 ? atoi(argv[7]) : 20;
  const int ragged = argc > 8 ? atoi(argv[8]) : 1;
  std::vector<Build> builds = {{"base", LAUNCHER(mt_base)}, {"new", LAUNCHER(mt)}};
#define VARIANT(name, ns) builds.push_back({#name, LAUNCHER(ns)});
#include "variants.inc"
#undef VARIANT

  srand(4321);
  auto rnd = [] { return (float)((double)rand() / RAND_MAX * 2.0 - 1.0); };
  const size_t nx = (size_t)B * L * C, nw = (size_t)C * C * k;
  std::vector<uint16_t> hx(nx), hr(nx), hw(nw);
  for (auto& v : hx) v = to_bf16(rnd());
  for (auto& v : hr) v = to_bf16(rnd());
  const float ws = 1.f / std::sqrt((float)C * k);
  for (auto& v : hw) v = to_bf16(rnd() * ws);
  std::vector<float> hb(C);
  for (auto& v : hb) v = rnd() * 0.1f;
  std::vector<int> lens(B);
  for (int b = 0; b < B; ++b) lens[b] = ragged ? (int)(L * (0.6 + 0.4 * (double)rand() / RAND_MAX)) : L;
  if (ragged) lens[0] = L;

  mt::bf16 *x, *w, *y, *y2, *resid, *zero, *trash;
  float* bias;
  int* dl;
  CK(hipMalloc(&x, nx * 2));
  CK(hipMalloc(&resid, nx * 2));
  CK(hipMalloc(&y, nx * 2));
  CK(hipMalloc(&y2, nx * 2));
  CK(hipMalloc(&w, nw * 2));
  CK(hipMalloc(&zero, 4096));
  CK(hipMalloc(&trash, 65536));
  CK(hipMalloc(&bias, C * 4));
  CK(hipMalloc(&dl, B * 4));
  CK(hipMemcpy(x, hx.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(resid, hr.data(), nx * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(w, hw.data(), nw * 2, hipMemcpyHostToDevice));
  CK(hipMemcpy(bias, hb.data(), C * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(dl, lens.data(), B * 4, hipMemcpyHostToDevice));
  CK(hipMemset(zero, 0, 4096));

  mt::VConvArgs a{};
  a.x = x;
  a.B = B;
  a.L = L;
  a.cin = a.c0 = C;
  a.w = w;
  a.bias = bias;
  a.M = a.Mpad = C;
  a.taps = k;
  a.dil = d;
  a.pad = d * (k - 1) / 2;
  a.y = y;
  a.y2 = y2;
  a.resid = resid;
  a.div = 3.f;
  a.slope = 0.1f;
  a.zero = zero;
  a.trash = trash;
  a.Lout = L;
  a.ldy = C;
  a.ylim = L * C;
  a.ystride = (long long)L * C;
  a.lens = ragged ? dl : nullptr;
  a.lmul = 1;
  const long ntiles = (long)B * ((L + 255) / 256) * (C / 128);
  const int G = (int)std::min<long>(ntiles, 256);
  a.xcd_tiles = ntiles <= 3L * G;

  auto reset = [&] {  // VE_ACCUM reads y: every compared launch starts from the same y
    CK(hipMemcpy(y, hr.data(), nx * 2, hipMemcpyHostToDevice));
    CK(hipMemset(y2, 0, nx * 2));
  };
  reset();
  for (auto& bd : builds)
    for (int i = 0; i < 2; ++i)
      if (bd.l(ef, &a, G, 0) != 0) {
        fprintf(stderr, "%s launch: %s\n", bd.name.c_str(), mt::last_error());
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
      for (int i = 0; i < reps; ++i) builds[j].l(ef, &a, G, 0);
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      t[j] += ms / reps / rounds;
    }
  long frames = 0;
  for (int b = 0; b < B; ++b) frames += lens[b];
  const double flops = 2.0 * C * C * k * (double)frames;
  const bool dual = (ef & mt::VE_DUAL) != 0;
  std::vector<uint16_t> ref(nx), out(nx), ref2(nx), out2(nx);
  auto run_get = [&](Launch l, std::vector<uint16_t>& o, std::vector<uint16_t>& o2) {
    reset();
    l(ef, &a, G, 0);
    CK(hipDeviceSynchronize());
    CK(hipMemcpy(o.data(), y, nx * 2, hipMemcpyDeviceToHost));
    CK(hipMemcpy(o2.data(), y2, nx * 2, hipMemcpyDeviceToHost));
  };
  auto ndiff = [&](const std::vector<uint16_t>& p, const std::vector<uint16_t>& q) {
    size_t nd = 0;
    for (int b = 0; b < B; ++b)
      for (size_t i = (size_t)b * L * C; i < ((size_t)b * L + lens[b]) * C; ++i) nd += p[i] != q[i];
    return nd;
  };
  for (size_t j = 0; j < builds.size(); ++j) {
    run_get(builds[j].l, j == 0 ? ref : out, j == 0 ? ref2 : out2);
    const size_t nd = j ? ndiff(ref, out) + (dual ? ndiff(ref2, out2) : 0) : 0;
    printf("rblab C=%d k=%d d=%d B=%d L=%d ef=%d ragged=%d  %-6s %.4f ms  x%.3f vs base  %6.1f TFLOP/s%s\n", C, k, d,
           B, L, ef, ragged, builds[j].name.c_str(), t[j], t[j] / t[0], flops / t[j] * 1e-9,
           j == 0 ? "" : nd ? "  <-- DIFFERS FROM BASE" : "  bit-identical");
  }

  // phase stamps (the working tree with -DVPAIR_TS)
  unsigned long long* ts;
  CK(hipMalloc(&ts, (size_t)G * 2 * 12 * 8));
  CK(hipMemset(ts, 0, (size_t)G * 2 * 12 * 8));
  if (mt_ts::rbconv_ts_bind(ts) != 0) {
    fprintf(stderr, "ts bind failed\n");
    return 1;
  }
  reset();
  mt_ts::launch_rbconv(ef, *reinterpret_cast<const mt_ts::VConvArgs*>(&a), G, 0);
  CK(hipDeviceSynchronize());
  CK(hipMemcpy(out.data(), y, nx * 2, hipMemcpyDeviceToHost));
  run_get(builds[1].l, ref, ref2);
  printf("stamped build vs new: %zu outputs differ\n", ndiff(ref, out));
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
      if (sum[i] > 0) printf(" %s %.1f%%", PHASES[i], 100.0 * sum[i] / tot);
    printf("\n");
  }
  return 0;
}
