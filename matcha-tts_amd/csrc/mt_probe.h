// Launch probe: HIP events recorded on the launching stream around every launch of one kernel
// site, so a caller (bench.py) can time that kernel inside its own timed region and read the
// algorithmic work the launches did. Off unless mt_probe_start() armed it; host-only state.
#pragma once
#include "mt_common.h"

namespace mt {

enum ProbeSite {
  PROBE_NONE = 0,
  PROBE_RBFUSE_C64 = 1,  // fused HiFi-GAN ResBlock stage, 64 channels (stage 3 of v1)
  PROBE_RBFUSE_C32 = 2,  // fused HiFi-GAN ResBlock stage, 32 channels (stage 4 of v1)
  PROBE_VCONV = 3,       // LDS-DMA persistent conv, HiFi-GAN ResBlock convs (k >= 3)
  PROBE_VCONV_DEC = 4,   // LDS-DMA persistent conv, CFM decoder k = 3 convs (ResnetBlock, up/down, final)
};

bool probe_armed(int site);
bool probe_any_armed();  // some site armed (its launches need per-launch host bookkeeping)
void probe_begin(int site, hipStream_t st);
// tag: the launching kernel's kind (PROBE_TAG_*), reported per launch by probe_detail
enum ProbeTag { PROBE_TAG_VCONV = 0, PROBE_TAG_VPAIR = 1, PROBE_TAG_VPAIR32 = 2, PROBE_TAG_RBFUSE = 3, PROBE_TAG_VPAIR128 = 4, PROBE_TAG_RBCONV = 5 };
void probe_end(int site, hipStream_t st, double flops, double bytes, int tag = PROBE_TAG_VCONV);
// per-launch duration (ms), algorithmic FLOPs / bytes and tag of the recorded launches (synchronizes their
// events; call before probe_stop) -> launches written (<= cap)
int probe_detail(int cap, double* ms, double* flops, double* bytes, int* tags);
int probe_start(int site, int max_launches);
int probe_pause(bool paused);
// roof_ms: sum over launches of max(flops / peak_flops, bytes / peak_bw) in ms (the roofline time)
int probe_stop(int* launches, double* total_ms, double* flops, double* bytes, double peak_flops, double peak_bw,
               double* roof_ms);

// Launch log (test coverage only): while armed, every launch_vconv appends the variant it picked and
// the grid it used, so parity tests can show which instantiations ran and whether workgroups walked
// more than one tile. Host-only state, off unless vclog_start() armed it.
constexpr int VCLOG_FIELDS = 11;  // ef, BM, BN, K1, ntiles, grid, taps, M, cin, B, L
void vclog_record(const int (&rec)[VCLOG_FIELDS]);
int vclog_start(int cap);
int vclog_stop(int* out, int cap);  // -> records written (cap records of VCLOG_FIELDS ints)
bool vclog_armed();

}  // namespace mt
