// Phase stamps for the pair kernels, DIAGNOSTIC builds only (tools/pairlab: -DVPAIR_TS). In the library the macros
// expand to nothing. With VPAIR_TS, waves 0 and 4 of every workgroup add the s_memtime cycles of each named phase
// into scalar sums and store them once at the end to g_vp_ts[(blockIdx.x * 2 + wave / 4) * VP_TS_N + phase], a
// buffer only the lab reads (cdna_hip_programming.md §7, In-kernel stamps: each stamp waits lgkmcnt(0), so read the
// phase SHARES of such a build, not its run time).
#pragma once

#if defined(VPAIR_TS)
#include "mt_common.h"
namespace mt {
constexpr int VP_TS_N = 12;
static __device__ unsigned long long* g_vp_ts;  // one per translation unit (bound by VP_TS_BINDER's function)
__device__ __forceinline__ unsigned long long vp_stamp() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
}  // namespace mt
#define VP_TS_DECL                               \
  unsigned long long vp_ts_sum[mt::VP_TS_N] = {}; \
  unsigned long long vp_ts_last = mt::vp_stamp();
#define VP_TS(i)                                   \
  do {                                             \
    const unsigned long long t_ = mt::vp_stamp(); \
    vp_ts_sum[i] += t_ - vp_ts_last;               \
    vp_ts_last = t_;                               \
  } while (0)
// a host function `name(buffer)` pointing this translation unit's stamp buffer at `buffer` (device memory)
#define VP_TS_BINDER(name)                                                      \
  int name(unsigned long long* p) {                                             \
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(mt::g_vp_ts), &p, sizeof(p));       \
  }
#define VP_TS_END(wave, lane)                                                                          \
  do {                                                                                                 \
    if (((wave) & 3) == 0 && (lane) == 0 && mt::g_vp_ts)                                               \
      _Pragma("unroll") for (int i_ = 0; i_ < mt::VP_TS_N; ++i_)                                                         \
        mt::g_vp_ts[((size_t)blockIdx.x * 2 + ((wave) >> 2)) * mt::VP_TS_N + i_] = vp_ts_sum[i_];       \
  } while (0)
#else
#define VP_TS_DECL
#define VP_TS(i) \
  do {           \
  } while (0)
#define VP_TS_END(wave, lane) \
  do {                        \
  } while (0)
#define VP_TS_BINDER(name)
#endif
