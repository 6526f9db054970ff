#!/bin/bash
# VE_ACTIN pass interleave (RB_ACTIN_NV builds): ragged vocoder time, interleaved, B = 32
mkdir -p gpurun_out/rbnv
for r in 1 2; do for n in 0 2 3 4; do
  MT_LIB=$PWD/matcha-tts_amd/ab/rbnv$n.so timeout -k 10 200 python -u tools/voc_time.py 32 10 > gpurun_out/rbnv/v$n.log 2>&1 || { tail -3 gpurun_out/rbnv/v$n.log; exit 1; }
  echo "nv=$n $(tail -1 gpurun_out/rbnv/v$n.log)"
done; done
# the plain upsamplers: compile-time K loop (rbnv3 = the default build) vs runtime loop (upnoct)
for r in 1 2; do for n in rbnv3 upnoct; do
  MT_LIB=$PWD/matcha-tts_amd/ab/$n.so timeout -k 10 200 python -u tools/voc_time.py 32 10 > gpurun_out/rbnv/u$n.log 2>&1 || { tail -3 gpurun_out/rbnv/u$n.log; exit 1; }
  echo "$n $(tail -1 gpurun_out/rbnv/u$n.log)"
done; done
# the ring pair kernel's frame-only prefetch (vpfb1 = default) vs the full-slice prefetch (vpfb0), per-launch times
for r in 1 2; do for n in vpfb1 vpfb0; do
  MT_LIB=$PWD/matcha-tts_amd/ab/$n.so timeout -k 10 180 python tools/pair_probe.py 32 728 3 > gpurun_out/rbnv/p$n.log 2>&1 || { tail -3 gpurun_out/rbnv/p$n.log; exit 1; }
  echo "== $n"; grep -E "vpair  " gpurun_out/rbnv/p$n.log | sed 's/\[MT_VPAIR3.*\] //'
done; done
