#!/bin/bash
# vpair ablation timing (wrong-result builds, timing only)
mkdir -p gpurun_out/vpx
for n in ${VPX:-0 1 2 4 8 7 0}; do
  MT_LIB=$PWD/matcha-tts_amd/ab/vpx$n.so timeout -k 10 180 python tools/pair_probe.py 32 728 3 > gpurun_out/vpx/p$n.log 2>&1 || { tail -5 gpurun_out/vpx/p$n.log; exit 1; }
  echo "== vpx$n"; grep -v "Removing" gpurun_out/vpx/p$n.log
done
