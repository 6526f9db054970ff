#!/bin/bash
# the ring pair kernel's frame-only prefetch (vpfb1 = default) vs the full-slice prefetch (vpfb0), per-launch times
mkdir -p gpurun_out/vpfb
for r in 1 2; do for n in vpfb1 vpfb0; do
  MT_LIB=$PWD/matcha-tts_amd/ab/$n.so timeout -k 10 180 python tools/pair_probe.py 32 728 3 > gpurun_out/vpfb/p$n.log 2>&1 || { tail -3 gpurun_out/vpfb/p$n.log; exit 1; }
  echo "== $n"; grep -E "vpair  " gpurun_out/vpfb/p$n.log | sed 's/\[MT_VPAIR3.*\] //'
done; done
for n in vpfb1 vpfb0; do MT_LIB=$PWD/matcha-tts_amd/ab/$n.so timeout -k 10 120 python tools/gen_hash.py 2>&1 | grep gen_hash | sed "s/^/$n /"; done
