#!/bin/bash
# the fused FeedForward's frame threshold at the bench batch: every level vs level 0 only vs none (B=32, T=728)
mkdir -p gpurun_out/ffnmin
for m in 0 16384 1000000 0 16384 1000000; do
  FFN_MIN=$m timeout -k 10 200 python -u tools/ffn_ab.py 32 728 10 2 > gpurun_out/ffnmin/m$m.log 2>&1 || { tail -3 gpurun_out/ffnmin/m$m.log; exit 1; }
  echo "min $m: $(grep -E '^fused\+pfb|^two-launch' gpurun_out/ffnmin/m$m.log | tr '\n' ' ')"
done
