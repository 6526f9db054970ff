#!/bin/bash
# A/B of the 1x1 vconv tile-width rule (MT_K1_TILES) on the CFM solve, then the GPU parity tests.
mkdir -p gpurun_out/k1
for r in 1 2; do for m in 0 1; do
  MT_K1_TILES=$m timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/k1/b32_${m}_$r.log 2>&1 || exit 1
  echo "K1=$m B=32 $(grep '^one' gpurun_out/k1/b32_${m}_$r.log | head -1)"
done; done
for m in 0 1; do
  MT_K1_TILES=$m timeout -k 10 200 python tools/dec_2stream.py 256 756 3 > gpurun_out/k1/b256_$m.log 2>&1 || exit 1
  echo "K1=$m B=256 $(grep '^one' gpurun_out/k1/b256_$m.log | head -1)"
done
timeout -k 10 600 python -m pytest tests -m gpu -q -rf --tb=short -p no:cacheprovider > gpurun_out/k1/tests.log 2>&1; tail -2 gpurun_out/k1/tests.log
