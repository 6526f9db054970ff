#!/bin/bash
# VE_ACTIN: the rbconv bit-identity tests, then the ragged vocoder with the in-LDS activation on / off (interleaved
# processes, B = 32 and B = 256)
mkdir -p gpurun_out/actin
timeout -k 10 500 python -u -m pytest tests/test_gpu_rbconv.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/actin/tests.log 2>&1
rc=$?; tail -4 gpurun_out/actin/tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do for a in 1 0; do
  MT_ACTIN=$a timeout -k 10 200 python -u tools/voc_time.py 32 10 > gpurun_out/actin/v32_$a.log 2>&1 || { tail -3 gpurun_out/actin/v32_$a.log; exit 1; }
  echo "B=32 actin=$a $(tail -1 gpurun_out/actin/v32_$a.log)"
done; done
for a in 1 0; do
  MT_ACTIN=$a timeout -k 10 300 python -u tools/voc_time.py 256 3 > gpurun_out/actin/v256_$a.log 2>&1 || { tail -3 gpurun_out/actin/v256_$a.log; exit 1; }
  echo "B=256 actin=$a $(tail -1 gpurun_out/actin/v256_$a.log)"
done
exit $rc
