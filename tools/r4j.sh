#!/bin/bash
# plain upsamplers on the compile-time K loop: the CT bit-identity tests, then the ragged vocoder
mkdir -p gpurun_out/r4j
timeout -k 10 400 python -u -m pytest tests/test_gpu_vconv_ct.py tests/test_gpu_model.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4j/tests.log 2>&1
rc=$?; tail -3 gpurun_out/r4j/tests.log
[ $rc -le 1 ] || exit $rc
for r in 1 2; do
  timeout -k 10 200 python -u tools/voc_time.py 32 10 > gpurun_out/r4j/v32.log 2>&1 || { tail -3 gpurun_out/r4j/v32.log; exit 1; }
  echo "B=32 $(tail -1 gpurun_out/r4j/v32.log)"
done
timeout -k 10 300 python -u tools/voc_time.py 256 3 > gpurun_out/r4j/v256.log 2>&1 || { tail -3 gpurun_out/r4j/v256.log; exit 1; }
echo "B=256 $(tail -1 gpurun_out/r4j/v256.log)"
exit $rc
