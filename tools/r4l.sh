#!/bin/bash
# the decoder keeps its graph in the bench's probed step: the probe / graph tests, then the bench line
mkdir -p gpurun_out/r4l
timeout -k 10 400 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_ffn.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r4l/tests.log 2>&1
rc=$?; tail -2 gpurun_out/r4l/tests.log
[ $rc -le 1 ] || exit $rc
bash tools/bench_quick.sh r4l
exit $rc
