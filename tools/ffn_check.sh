#!/bin/bash
# mt_ffn on the GPU: its bit-identity tests, then the in-process solve A/B at B=32 and B=256.
mkdir -p gpurun_out/ffn
timeout -k 10 400 python -u -m pytest tests/test_gpu_ffn.py -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ffn/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|error|passed|failed" gpurun_out/ffn/tests.log | tail -12
timeout -k 10 200 python -u tools/ffn_ab.py 32 728 10 3 > gpurun_out/ffn/ab32.log 2>&1 || { tail -5 gpurun_out/ffn/ab32.log; exit 1; }
cat gpurun_out/ffn/ab32.log | grep -v Removing
timeout -k 10 300 python -u tools/ffn_ab.py 256 756 3 2 > gpurun_out/ffn/ab256.log 2>&1 || { tail -5 gpurun_out/ffn/ab256.log; exit 1; }
cat gpurun_out/ffn/ab256.log | grep -v Removing
exit $rc
