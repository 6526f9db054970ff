#!/bin/bash
# mt_ffn variants: bit-identity tests, then the solve A/B at B=32 / B=256 (every level fused)
mkdir -p gpurun_out/ffn2
timeout -k 10 500 python -u -m pytest tests/test_gpu_ffn.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ffn2/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/ffn2/tests.log | tail -8
[ $rc -le 1 ] || exit $rc
timeout -k 10 240 python -u tools/ffn_ab.py 32 728 10 3 > gpurun_out/ffn2/ab32.log 2>&1 || { tail -5 gpurun_out/ffn2/ab32.log; exit 1; }
grep -v Removing gpurun_out/ffn2/ab32.log
timeout -k 10 400 python -u tools/ffn_ab.py 256 756 3 2 > gpurun_out/ffn2/ab256.log 2>&1 || { tail -5 gpurun_out/ffn2/ab256.log; exit 1; }
grep -v Removing gpurun_out/ffn2/ab256.log
exit $rc
