#!/bin/bash
# mt_ffn on the GPU: its bit-identity tests (every case, no -x), then the in-process solve A/B at B=32 and B=256
# (every level fused, FFN_MIN=0), then the bf16 parity tests that run through it by default.
mkdir -p gpurun_out/ffn
timeout -k 10 500 python -u -m pytest tests/test_gpu_ffn.py -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ffn/tests.log 2>&1
rc=$?; grep -E "PASS|FAIL|Error|passed|failed" gpurun_out/ffn/tests.log | tail -12
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -u tools/ffn_ab.py 32 728 10 3 > gpurun_out/ffn/ab32.log 2>&1 || { tail -5 gpurun_out/ffn/ab32.log; exit 1; }
grep -v Removing gpurun_out/ffn/ab32.log
timeout -k 10 300 python -u tools/ffn_ab.py 256 756 3 2 > gpurun_out/ffn/ab256.log 2>&1 || { tail -5 gpurun_out/ffn/ab256.log; exit 1; }
grep -v Removing gpurun_out/ffn/ab256.log
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity_bf16.py tests/test_gpu_bench_shapes.py tests/test_gpu_model.py -q --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/ffn/parity.log 2>&1
echo "parity rc=$?"; tail -3 gpurun_out/ffn/parity.log
exit $rc
