# fp32 vocoder ragged on the generic kernel: ragged + model tests, full suite, then the bench
set -o pipefail
mkdir -p gpurun_out/r3cc
timeout -k 10 300 python -u -m pytest tests/test_gpu_ragged.py -x -v --timeout 240 --timeout-method thread > gpurun_out/r3cc/ragged.log 2>&1; rc=$?; echo "ragged rc=$rc"; grep -E "PASS|FAIL|Error" gpurun_out/r3cc/ragged.log | head; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tests.sh r3cc_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3cc/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3cc/bench.log | head -c 400
