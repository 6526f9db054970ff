# ragged vocoder: its own tests first, then the whole GPU suite + smoke, then the bench
set -o pipefail
mkdir -p gpurun_out/r3u
timeout -k 10 300 python -u -m pytest tests/test_gpu_ragged.py -x -v --timeout 240 --timeout-method thread -s > gpurun_out/r3u/ragged.log 2>&1
rc=$?; echo "ragged rc=$rc"; grep -E "PASS|FAIL|Error|rel-RMS" gpurun_out/r3u/ragged.log | head -30; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_tests.sh r3u_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3u/bench.log 2>&1; echo bench rc=$?; tail -c 2500 gpurun_out/r3u/bench.log
