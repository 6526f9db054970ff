set -o pipefail
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity_bf16.py tests/test_gpu_batch1.py -s > gpurun_out/r3a/tests.log 2>&1; echo "tests rc=$?"
timeout -k 10 300 python -u tools/bf16_diag.py 32 728 > gpurun_out/r3a/diag.log 2>&1; echo "diag rc=$?"
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3a/bench.log 2>&1; echo "bench rc=$?"
