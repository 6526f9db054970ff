# mixed-precision training: GEMM op tests, step error vs fp32 oracle and autocast, step time per precision
set -o pipefail
mkdir -p gpurun_out/r3q
timeout -k 10 300 python -u -m pytest tests/test_gpu_train.py -k "gemm" -x -q --timeout 200 --timeout-method thread > gpurun_out/r3q/gemm_tests.log 2>&1
rc=$?; echo "gemm tests rc=$rc"; tail -3 gpurun_out/r3q/gemm_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/mixed_diag.py > gpurun_out/r3q/diag_small.log 2>&1; echo "diag small rc=$?"; cat gpurun_out/r3q/diag_small.log | tail -8
timeout -k 10 400 python -u tools/mixed_diag.py big > gpurun_out/r3q/diag_big.log 2>&1; echo "diag big rc=$?"; tail -8 gpurun_out/r3q/diag_big.log
for p in 32 16-mixed bf16-mixed; do
  timeout -k 10 200 python -u tools/train_bench.py --precision $p --steps 10 --warmup 3 >> gpurun_out/r3q/train_bench.log 2>&1 || { echo "bench $p failed"; tail -5 gpurun_out/r3q/train_bench.log; exit 1; }
done
cat gpurun_out/r3q/train_bench.log | grep '^{'
