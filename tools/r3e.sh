set -o pipefail
mkdir -p gpurun_out/r3e
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_encoder.py tests/test_gpu_train.py tests/test_gpu_train_dist.py tests/test_gpu_parity_bf16.py::test_bf16_model_index_path_bit_exact_unforced_durations > gpurun_out/r3e/tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r3e/tests.log
timeout -k 10 200 python -u tools/enc_bench.py 32 20 fp32 > gpurun_out/r3e/enc.log 2>&1 && timeout -k 10 200 python -u tools/enc_bench.py 256 5 fp32 >> gpurun_out/r3e/enc.log 2>&1
grep encoder gpurun_out/r3e/enc.log
