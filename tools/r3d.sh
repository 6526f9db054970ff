set -o pipefail
mkdir -p gpurun_out/r3d
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread -s tests/test_gpu_encoder.py tests/test_gpu_parity_bf16.py::test_bf16_model_index_path_bit_exact_unforced_durations > gpurun_out/r3d/tests.log 2>&1; echo "tests rc=$?"; tail -3 gpurun_out/r3d/tests.log
timeout -k 10 200 python -u tools/enc_bench.py 32 20 fp32 > gpurun_out/r3d/enc.log 2>&1 && timeout -k 10 200 python -u tools/enc_bench.py 256 5 fp32 >> gpurun_out/r3d/enc.log 2>&1
grep encoder gpurun_out/r3d/enc.log
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3d/prof -o run --output-format csv -- python3 tools/enc_bench.py 32 5 fp32 > gpurun_out/r3d/prof.log 2>&1
head -16 gpurun_out/r3d/prof/run_kernel_stats.csv | cut -c1-150
