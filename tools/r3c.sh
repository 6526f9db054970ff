set -o pipefail
mkdir -p gpurun_out/r3c
timeout -k 10 200 python -u tools/enc_bench.py 32 20 fp32 > gpurun_out/r3c/enc.log 2>&1 && timeout -k 10 200 python -u tools/enc_bench.py 256 5 fp32 >> gpurun_out/r3c/enc.log 2>&1 && timeout -k 10 200 python -u tools/enc_bench.py 32 20 bf16 >> gpurun_out/r3c/enc.log 2>&1
cat gpurun_out/r3c/enc.log | grep encoder
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r3c/prof -o run --output-format csv -- python3 tools/enc_bench.py 32 5 fp32 > gpurun_out/r3c/prof.log 2>&1
head -25 gpurun_out/r3c/prof/run_kernel_stats.csv | cut -c1-200
