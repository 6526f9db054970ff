set -o pipefail
bash tools/gpu_tests.sh r3i || exit 1
timeout -k 10 500 python -u bench.py > gpurun_out/r3i/bench.log 2>&1; echo "bench rc=$?"
tail -c 3000 gpurun_out/r3i/bench.log
