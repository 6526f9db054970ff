set -o pipefail
bash tools/gpu_tests.sh r3f || exit 1
timeout -k 10 400 python -u bench.py --steps 20 --warmup 5 > gpurun_out/r3f/bench.log 2>&1; echo "bench rc=$?"
tail -c 1500 gpurun_out/r3f/bench.log
