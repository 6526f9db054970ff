# current build: whole GPU suite + smoke, then the bench (default command)
set -o pipefail
mkdir -p gpurun_out/r3z
bash tools/gpu_tests.sh r3z_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3z/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3z/bench.log | head -c 1200
