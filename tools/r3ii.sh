# final build (next-launch prefetch on multi-round grids): whole GPU suite + smoke, bench line
set -o pipefail
mkdir -p gpurun_out/r3ii
bash tools/gpu_tests.sh r3ii_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3ii/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3ii/bench.log | head -c 300; echo
