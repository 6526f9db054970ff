# final build (prologue split default 1): whole GPU suite + smoke, bench line
set -o pipefail
mkdir -p gpurun_out/r3kk
bash tools/gpu_tests.sh r3kk_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3kk/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3kk/bench.log | head -c 300; echo
