# block-parallel durations scan + split alignment writes: model / bench-shape tests, then the step breakdown
set -o pipefail
mkdir -p gpurun_out/r3bb
timeout -k 10 500 python -u -m pytest tests/test_gpu_model.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity_bf16.py tests/test_gpu_batch1.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3bb/t.log 2>&1; rc=$?; echo "tests rc=$rc"; tail -3 gpurun_out/r3bb/t.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_step.sh r03c > gpurun_out/r3bb/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3bb/prof_step.out; exit 1; }
head -8 gpurun_out/r03c/step_breakdown.txt; grep -E "durations|alignment" gpurun_out/r03c/kernel_stats.csv | cut -c1-160
