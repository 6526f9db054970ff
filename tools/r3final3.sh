# round-3 final build (loader subset, prefetch and prologue split reverted): suite + smoke, bench, trace, HBM passes, PMC
set -o pipefail
mkdir -p gpurun_out/r3final3
bash tools/gpu_tests.sh r3final3_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3final3/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3final3/bench.log | head -c 300; echo
bash tools/prof_step.sh r03g > gpurun_out/r3final3/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3final3/prof_step.out; exit 1; }
head -8 gpurun_out/r03g/step_breakdown.txt
bash tools/round_profile.sh r03g || { echo "round_profile failed"; exit 1; }
bash tools/pmc.sh r03gpmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03gpmc > gpurun_out/r3final3/pmc_kernels.txt 2>&1; echo "table rc=$?"
