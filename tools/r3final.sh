# round-3 final build: whole GPU suite + smoke, bench, kernel-trace step breakdown, the family's HBM passes, per-kernel PMC
set -o pipefail
mkdir -p gpurun_out/r3final
bash tools/gpu_tests.sh r3final_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3final/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3final/bench.log | head -c 300; echo
bash tools/prof_step.sh r03c > gpurun_out/r3final/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3final/prof_step.out; exit 1; }
head -8 gpurun_out/r03c/step_breakdown.txt
bash tools/round_profile.sh r03c || { echo "round_profile failed"; exit 1; }
bash tools/pmc.sh r03cpmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03cpmc > gpurun_out/r3final/pmc_kernels.txt 2>&1; echo "table rc=$?"
