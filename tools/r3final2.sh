# round-3 final build (4 loader waves): whole GPU suite + smoke, bench, kernel-trace step breakdown, HBM passes, PMC
set -o pipefail
mkdir -p gpurun_out/r3final2
bash tools/gpu_tests.sh r3final2_tests || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r3final2/bench.log 2>&1; echo bench rc=$?; grep '^{' gpurun_out/r3final2/bench.log | head -c 300; echo
bash tools/prof_step.sh r03d > gpurun_out/r3final2/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3final2/prof_step.out; exit 1; }
head -8 gpurun_out/r03d/step_breakdown.txt
bash tools/round_profile.sh r03d || { echo "round_profile failed"; exit 1; }
bash tools/pmc.sh r03dpmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03dpmc > gpurun_out/r3final2/pmc_kernels.txt 2>&1; echo "table rc=$?"
