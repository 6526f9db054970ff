# Round-3 profiles: configs[4]-size training tests, kernel-trace step breakdown, family HBM passes, per-kernel PMC.
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -k configs4 -x -v --timeout 500 --timeout-method thread -s > gpurun_out/r03/train_tests.log 2>&1
rc=$?; echo "train tests rc=$rc"; tail -4 gpurun_out/r03/train_tests.log; [ $rc -eq 0 ] || exit $rc
bash tools/prof_step.sh r03 > gpurun_out/r03/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r03/prof_step.out; exit 1; }
bash tools/round_profile.sh r03 || { echo "round_profile failed"; exit 1; }
bash tools/pmc.sh r03pmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03pmc > gpurun_out/r03/pmc_kernels.txt 2>&1; echo "table rc=$?"
head -30 gpurun_out/r03/pmc_kernels.txt
