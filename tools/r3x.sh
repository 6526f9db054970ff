# round-3 profiles of the current build (ragged vocoder, XCD-major decoder tiles): kernel-trace step breakdown, the
# family's HBM passes, per-kernel PMC; then the mixed-precision training diagnostics and step times
set -o pipefail
mkdir -p gpurun_out/r3x
bash tools/prof_step.sh r03b > gpurun_out/r3x/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3x/prof_step.out; exit 1; }
head -14 gpurun_out/r03b/step_breakdown.txt
bash tools/round_profile.sh r03b || { echo "round_profile failed"; exit 1; }
cat gpurun_out/r03b/pmc_vconv.json | head -c 600; echo
bash tools/pmc.sh r03bpmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03bpmc > gpurun_out/r3x/pmc_kernels.txt 2>&1; echo "table rc=$?"
head -8 gpurun_out/r3x/pmc_kernels.txt
bash tools/r3q.sh
