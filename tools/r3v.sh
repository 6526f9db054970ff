# fp32 encoder tile model: encoder parity + variant coverage, encoder A/B vs the round-3 start build; then the round
# profiles of the ragged-vocoder build (kernel trace step breakdown, family HBM passes, per-kernel PMC)
set -o pipefail
mkdir -p gpurun_out/r3v
: timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_shapes.py -x -v --timeout 500 --timeout-method thread -s > gpurun_out/r3v/shapes.log 2>&1
rc=0; echo "shapes skipped (passed in the previous call)"; grep -E "passed|failed|encoder" gpurun_out/r3v/shapes.log | tail -6; [ $rc -eq 0 ] || exit $rc
for L in matcha-tts_amd/libmatcha_hip_base.so matcha-tts_amd/libmatcha_hip.so matcha-tts_amd/libmatcha_hip_base.so matcha-tts_amd/libmatcha_hip.so; do
  MT_LIB=$L timeout -k 10 120 python tools/enc_bench.py 32 30 > gpurun_out/r3v/enc.log 2>&1 || exit 1
  echo "$L $(tail -1 gpurun_out/r3v/enc.log)"
done
bash tools/prof_step.sh r03b > gpurun_out/r3v/prof_step.out 2>&1 || { echo "prof_step failed"; tail gpurun_out/r3v/prof_step.out; exit 1; }
head -12 gpurun_out/r03b/step_breakdown.txt
bash tools/round_profile.sh r03b || { echo "round_profile failed"; exit 1; }
bash tools/pmc.sh r03bpmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/r03bpmc > gpurun_out/r3v/pmc_kernels.txt 2>&1; echo "table rc=$?"
head -12 gpurun_out/r3v/pmc_kernels.txt
