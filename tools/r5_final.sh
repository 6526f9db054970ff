#!/bin/bash
# Round-5 end evidence, in parts (each within one gpurun call). Usage: bash tools/r5_final.sh PART TAG
#   tests:   the whole -m gpu suite + smoke + a bench line (tools/gpu_round.sh)
#   profile: kernel trace + step breakdown + the family's HBM passes at B = 32 and B = 256 (tools/round_profile.sh);
#            the trace / counter directories are removed once summarised (gpurun_out is capped at 64 MiB)
#   pmc:     per-kernel SQ / TCC counters on one B = 32 bench step (tools/pmc.sh + tools/pmc_table.py)
#   bench:   the default bench.py line (with the CPU baseline)
set -o pipefail
PART=$1; TAG=$2
case $PART in
  tests) bash tools/gpu_round.sh "$TAG" ;;
  profile)
    bash tools/round_profile.sh "${TAG}_b32" || { echo "profile b32 failed"; exit 1; }
    head -8 "gpurun_out/${TAG}_b32/step_breakdown.txt"
    bash tools/round_profile.sh "${TAG}_b256" --batch 256 || { echo "profile b256 failed"; exit 1; }
    head -8 "gpurun_out/${TAG}_b256/step_breakdown.txt"
    rm -rf "gpurun_out/${TAG}_b32"/{trace,fetch,write} "gpurun_out/${TAG}_b256"/{trace,fetch,write} ;;
  pmc)
    bash tools/pmc.sh "${TAG}_pmc" "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
    python3 tools/pmc_table.py "gpurun_out/${TAG}_pmc" > "gpurun_out/${TAG}_pmc/pmc_kernels.txt" 2>&1; echo "pmc table rc=$?"
    rm -rf "gpurun_out/${TAG}_pmc"/p[0-9] ;;
  bench) timeout -k 10 900 python -u bench.py > "gpurun_out/${TAG}_bench.log" 2>&1; echo "bench rc=$?"; tail -c 600 "gpurun_out/${TAG}_bench.log" ;;
esac
