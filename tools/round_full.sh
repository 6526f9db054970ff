#!/bin/bash
# Round-end style GPU call: the whole -m gpu suite + smoke + the default bench line, then the round profiles at the
# headline (B=32) and north-star (B=256) workloads: kernel trace + step breakdown + the family's HBM passes
# (tools/round_profile.sh), and the per-kernel SQ counters at B=32 (tools/pmc.sh). Stops at the first failure.
# Usage: bash tools/round_full.sh TAG
TAG=${1:-round}
bash tools/gpu_round.sh $TAG || exit 1
bash tools/round_profile.sh ${TAG}_b32 || { echo "profile b32 failed"; exit 1; }
head -8 gpurun_out/${TAG}_b32/step_breakdown.txt
bash tools/round_profile.sh ${TAG}_b256 --batch 256 || { echo "profile b256 failed"; exit 1; }
head -8 gpurun_out/${TAG}_b256/step_breakdown.txt
bash tools/pmc.sh ${TAG}_pmc "." -- python3 bench.py --quick --steps 1 --warmup 1 || exit 1
python3 tools/pmc_table.py gpurun_out/${TAG}_pmc > gpurun_out/${TAG}_pmc/pmc_kernels.txt 2>&1; echo "pmc table rc=$?"
echo done
