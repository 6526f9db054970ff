#!/bin/bash
# GPU box: pairlab timing + phase stamps at the bench's B = 32 shapes (ragged): stage 2 (C = 128, k = 3),
# stage 3 (C = 64) and stage 4 (C = 32), k = 3 / 7 / 11 at d = 3. Usage: bash tools/pairlab/run.sh TAG [CASES]
# CASES: "C:k:d:ef ..." (default below); each run has its own time limit.
set -o pipefail
TAG=$1; CASES=${2:-"128:3:3:0 64:3:3:0 64:7:3:0 64:11:3:0 64:11:5:22 32:3:3:0 32:7:3:0 32:11:3:0 32:11:5:22"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CASES; do
  IFS=: read -r C k d ef <<< "$c"
  L=$((728 * 8192 / C))  # samples per utterance at the stage: T_mel * (8192 / C)
  timeout -k 10 120 tools/pairlab/pairlab "$C" "$k" "$d" 32 "$L" "$ef" 20 1 > "$OUT/p_${C}_${k}_${d}_${ef}.txt" 2>&1 \
    || { echo "FAILED $c"; cat "$OUT/p_${C}_${k}_${d}_${ef}.txt"; exit 1; }
  cat "$OUT/p_${C}_${k}_${d}_${ef}.txt"
done
