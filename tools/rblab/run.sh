#!/bin/bash
# GPU box: rblab timing + phase stamps at the bench's B = 32 shapes (ragged). Usage: bash tools/rblab/run.sh TAG [CASES]
# CASES: "C:k:d:ef ..." (default: the stage 1-2 conv1 / conv2 shapes of the vocoder); each run has its own time limit.
set -o pipefail
TAG=$1; CASES=${2:-"128:11:5:16392 128:7:3:16392 128:11:1:1 128:11:1:23 256:11:5:16392 256:7:1:1"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
for c in $CASES; do
  IFS=: read -r C k d ef <<< "$c"
  [ "$C" = 256 ] && L=$((728 * 8)) || L=$((728 * 64))
  timeout -k 10 120 tools/rblab/rblab "$C" "$k" "$d" 32 "$L" "$ef" 20 1 > "$OUT/r_${C}_${k}_${d}_${ef}.txt" 2>&1 \
    || { echo "FAILED $c"; cat "$OUT/r_${C}_${k}_${d}_${ef}.txt"; exit 1; }
  cat "$OUT/r_${C}_${k}_${d}_${ef}.txt"
done
