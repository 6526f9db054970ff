#!/bin/bash
# GPU box: rocprofv3 kernel stats of the text encoder + duration predictor alone (tools/enc_bench.py) at B = 256.
# Usage: bash tools/r5_enc_prof.sh TAG
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/encprof -o enc -- \
  python3 "$GRAFT_REPO_ROOT/tools/enc_bench.py" 256 10 > "$GRAFT_REPO_ROOT/$OUT/enc.log" 2>&1 || { tail -20 "$GRAFT_REPO_ROOT/$OUT/enc.log"; exit 1; }
cp "$(find /tmp/encprof -name '*kernel_stats.csv' | head -1)" "$GRAFT_REPO_ROOT/$OUT/enc_kernel_stats.csv"
tail -3 "$GRAFT_REPO_ROOT/$OUT/enc.log"
