#!/bin/bash
# GPU box: rocprofv3 kernel stats of the 16-mixed training step (tools/train_bench.py, 3 timed steps), the
# hipBLASLt path and (MT_HBLT=0) the in-tree 16-bit GEMM. Usage: bash tools/r5_train_prof.sh TAG
set -o pipefail
TAG=$1; OUT=$GRAFT_REPO_ROOT/gpurun_out/$TAG; mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
for m in ${MODES:-1 0}; do
  MT_HBLT=$m timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/trprof$m -o tr -- \
    python3 "$GRAFT_REPO_ROOT/tools/train_bench.py" --precision 16-mixed --steps 3 --warmup 2 > "$OUT/train$m.log" 2>&1 \
    || { tail -20 "$OUT/train$m.log"; exit 1; }
  cp "$(find /tmp/trprof$m -name '*kernel_stats.csv' | head -1)" "$OUT/train${m}_kernel_stats.csv"
  grep cfm_training_step "$OUT/train$m.log" | tail -1
done
