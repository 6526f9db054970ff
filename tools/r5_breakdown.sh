#!/bin/bash
# GPU box: kernel-trace step breakdown (tools/prof_summary.py) of the bench's step at B = 32 and at the north-star
# B = 256, trace directories removed afterwards (only the summaries come back). Usage: bash tools/r5_breakdown.sh TAG
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
export TMPDIR=/tmp
for b in 32 256; do
  sfx=$([ $b = 32 ] && echo "" || echo "_b256")
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d /tmp/bd$b -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-north-star --quick --batch $b > "$OUT/trace$sfx.log" 2>&1 \
    || { tail -20 "$OUT/trace$sfx.log"; exit 1; }
  python3 tools/prof_summary.py "$(find /tmp/bd$b -name '*kernel_trace.csv' | head -1)" 40 > "$OUT/step_breakdown$sfx.txt" 2>&1
  cp "$(find /tmp/bd$b -name '*kernel_stats.csv' | head -1)" "$OUT/kernel_stats$sfx.csv"
  rm -rf /tmp/bd$b
  head -7 "$OUT/step_breakdown$sfx.txt"
done
