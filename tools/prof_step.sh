#!/bin/bash
# rocprofv3 kernel trace + stats of a short default bench run, then the per-step component breakdown.
# Usage: bash tools/prof_step.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --quick --steps 4 --warmup 2 "$@" > $OUT/bench.log 2>&1 || { echo "prof rc=$?"; tail $OUT/bench.log; exit 1; }
python3 tools/prof_summary.py $(find $OUT/prof -name '*kernel_trace.csv' | head -1) 40 > $OUT/step_breakdown.txt 2>&1
cp $(find $OUT/prof -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
head -60 $OUT/step_breakdown.txt
