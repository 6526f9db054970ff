#!/bin/bash
# One GPU call: parity tests, then (only if they ran cleanly) a profiled bench, a plain bench and the per-kind
# ResBlock launch probe at the north-star batch.
# Usage: bash tools/gpu_check.sh TAG [bench args...]
TAG=$1; shift
mkdir -p gpurun_out/$TAG
timeout -k 10 600 python -m pytest tests -m gpu -q -rf --tb=short -p no:cacheprovider > gpurun_out/$TAG/tests.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 gpurun_out/$TAG/tests.log
if [ $rc -gt 1 ]; then exit $rc; fi
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/$TAG/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/$TAG/prof_bench.log 2>&1 || exit $?
timeout -k 10 600 python3 bench.py --steps 5 --warmup 2 "$@" > gpurun_out/$TAG/bench.log 2>&1 || exit $?
tail -1 gpurun_out/$TAG/bench.log | cut -c1-300
timeout -k 10 120 python3 tools/pair_probe.py 256 756 2 > gpurun_out/$TAG/probe256.log 2>&1 || exit $?
grep launches gpurun_out/$TAG/probe256.log
