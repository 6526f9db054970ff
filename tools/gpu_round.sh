#!/bin/bash
# One GPU call: the whole -m gpu suite (no -x: every failure is listed), smoke, then a short bench.
# Usage: bash tools/gpu_round.sh TAG [bench args...]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -v -rf --timeout 300 --timeout-method thread -s -p no:cacheprovider > $OUT/tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "^(FAILED|ERROR)|passed|failed" $OUT/tests.log | tail -15
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $OUT/smoke.log; exit 1; }
echo "smoke ok"
timeout -k 10 400 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline "$@" > $OUT/bench.log 2>&1; echo "bench rc=$?"
tail -c 1200 $OUT/bench.log
