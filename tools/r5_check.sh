#!/bin/bash
# GPU box: the round-5 pair-kernel checks: GPU tests of the vocoder paths, then the bench line (no CPU baseline / fp32
# record) and the ragged vocoder alone at B = 32 / 256. Usage: bash tools/r5_check.sh TAG   (TESTS=... adds tests)
set -o pipefail
TAG=$1; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_vpair_variants.py \
  tests/test_gpu_ragged.py ${TESTS:-} > "$OUT/tests.log" 2>&1 || { echo "tests failed"; tail -30 "$OUT/tests.log"; exit 1; }
tail -2 "$OUT/tests.log"
timeout -k 10 600 python -u bench.py --no-cpu-baseline --no-fp32 > "$OUT/bench.log" 2>&1 || { echo "bench failed"; tail -20 "$OUT/bench.log"; exit 1; }
tail -1 "$OUT/bench.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value'], d['ms_per_step'], 'north', d.get('north_star',{}).get('value'), d.get('north_star',{}).get('ms_per_step'))"
for b in 32 256; do
  timeout -k 10 300 python3 tools/voc_time.py $b 5 > "$OUT/voc$b.log" 2>&1 || { echo "voc_time failed"; tail -5 "$OUT/voc$b.log"; exit 1; }
  tail -1 "$OUT/voc$b.log"
done
