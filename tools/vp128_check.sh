#!/bin/bash
# Fused-pair iteration: pair bit-identity + probe tests, a traced bench, a plain bench and the per-kind ResBlock
# launch probe at B = 256. Usage: bash tools/vp128_check.sh TAG
OUT=gpurun_out/${1:-vp128a}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "pair or probe or vconv_stages or generator" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > $OUT/prof_bench.log 2>&1 || { tail $OUT/prof_bench.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench.log 2>&1 || { tail $OUT/bench.log; exit 1; }
tail -1 $OUT/bench.log | cut -c1-400
timeout -k 10 120 python3 tools/pair_probe.py 256 756 2 > $OUT/probe256.log 2>&1 || { tail $OUT/probe256.log; exit 1; }
grep "launches" $OUT/probe256.log
