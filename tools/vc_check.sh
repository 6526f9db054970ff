#!/bin/bash
# vconv iteration: op + vocoder parity tests, vocoder A/B (vconv on/off), kernel trace of one A/B run.
# Usage: bash tools/vc_check.sh TAG
TAG=$1
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 200 python -u -m pytest tests/test_gpu_ops.py tests/test_gpu_model.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 120 python tools/voc_ab.py 32 728 3 > $OUT/ab.log 2>&1 || { tail $OUT/ab.log; exit 1; }
grep vocoder $OUT/ab.log
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- python3 tools/voc_ab.py 32 728 1 > $OUT/prof.log 2>&1 || exit 1
python3 tools/vc_table.py $OUT/prof/run_kernel_trace.csv
