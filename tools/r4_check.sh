#!/bin/bash
# Round-4 working check (one GPU call): bit-identity tests of mt_vconv's compile-time K loop (base build) and of
# mt_rbconv's ping-pong variant (matcha-tts_amd/ab/pp.so, copied over the box's scratch copy of the library), the
# op-level rbconv timing of both builds, and the compile-time / runtime-cursor decoder A/B. Usage: bash tools/r4_check.sh TAG
TAG=${1:-r4check}
OUT=gpurun_out/$TAG
mkdir -p $OUT
LIB=matcha-tts_amd/libmatcha_hip.so
timeout -k 10 300 python -u -m pytest tests/test_gpu_vconv_ct.py -x -v --timeout 250 --timeout-method thread -p no:cacheprovider > $OUT/ct_tests.log 2>&1; rc=$?
grep -E "PASSED|FAILED|Error" $OUT/ct_tests.log | tail -6; [ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u tools/rbconv_bench.py 3 > $OUT/rbconv_bench_base.log 2>&1; tail -1 $OUT/rbconv_bench_base.log
for ct in 1 0; do MT_VCONV_CT=$ct timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > $OUT/d32_$ct.log 2>&1 || exit 1; echo "ct=$ct B=32 $(grep '^one' $OUT/d32_$ct.log | head -1)"; done
if [ -f matcha-tts_amd/ab/pp.so ]; then
  cp matcha-tts_amd/ab/pp.so $LIB
  timeout -k 10 240 python -u -m pytest tests/test_gpu_rbconv.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pp_tests.log 2>&1; rc=$?
  tail -3 $OUT/pp_tests.log; [ $rc -le 1 ] || exit $rc
  timeout -k 10 300 python -u tools/rbconv_bench.py 3 > $OUT/rbconv_bench_pp.log 2>&1; cat $OUT/rbconv_bench_pp.log
  MT_LIB=$PWD/matcha-tts_amd/ab/pp.so timeout -k 10 200 python tools/voc_time.py 32 10 > $OUT/v32_pp.log 2>&1; echo "pp $(tail -1 $OUT/v32_pp.log)"
  MT_LIB=$PWD/matcha-tts_amd/ab/base.so timeout -k 10 200 python tools/voc_time.py 32 10 > $OUT/v32_base.log 2>&1; echo "base $(tail -1 $OUT/v32_base.log)"
  cp matcha-tts_amd/ab/base.so $LIB
fi
echo done
