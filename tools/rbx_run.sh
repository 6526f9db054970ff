#!/bin/bash
# rbconv epilogue ablation timing (wrong-result builds from tools/exp_build.sh, timing only)
mkdir -p gpurun_out/rbx
for n in ${RBX:-0 1 2 3 0}; do
  MT_LIB=$PWD/matcha-tts_amd/ab/rbx$n.so timeout -k 10 240 python tools/rbconv_bench.py 3 32 > gpurun_out/rbx/r$n.log 2>&1 || { tail -5 gpurun_out/rbx/r$n.log; exit 1; }
  echo "== rbx$n"; cat gpurun_out/rbx/r$n.log
done
