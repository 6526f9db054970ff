#!/bin/bash
# Interleaved A/B of two library builds on the CFM solve (B=32 and B=256): bash tools/lib_ab.sh TAG LIB_A LIB_B
TAG=$1; A=$2; Bl=$3
mkdir -p gpurun_out/$TAG
for r in 1 2; do for L in $A $Bl; do
  MT_LIB=$L timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/$TAG/b32.log 2>&1 || exit 1
  echo "$L B=32 $(grep '^one' gpurun_out/$TAG/b32.log | head -1)"
done; done
for L in $A $Bl; do
  MT_LIB=$L timeout -k 10 200 python tools/dec_2stream.py 256 756 3 > gpurun_out/$TAG/b256.log 2>&1 || exit 1
  echo "$L B=256 $(grep '^one' gpurun_out/$TAG/b256.log | head -1)"
done
