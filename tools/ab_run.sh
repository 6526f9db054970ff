#!/bin/bash
# Build-vs-build A/B, step 2 (GPU box): interleaved timing of libraries built by tools/ab_build.sh.
#   bash tools/ab_run.sh TAG NAME_A NAME_B [PAIRS]
# Per pair and library: the B=32 10-step CFM solve (tools/dec_2stream.py) and the bench step's ragged vocoder
# (tools/voc_time.py); then once per library the B=256 CFM solve. Every GPU step has its own time limit and the
# script stops at the first failure.
set -o pipefail
TAG=$1; A=$2; Bn=$3; PAIRS=${4:-2}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
lib() { echo "$PWD/matcha-tts_amd/ab/$1.so"; }
for n in "$A" "$Bn"; do [ -f "$(lib "$n")" ] || { echo "missing $(lib "$n"): run tools/ab_build.sh first"; exit 2; }; done
for r in $(seq "$PAIRS"); do for n in "$A" "$Bn"; do
  MT_LIB=$(lib "$n") timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > "$OUT/d32_$n.log" 2>&1 || { tail -5 "$OUT/d32_$n.log"; exit 1; }
  echo "$n decoder B=32 $(grep '^one' "$OUT/d32_$n.log" | head -1)"
  MT_LIB=$(lib "$n") timeout -k 10 200 python tools/voc_time.py 32 10 > "$OUT/v32_$n.log" 2>&1 || { tail -5 "$OUT/v32_$n.log"; exit 1; }
  echo "$n $(tail -1 "$OUT/v32_$n.log")"
done; done
for n in "$A" "$Bn"; do
  MT_LIB=$(lib "$n") timeout -k 10 300 python tools/dec_2stream.py 256 756 3 > "$OUT/d256_$n.log" 2>&1 || { tail -5 "$OUT/d256_$n.log"; exit 1; }
  echo "$n decoder B=256 $(grep '^one' "$OUT/d256_$n.log" | head -1)"
done
