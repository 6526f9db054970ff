#!/bin/bash
# GPU box: decoder-focused build A/B (tools/ab_build.sh libraries): bench-step hashes, then the CFM solve at B = 32
# and B = 256 (tools/dec_2stream.py), interleaved twice. Usage: bash tools/r5_decab.sh TAG A B
set -o pipefail
TAG=$1; A=$2; Bn=$3; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
lib() { echo "$PWD/matcha-tts_amd/ab/$1.so"; }
for n in "$A" "$Bn"; do
  MT_LIB=$(lib "$n") timeout -k 10 300 python3 tools/syn_hash.py > "$OUT/hash_$n.log" 2>&1 || { echo "hash $n failed"; tail -5 "$OUT/hash_$n.log"; exit 1; }
  echo "$n: $(grep hash "$OUT/hash_$n.log" | tr '\n' ' ')"
done
for r in 1 2; do for n in "$A" "$Bn"; do for b in 32 256; do
  MT_LIB=$(lib "$n") timeout -k 10 300 python3 tools/dec_2stream.py $b 728 10 > "$OUT/d${b}_$n.log" 2>&1 || { echo "dec $n failed"; tail -5 "$OUT/d${b}_$n.log"; exit 1; }
  echo "$n decoder B=$b $(grep '^one' "$OUT/d${b}_$n.log" | head -1)"
done; done; done
