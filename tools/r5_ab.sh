#!/bin/bash
# GPU box: build-vs-build A/B of two libraries from tools/ab_build.sh: bit identity (bench-step and Generator hashes),
# then interleaved timings (CFM solve at B = 32, ragged vocoder at B = 32 / 256). Usage: bash tools/r5_ab.sh TAG A B
set -o pipefail
TAG=$1; A=$2; Bn=$3; OUT=gpurun_out/$TAG; mkdir -p "$OUT"
lib() { echo "$PWD/matcha-tts_amd/ab/$1.so"; }
for n in "$A" "$Bn"; do
  MT_LIB=$(lib "$n") timeout -k 10 300 python3 tools/syn_hash.py > "$OUT/hash_$n.log" 2>&1 || { echo "hash $n failed"; tail -5 "$OUT/hash_$n.log"; exit 1; }
  MT_LIB=$(lib "$n") timeout -k 10 120 python3 tools/gen_hash.py >> "$OUT/hash_$n.log" 2>&1 || { echo "gen_hash $n failed"; exit 1; }
  echo "$n: $(grep hash "$OUT/hash_$n.log" | tr '\n' ' ')"
done
for r in 1 2; do for n in "$A" "$Bn"; do
  MT_LIB=$(lib "$n") timeout -k 10 200 python3 tools/dec_2stream.py 32 728 10 > "$OUT/d32_$n.log" 2>&1 || { echo "dec $n failed"; tail -5 "$OUT/d32_$n.log"; exit 1; }
  echo "$n decoder B=32 $(grep '^one' "$OUT/d32_$n.log" | head -1)"
  for b in 32 256; do
    MT_LIB=$(lib "$n") timeout -k 10 300 python3 tools/voc_time.py $b 5 > "$OUT/v${b}_$n.log" 2>&1 || { echo "voc $n failed"; tail -5 "$OUT/v${b}_$n.log"; exit 1; }
    echo "$n $(tail -1 "$OUT/v${b}_$n.log")"
  done
done; done
