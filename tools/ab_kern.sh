#!/bin/bash
# Build-vs-build A/B per KERNEL (GPU box): the bench step's ragged vocoder (tools/voc_time.py) under
# `rocprofv3 --kernel-trace --stats` once per library and batch, interleaved A, B, A, B; prints the average launch
# time of every vocoder kernel per run (tools/kstats.py). Libraries from tools/ab_build.sh.
#   bash tools/ab_kern.sh TAG NAME_A NAME_B [BATCHES]
set -o pipefail
TAG=$1; A=$2; Bn=$3; BATCHES=${4:-"32 256"}
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
lib() { echo "$PWD/matcha-tts_amd/ab/$1.so"; }
for n in "$A" "$Bn"; do [ -f "$(lib "$n")" ] || { echo "missing $(lib "$n")"; exit 2; }; done
for bt in $BATCHES; do
  # the step's mel and lengths from the working tree's library, once (tools/voc_time.py VOC_CACHE)
  export VOC_CACHE=$OUT/mel_b$bt.pt
  timeout -k 10 300 python3 tools/voc_time.py "$bt" 2 > "$OUT/cache_b$bt.log" 2>&1 || { echo "FAILED cache"; tail -5 "$OUT/cache_b$bt.log"; exit 1; }
  for r in 1 2; do for n in "$A" "$Bn"; do
  d=$OUT/${n}_b${bt}_$r
  MT_LIB=$(lib "$n") timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$d" -o run --output-format csv -- \
    python3 tools/voc_time.py "$bt" 5 > "$d.log" 2>&1 || { echo "FAILED $d"; tail -5 "$d.log"; exit 1; }
  cp "$(find "$d" -name '*kernel_stats.csv' | head -1)" "$d.csv" && rm -rf "$d"  # gpurun_out stays small
  echo "== $n B=$bt run $r: $(grep vocoder "$d.log")"
  python3 tools/kstats.py "$d.csv" > "$d.txt"; head -24 "$d.txt"
done; done
rm -f "$VOC_CACHE"
done
