#!/bin/bash
# Round profile: kernel-trace stats + HBM counter passes on a bench command (default: the headline B=32 workload;
# extra args go to bench.py, e.g. `--batch 256` for the north-star configuration). The counter passes cover the
# bench's roofline family: the HiFi-GAN ResBlock convs of stages 1-2 (rbconv_kernel; vconv_kernel with the ResBlock
# epilogues ACT, RESID|DUAL, RESID[|ACCUM][|DIV][|DUAL] when mt_rbconv is off) and the fused ResBlock pairs
# (vpair128_kernel, vpair_kernel, vpair3_kernel, vpair32_kernel); the decoder's and the upsamplers' vconv launches
# are excluded.
# Usage: bash tools/round_profile.sh TAG [bench args...]
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
CMD="python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --no-north-star --quick $*"
RE="rbconv_kernel|vpair(32|128|3)?_kernel|vconv_kernel(ILi(8|17|1|3|5|7|21|23)ELi[0-9]+ELb0E|<(8|17|1|3|5|7|21|23), [0-9]+, false)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- $CMD > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --kernel-include-regex "$RE" -d $OUT/fetch -o pmc --output-format csv -- $CMD > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --kernel-include-regex "$RE" -d $OUT/write -o pmc --output-format csv -- $CMD > $OUT/write.log 2>&1 || exit $?
python3 tools/pmc_traffic.py $OUT/fetch/pmc_counter_collection.csv $OUT/write/pmc_counter_collection.csv \
  "$RE" $OUT/pmc_vconv.json "$CMD" || exit $?
python3 tools/prof_summary.py $(find $OUT/trace -name '*kernel_trace.csv' | head -1) 40 > $OUT/step_breakdown.txt 2>&1
cp $(find $OUT/trace -name '*kernel_stats.csv' | head -1) $OUT/kernel_stats.csv
echo "profile done"
