# next-launch weight prefetch on multi-round grids only: A/B decoder B=256 x3, B=32 x1, north-star bench
set -o pipefail
mkdir -p gpurun_out/r3gg
for r in 1 2 3; do for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 300 python tools/dec_2stream.py 256 756 3 > gpurun_out/r3gg/d.log 2>&1 || { tail -5 gpurun_out/r3gg/d.log; exit 1; }
  echo "pf=$k decoder B=256 $(grep '^one' gpurun_out/r3gg/d.log | head -1)"
done; done
for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3gg/d.log 2>&1 || exit 1
  echo "pf=$k decoder B=32 $(grep '^one' gpurun_out/r3gg/d.log | head -1)"
done
for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/r3gg/b.log 2>&1 || exit 1
  echo "pf=$k $(python3 -c "import json,sys;d=json.loads([l for l in open('gpurun_out/r3gg/b.log') if l.startswith('{')][0]);print('bench',d['value'],d['ms_per_step'],'north',d['north_star']['value'],d['north_star']['ms_per_step'])")"
done
