# late next-launch prefetch on one-round grids (MT_VCONV_PF_LATE=1) vs none: decoder B=32 x3, bench line x2
set -o pipefail
mkdir -p gpurun_out/r3hh
for r in 1 2 3; do for k in 0 1; do
  MT_VCONV_PF_LATE=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3hh/d.log 2>&1 || { tail -5 gpurun_out/r3hh/d.log; exit 1; }
  echo "late=$k decoder B=32 $(grep '^one' gpurun_out/r3hh/d.log | head -1)"
done; done
for r in 1 2; do for k in 0 1; do
  MT_VCONV_PF_LATE=$k timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/r3hh/b.log 2>&1 || exit 1
  echo "late=$k $(grep '^{' gpurun_out/r3hh/b.log | head -c 150)"
done; done
