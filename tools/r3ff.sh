# next-launch weight prefetch into L2 (VConvArgs::pf, MT_VCONV_PF) A/B on the decoder + bench, then tests
set -o pipefail
mkdir -p gpurun_out/r3ff
for r in 1 2; do for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3ff/d.log 2>&1 || { tail -5 gpurun_out/r3ff/d.log; exit 1; }
  echo "pf=$k decoder B=32 $(grep '^one' gpurun_out/r3ff/d.log | head -1)"
done; done
for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 300 python tools/dec_2stream.py 256 756 3 > gpurun_out/r3ff/d.log 2>&1 || exit 1
  echo "pf=$k decoder B=256 $(grep '^one' gpurun_out/r3ff/d.log | head -1)"
done
for k in 0 1; do
  MT_VCONV_PF=$k timeout -k 10 300 python bench.py --no-cpu-baseline --no-north-star > gpurun_out/r3ff/b.log 2>&1 || exit 1
  echo "pf=$k bench $(grep '^{' gpurun_out/r3ff/b.log | head -c 200)"
done
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity_bf16.py tests/test_gpu_model.py tests/test_gpu_batch1.py tests/test_gpu_bench_shapes.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ff/t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r3ff/t.log
