# prologue DMA split (MT_VCONV_PRO 0 / 1 / 2): correctness on the vconv-heavy tests first, then decoder / vocoder A/B
set -o pipefail
mkdir -p gpurun_out/r3jj
for k in 1 2; do
  MT_VCONV_PRO=$k timeout -k 10 400 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_bench_shapes.py tests/test_gpu_parity_bf16.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r3jj/t$k.log 2>&1; rc=$?; echo "tests pro=$k rc=$rc $(tail -1 gpurun_out/r3jj/t$k.log)"; [ $rc -eq 0 ] || exit 1
done
for r in 1 2; do for k in 0 1 2; do
  MT_VCONV_PRO=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3jj/d.log 2>&1 || { tail -5 gpurun_out/r3jj/d.log; exit 1; }
  echo "pro=$k decoder B=32 $(grep '^one' gpurun_out/r3jj/d.log | head -1)"
done; done
for r in 1 2; do for k in 0 1 2; do
  MT_VCONV_PRO=$k timeout -k 10 200 python tools/voc_time.py 32 10 > gpurun_out/r3jj/v.log 2>&1 || exit 1
  echo "pro=$k $(tail -1 gpurun_out/r3jj/v.log)"
done; done
