# mt_vconv with 4 loader waves that alone keep the staging cursors (MT_VCONV_LOADERS=4) vs all 8: A/B + tests
# with 4 loaders
set -o pipefail
mkdir -p gpurun_out/r3ee
for r in 1 2; do for k in 8 4; do
  MT_VCONV_LOADERS=$k timeout -k 10 200 python tools/voc_time.py 32 10 > gpurun_out/r3ee/v.log 2>&1 || { tail -5 gpurun_out/r3ee/v.log; exit 1; }
  echo "loaders=$k $(tail -1 gpurun_out/r3ee/v.log)"
done; done
for k in 8 4; do
  MT_VCONV_LOADERS=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3ee/d.log 2>&1 || exit 1
  echo "loaders=$k decoder $(grep '^one' gpurun_out/r3ee/d.log | head -1)"
  MT_VCONV_LOADERS=$k timeout -k 10 120 python tools/enc_bench.py 32 30 > gpurun_out/r3ee/e.log 2>&1 || exit 1
  echo "loaders=$k $(tail -1 gpurun_out/r3ee/e.log)"
done
for k in 8 4; do
  MT_VCONV_LOADERS=$k timeout -k 10 200 python tools/voc_time.py 256 3 > gpurun_out/r3ee/v.log 2>&1 || exit 1
  echo "loaders=$k $(tail -1 gpurun_out/r3ee/v.log)"
done
MT_VCONV_LOADERS=4 timeout -k 10 500 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_bench_shapes.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3ee/t.log 2>&1; echo "tests(4 loaders) rc=$?"; tail -2 gpurun_out/r3ee/t.log
