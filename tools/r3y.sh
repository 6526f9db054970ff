# XCD-aligned decoder streaming kernels (gn_apply, uniform attention part / apply) + prefetched o_b GEMVs: A/B
set -o pipefail
mkdir -p gpurun_out/r3y
for r in 1 2; do for k in 0 1; do
  MT_XCD_TILES=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3y/b32.log 2>&1 || exit 1
  echo "xcd_tiles=$k B=32 $(grep '^one' gpurun_out/r3y/b32.log | head -1)"
done; done
for k in 0 1; do
  MT_XCD_TILES=$k timeout -k 10 200 python tools/dec_2stream.py 256 756 3 > gpurun_out/r3y/b256.log 2>&1 || exit 1
  echo "xcd_tiles=$k B=256 $(grep '^one' gpurun_out/r3y/b256.log | head -1)"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_shapes.py tests/test_gpu_model.py tests/test_gpu_parity_bf16.py -x -q --timeout 250 --timeout-method thread > gpurun_out/r3y/t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r3y/t.log
