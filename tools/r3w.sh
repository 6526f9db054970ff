# XCD-major vconv tile ownership: decoder CFM solve A/B (MT_XCD_TILES=0 vs default), encoder A/B, quick GPU check
set -o pipefail
mkdir -p gpurun_out/r3w
for r in 1 2; do for k in 0 1; do
  MT_XCD_TILES=$k timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3w/b32.log 2>&1 || exit 1
  echo "xcd_tiles=$k B=32 $(grep '^one' gpurun_out/r3w/b32.log | head -1)"
done; done
for k in 0 1; do
  MT_XCD_TILES=$k timeout -k 10 200 python tools/dec_2stream.py 256 756 3 > gpurun_out/r3w/b256.log 2>&1 || exit 1
  echo "xcd_tiles=$k B=256 $(grep '^one' gpurun_out/r3w/b256.log | head -1)"
done
for k in 0 1 0 1; do
  MT_XCD_TILES=$k timeout -k 10 120 python tools/enc_bench.py 32 30 > gpurun_out/r3w/enc.log 2>&1 || exit 1
  echo "xcd_tiles=$k $(tail -1 gpurun_out/r3w/enc.log)"
done
for L in matcha-tts_amd/libmatcha_hip_base.so matcha-tts_amd/libmatcha_hip_base.so; do
  MT_LIB=$L timeout -k 10 120 python tools/enc_bench.py 32 30 > gpurun_out/r3w/enc.log 2>&1 || exit 1
  echo "base $(tail -1 gpurun_out/r3w/enc.log)"
done
timeout -k 10 300 python -u -m pytest tests/test_gpu_bench_shapes.py -x -q --timeout 250 --timeout-method thread -k "decoder or encoder or variant" > gpurun_out/r3w/t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r3w/t.log
