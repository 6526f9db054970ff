# EARLY residual loads in mt_vconv's HiFi-GAN conv2 epilogues: vocoder A/B (MT_VCONV_EARLY=0 vs default), then the
# generator / bench-shape parity tests
set -o pipefail
mkdir -p gpurun_out/r3aa
for r in 1 2; do for k in 0 1; do
  MT_VCONV_EARLY=$k timeout -k 10 200 python tools/voc_time.py 32 10 > gpurun_out/r3aa/v.log 2>&1 || { tail -5 gpurun_out/r3aa/v.log; exit 1; }
  echo "early=$k $(tail -1 gpurun_out/r3aa/v.log)"
done; done
for k in 0 1; do
  MT_VCONV_EARLY=$k timeout -k 10 200 python tools/voc_time.py 256 3 > gpurun_out/r3aa/v.log 2>&1 || { tail -5 gpurun_out/r3aa/v.log; exit 1; }
  echo "early=$k $(tail -1 gpurun_out/r3aa/v.log)"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_ragged.py tests/test_gpu_bench_shapes.py tests/test_gpu_model.py -x -q --timeout 300 --timeout-method thread > gpurun_out/r3aa/t.log 2>&1; echo "tests rc=$?"; tail -2 gpurun_out/r3aa/t.log
