# build A/B: libmatcha_hip_old.so (whichever older build was copied there) vs the current library
set -o pipefail
mkdir -p gpurun_out/r3ll
OLD=$PWD/matcha-tts_amd/libmatcha_hip_old.so
NEW=$PWD/matcha-tts_amd/libmatcha_hip.so
for r in 1 2; do for L in old new; do
  [ $L = old ] && LIB=$OLD || LIB=$NEW
  MT_LIB=$LIB timeout -k 10 200 python tools/dec_2stream.py 32 728 10 > gpurun_out/r3ll/d.log 2>&1 || { tail -5 gpurun_out/r3ll/d.log; exit 1; }
  echo "$L decoder B=32 $(grep '^one' gpurun_out/r3ll/d.log | head -1)"
  MT_LIB=$LIB timeout -k 10 200 python tools/voc_time.py 32 10 > gpurun_out/r3ll/v.log 2>&1 || { tail -5 gpurun_out/r3ll/v.log; exit 1; }
  echo "$L $(tail -1 gpurun_out/r3ll/v.log)"
done; done
for L in old new; do
  [ $L = old ] && LIB=$OLD || LIB=$NEW
  MT_LIB=$LIB timeout -k 10 300 python tools/dec_2stream.py 256 756 3 > gpurun_out/r3ll/d.log 2>&1 || exit 1
  echo "$L decoder B=256 $(grep '^one' gpurun_out/r3ll/d.log | head -1)"
done
