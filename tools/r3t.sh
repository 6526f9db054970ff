# deeper vconv rings: GPU suite, A/B vs the round-3 start build, phase timestamps
set -o pipefail
mkdir -p gpurun_out/r3t
bash tools/gpu_tests.sh r3t_tests || exit 1
bash tools/lib_ab.sh r3t_ab matcha-tts_amd/libmatcha_hip_base.so matcha-tts_amd/libmatcha_hip.so || exit 1
MT_LIB=matcha-tts_amd/libmatcha_hip_ts.so timeout -k 10 200 python -u tools/vconv_ts.py 32 728 > gpurun_out/r3t/ts32.txt 2>&1 || echo "ts (no ts build) rc=$?"
