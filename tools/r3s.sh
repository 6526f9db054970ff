# round 3 (second session): GPU suite, A/B of the vconv table-DMA prologue vs the HEAD build, phase timestamps, bench
set -o pipefail
mkdir -p gpurun_out/r3s
bash tools/gpu_tests.sh r3s_tests || exit 1
bash tools/lib_ab.sh r3s_ab matcha-tts_amd/libmatcha_hip_base.so matcha-tts_amd/libmatcha_hip.so || exit 1
MT_LIB=matcha-tts_amd/libmatcha_hip_ts.so timeout -k 10 200 python -u tools/vconv_ts.py 32 728 > gpurun_out/r3s/ts32.txt 2>&1 || { echo ts failed; tail gpurun_out/r3s/ts32.txt; exit 1; }
head -40 gpurun_out/r3s/ts32.txt
timeout -k 10 400 python -u bench.py > gpurun_out/r3s/bench.log 2>&1; echo bench rc=$?; tail -c 1500 gpurun_out/r3s/bench.log
