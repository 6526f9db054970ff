set -o pipefail
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_model.py tests/test_gpu_ops.py tests/test_gpu_bench_shapes.py -k "generator or pair or fused or vconv or vocoder or bench_step or uniform or cfm" > gpurun_out/r3h/t.log 2>&1; echo "tests rc=$?"; grep -E "rel-RMS|oracle:|passed|failed" gpurun_out/r3h/t.log | tail -20
timeout -k 10 300 python -u bench.py --quick --steps 20 --warmup 5 > gpurun_out/r3h/bench.log 2>&1; echo "bench rc=$?"
python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r3h/bench.log') if l.startswith('{')][-1]);print(d['value'],d['ms_per_step'],d['roofline']['frac'],json.dumps(d['roofline']['by_kernel']))"
timeout -k 10 200 python -u tools/dec_2stream.py 32 728 10 > gpurun_out/r3h/dec_fused.log 2>&1; tail -2 gpurun_out/r3h/dec_fused.log
MT_UNI_FUSED=0 timeout -k 10 200 python -u tools/dec_2stream.py 32 728 10 > gpurun_out/r3h/dec_split.log 2>&1; tail -2 gpurun_out/r3h/dec_split.log
