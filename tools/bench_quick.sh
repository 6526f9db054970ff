#!/bin/bash
# the default bench line (north-star record included), no CPU baseline
mkdir -p gpurun_out/$1
timeout -k 10 500 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/$1/bench.log 2>&1; echo "bench rc=$?"
grep '^{"metric"' gpurun_out/$1/bench.log | python3 -c "
import json,sys
d=json.loads(sys.stdin.read())
ns=d.get('north_star') or {}
print('value', d['value'], 'ms', d['ms_per_step'], 'ns', ns.get('value'), ns.get('ms_per_step'))
for k,v in d['roofline'].get('by_kernel',{}).items(): print(' ', k, v['launch_ms'], v['tflops'], v['frac'])
"
