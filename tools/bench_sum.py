#!/usr/bin/env python3
"""One-screen summary of a bench.py JSON line (the headline, north star, general attention, roofline by kernel).
Usage: python tools/bench_sum.py gpurun_out/TAG/bench.log"""
import json
import sys

line = next(l for l in open(sys.argv[1]) if l.startswith('{"metric"'))
d = json.loads(line)
ns = d.get("north_star") or {}
ga = d.get("general_attention") or {}
print(f"value {d['value']:.1f} ({d['ms_per_step']} ms) | north star {ns.get('value')} ({ns.get('ms_per_step')} ms) | "
      f"general attention {ga.get('value')}")
print(f"roofline frac {d['roofline']['frac']} | north star {ns.get('roofline', {}).get('frac')} | traffic "
      f"{d['roofline'].get('traffic')}")
for k, v in d["roofline"].get("by_kernel", {}).items():
    print(f"  {k:9s} {v['launch_ms']:.4f} ms/launch {v['tflops']:7.1f} TF/s frac {v['frac']}")
