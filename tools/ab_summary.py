"""Print ms/step, aggregate GB/s and GEMM GB/s of bench.py JSON lines (argv: files)."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith("{"):
            d = json.loads(line)
            r, g = d.get("roofline") or {}, d.get("gemm") or {}
            print(f"{f}: {d['ms_per_step']:.2f} ms/step  aggregate {r.get('achieved')} GB/s  gemm {g.get('achieved')} GB/s "
                  f"({g.get('avg_launch_ms')} ms avg)")
