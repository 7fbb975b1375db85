"""Summarise a rocprofv3 --stats kernel CSV: per-kernel total / per-step time (argv: csv, steps)."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
steps = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'ms/step':>9} {'%':>6} {'calls':>6} {'avg_us':>9}  kernel")
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    t = float(r["TotalDurationNs"])
    if t / tot < 0.002:
        continue
    print(f"{t / 1e6 / steps:9.3f} {100 * t / tot:6.2f} {r['Calls']:>6} {float(r['AverageNs']) / 1e3:9.1f}  "
          f"{r['Name'][:100]}")
print(f"total {tot / 1e6 / steps:.3f} ms/step over {steps:g} steps")
# the aggregate family (what bench.py's roofline averages over: every hgin_aggregate_* launch)
agg = [r for r in rows if "k_agg" in r["Name"]]
if agg:
    calls = sum(int(r["Calls"]) for r in agg)
    ns = sum(float(r["TotalDurationNs"]) for r in agg)
    print(f"aggregate family (k_aggregate* + k_agg_q*): {calls} launches, average {ns / calls / 1e3:.1f} us, "
          f"{ns / 1e6 / steps:.3f} ms/step")
