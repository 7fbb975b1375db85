"""One training step's kernel sequence from a rocprofv3 --kernel-trace CSV (argv: csv [marker]).
The step is the span between the last two launches whose name contains the marker (default: the fused
head's forward kernel, launched once per step)."""
import csv
import re
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
marker = sys.argv[2] if len(sys.argv) > 2 else "k_head_fwd_vec"
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
step = rows[idx[-3] + 1: idx[-2] + 1]
tot = 0.0
for r in step:
    n = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    n = re.sub(r"^void ", "", n)
    n = re.sub(r"\(.*", "", n)[:70]
    d = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
    tot += d
    print(f"{d:8.1f} {r['Grid_Size_X']:>9} {r['Grid_Size_Y']:>3}  {n}")
wall = (int(step[-1]["End_Timestamp"]) - int(step[0]["Start_Timestamp"])) / 1e3
print(f"kernels {tot:.1f} us, wall {wall:.1f} us, {len(step)} launches")
