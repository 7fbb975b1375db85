"""Kernel-busy time against wall time per batch of the fused small-batch step, from a rocprofv3 --kernel-trace CSV of
tools/sb_prof.py (VERDICT r05 "next" 7).  A batch = one k_batched_copy (the device collation) and the step kernels after
it (k_sb_*); the last --steps batches are summarised: kernel-busy = the sum of their kernel durations (one stream: no
overlap), wall = first collation start to last kernel end, launch gaps = wall - busy.

    python tools/sb_busy.py <dir with *kernel_trace.csv> [--steps 200] [--label default] > profiles/r06/sb_busy_<label>.json
"""
import argparse
import collections
import csv
import glob
import json
import os
import re
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--label", default="")
    args = ap.parse_args()
    rows = []
    for f in glob.glob(os.path.join(args.dir, "**", "*kernel_trace.csv"), recursive=True):
        rows += list(csv.DictReader(open(f)))
    rows = [r for r in rows if "k_batched_copy" in r["Kernel_Name"] or "k_sb_" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    batches, cur = [], None
    for r in rows:
        if "k_batched_copy" in r["Kernel_Name"]:
            cur = []
            batches.append(cur)
        if cur is not None:
            cur.append(r)
    batches = batches[-args.steps:]
    busy = [sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in b) for b in batches]
    wall = (int(batches[-1][-1]["End_Timestamp"]) - int(batches[0][0]["Start_Timestamp"])) / len(batches)
    per = collections.defaultdict(list)
    for b in batches:
        for r in b:
            name = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("hgin::(anonymous namespace)::", ""))
            per[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {"label": args.label, "batches": len(batches), "launches_per_batch": statistics.median(len(b) for b in batches),
           "kernel_ms_per_batch": round(statistics.mean(busy) / 1e6, 5),
           "wall_ms_per_batch": round(wall / 1e6, 5),
           "gap_ms_per_batch": round(wall / 1e6 - statistics.mean(busy) / 1e6, 5),
           "kernels_us": {k: {"calls_per_batch": len(v) / len(batches), "avg_us": round(statistics.mean(v), 2)}
                          for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1]))},
           "source": "rocprofv3 --kernel-trace of tools/sb_prof.py; wall from the first collation start to the last "
                     "kernel end of the summarised batches"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
