"""Per-kernel HBM traffic from two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE), grouped by kernel name (template
arguments kept): dispatches, read / write GB per dispatch (read = 2 x FETCH_SIZE, MI355X_MICROARCH.md's gfx950
correction, as tools/pmc_traffic.py) and the total per step.
    python tools/pmc_kernels.py <fetch_dir> <write_dir> <steps> > profiles/.../pmc_kernels.txt"""
import collections
import csv
import glob
import os
import re
import sys


def load(d, counter):
    out = collections.defaultdict(dict)
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter:
                continue
            k = re.sub(r"\(.*", "", r["Kernel_Name"].replace("void ", "").replace("hgin::(anonymous namespace)::", ""))
            key = (f, r["Dispatch_Id"])
            out[k][key] = out[k].get(key, 0.0) + float(r["Counter_Value"])
    return out


def main():
    fetch, write, steps = load(sys.argv[1], "FETCH_SIZE"), load(sys.argv[2], "WRITE_SIZE"), float(sys.argv[3])
    print(f"{'kernel':60s} {'disp':>5s} {'read GB/disp':>13s} {'write GB/disp':>14s} {'GB/step':>9s}")
    tot = 0.0
    for k in sorted(fetch, key=lambda k: -sum(fetch[k].values())):
        n = len(fetch[k])
        rd = 2 * sum(fetch[k].values()) * 1024 / n / 1e9
        wr = sum(write.get(k, {}).values()) * 1024 / max(len(write.get(k, {})), 1) / 1e9
        per_step = (rd + wr) * n / steps
        tot += per_step
        print(f"{k[:60]:60s} {n:5d} {rd:13.3f} {wr:14.3f} {per_step:9.2f}")
    print(f"total {tot:.2f} GB per step (the --steps + --warmup steps of the command: pass the count)")


if __name__ == "__main__":
    main()
