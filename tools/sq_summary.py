"""Summarise rocprofv3 --pmc SQ / GRBM passes of one kernel (tools/gpu_gemm_pmc2.sh layout: <dir>/<variant>_p<i>/
.../run_counter_collection.csv): per variant and kernel the per-launch counter means and the derived figures —
effective clock (GRBM_GUI_ACTIVE / 8 XCDs / wall, MI355X_MICROARCH.md's DVFS method), MFMA busy fraction of the SIMD
cycles (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)), VALU instructions per MFMA, waiting
fraction of the wave cycles.

    python tools/sq_summary.py gpurun_out/r04b/gemm_pmc2 [kernel-substring] > profiles/r04/gemm_pmc2.txt
"""
import collections
import csv
import glob
import os
import re
import statistics
import sys


def load(path, sub):
    vals = collections.defaultdict(lambda: collections.defaultdict(list))   # kernel -> counter -> [values]
    wall = collections.defaultdict(list)
    for f in glob.glob(os.path.join(path, "**", "*counter_collection.csv"), recursive=True):
        seen = set()
        for row in csv.DictReader(open(f)):
            k = row["Kernel_Name"]
            if sub and sub not in k:
                continue
            k = re.sub(r"\(.*", "", k.replace("void ", "").replace("hgin::(anonymous namespace)::", ""))
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            key = (k, row["Dispatch_Id"])
            if key not in seen:
                seen.add(key)
                wall[k].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-9)
    return vals, wall


def main():
    root = sys.argv[1]
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    variants = sorted({re.sub(r"_p\d+$", "", os.path.basename(d)) for d in glob.glob(os.path.join(root, "*_p*"))
                       if os.path.isdir(d)})
    for v in variants:
        merged = collections.defaultdict(dict)
        walls = collections.defaultdict(list)
        for d in sorted(glob.glob(os.path.join(root, v + "_p*"))):
            if not os.path.isdir(d):
                continue
            vals, wall = load(d, sub)
            for k, cs in vals.items():
                for c, xs in cs.items():
                    merged[k][c] = statistics.mean(xs)
                walls[k] += wall[k]
        for k, c in merged.items():
            w = statistics.mean(walls[k]) if walls[k] else float("nan")
            print(f"== {v}: {k}  (mean over launches; wall {w * 1e3:.3f} ms per launch)")
            for name in sorted(c):
                print(f"  {name:28s} {c[name]:.4g}")
            g = c.get("GRBM_GUI_ACTIVE")
            if g:
                print(f"  -> effective clock {g / 8 / w / 1e9:.2f} GHz" if w == w else "")
                if "SQ_VALU_MFMA_BUSY_CYCLES" in c:
                    print(f"  -> MFMA busy {c['SQ_VALU_MFMA_BUSY_CYCLES'] / (g / 8 * 1024):.1%} of the SIMD cycles")
            if c.get("SQ_INSTS_MFMA"):
                print(f"  -> VALU per MFMA {c.get('SQ_INSTS_VALU', float('nan')) / c['SQ_INSTS_MFMA']:.2f}, "
                      f"LDS per MFMA {c.get('SQ_INSTS_LDS', float('nan')) / c['SQ_INSTS_MFMA']:.2f}")
            if c.get("SQ_WAVE_CYCLES"):
                print(f"  -> waiting {c.get('SQ_WAIT_ANY', float('nan')) / c['SQ_WAVE_CYCLES']:.1%} of the wave "
                      f"cycles (dependencies {c.get('SQ_WAIT_INST_ANY', float('nan')) / c['SQ_WAVE_CYCLES']:.1%})")


if __name__ == "__main__":
    main()
