"""Turn two rocprofv3 --pmc passes (FETCH_SIZE, WRITE_SIZE) into per-launch HBM bytes of one kernel.

    python tools/pmc_traffic.py <fetch_dir> <write_dir> <kernel-substring> <out.json> [algorithmic_bytes]

FETCH_SIZE / WRITE_SIZE are in KiB per dispatch (TCC_EA0_RDREQ / WRREQ based).  Per MI355X_MICROARCH.md
§HBM, on gfx950 FETCH_SIZE reports exactly half the bytes of a wide coalesced streaming read (128-B
requests tallied as 64 B), so the corrected read bytes are 2 x FETCH_SIZE; WRITE_SIZE is exact for 16-B
per lane stores.  Both raw and corrected values are recorded.
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kname):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        raise SystemExit(f"no counter_collection.csv under {d}")
    vals = {}
    for f in files:
        for r in csv.DictReader(open(f)):
            if r.get("Counter_Name") != counter or kname not in r.get("Kernel_Name", ""):
                continue
            key = (f, r["Dispatch_Id"])
            vals[key] = vals.get(key, 0.0) + float(r["Counter_Value"])
    return list(vals.values())


def main():
    fetch_dir, write_dir, kname, out = sys.argv[1:5]
    algo = float(sys.argv[5]) if len(sys.argv) > 5 else None
    fetch = per_dispatch(fetch_dir, "FETCH_SIZE", kname)
    write = per_dispatch(write_dir, "WRITE_SIZE", kname)
    f_kib = sum(fetch) / len(fetch)
    w_kib = sum(write) / len(write)
    raw = (f_kib + w_kib) * 1024
    corrected = (2 * f_kib + w_kib) * 1024
    res = {"kernel": kname, "dispatches_fetch": len(fetch), "dispatches_write": len(write),
           "fetch_kib_per_launch": f_kib, "write_kib_per_launch": w_kib, "bytes_per_launch_raw": raw,
           "bytes_per_launch": corrected,
           "source": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE (separate passes); bytes = (2*FETCH_SIZE + "
                     "WRITE_SIZE) * 1024 per MI355X_MICROARCH.md gfx950 FETCH_SIZE correction"}
    if algo:
        res["algorithmic_bytes_per_launch"] = algo
        res["traffic_over_algorithmic"] = corrected / algo
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
