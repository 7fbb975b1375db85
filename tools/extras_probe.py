"""Run bench.py's non-headline extras alone (no cfg3 headline): the HetroGAT relation (gat_extra) and the real-loop
batches with the per-switch configs (batches_extra).  Prints one JSON line.

    python tools/extras_probe.py [--only gat,batches]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--only", default="gat,batches")
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    out = {}
    for name in args.only.split(","):
        out[name] = bench.gat_extra(dev) if name == "gat" else bench.batches_extra(dev)
        print(json.dumps({name: out[name]}), flush=True)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
