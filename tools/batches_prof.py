"""bench.py's extras.batches workload alone (the reference's real loop: shuffled batches of 8 cfg1-schema graphs), a
rocprofv3 target:  rocprofv3 --kernel-trace --stats -- python3 tools/batches_prof.py [--steps 100]"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import torch  # noqa: E402

import bench  # noqa: E402

if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=100)
    args = ap.parse_args()
    print(json.dumps(bench.batches_extra(torch.device("cuda"), steps=args.steps)), flush=True)
