"""§8 F4 measurement: the queueing-theory baseline over a collated batch of RouteNet-shaped samples, HIP path
(hgin.qt.QTBaseline) vs the reference's CPU algorithm (oracle/qt_cpu.py = models.py:15-158 on torch CPU ops).

    python tools/qt_bench.py [--samples 256] [--reps 5]

Reports samples/s for each (GPU: plan + 3 iterations + delay, inputs already on the device; the plan is
also timed separately), and the edges processed."""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hgin.qt import QTBaseline, plan  # noqa: E402
from hgin.qt_data import RouteSample, collate_routes, route_sample  # noqa: E402
from oracle.qt_cpu import qt_baseline  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--samples", type=int, default=256)
    ap.add_argument("--reps", type=int, default=5)
    args = ap.parse_args()
    rng = np.random.default_rng(0)
    samples = [route_sample(int(k), seed=i) for i, k in enumerate(rng.integers(25, 51, args.samples))]
    cpu = collate_routes(samples)
    dev = RouteSample(*(t.cuda() for t in (cpu.edge_index, cpu.edge_type, cpu.type, cpu.P, cpu.L)))
    qt = QTBaseline()
    qt(dev)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.reps):
        out = qt(dev)
    torch.cuda.synchronize()
    t_gpu = (time.perf_counter() - t0) / args.reps
    t0 = time.perf_counter()
    for _ in range(args.reps):
        plan(dev.edge_index, dev.edge_type, dev.type, "cuda")
    torch.cuda.synchronize()
    t_plan = (time.perf_counter() - t0) / args.reps
    t0 = time.perf_counter()
    ref = qt_baseline(cpu.edge_index, cpu.edge_type, cpu.type, cpu.P, cpu.L)
    t_cpu = time.perf_counter() - t0
    err = float(((out[0].cpu() - ref[0]).abs() / ref[0].abs().clamp_min(1e-12)).max())
    print(json.dumps({"samples": args.samples, "vertices": cpu.num_nodes, "edges": int(cpu.edge_index.shape[1]),
                      "gpu_ms": round(t_gpu * 1e3, 3), "gpu_plan_ms": round(t_plan * 1e3, 3),
                      "cpu_ms": round(t_cpu * 1e3, 1), "gpu_samples_per_s": round(args.samples / t_gpu, 1),
                      "cpu_samples_per_s": round(args.samples / t_cpu, 2), "cpu_threads": torch.get_num_threads(),
                      "max_rel_err_delay": err}))


if __name__ == "__main__":
    main()
