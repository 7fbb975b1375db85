"""§8 F1 measurement: shuffled mini-batches of small graphs (the reference's real training loop).

    python tools/batch_bench.py [--graphs 512] [--batch 8] [--steps 50] [--warmup 5] [--schema cfg1|w128]

Reference loop (train.py:25-44 over dataset.py:239-244): each step the DataLoader collates 8 graphs on the
host, ``sample.cuda()`` copies the batch, and the GPU scatters from unsorted COO.  Three variants run the same
train step (zero_grad, fwd, sqrt-MAPE, bwd, Adam) on the same id sequence:

  host   — hgin.data.collate on the CPU + .to(device) + per-step CSR/CSC sort (what a drop-in without F1 does)
  device — GraphStore.collate: one hgin_batched_copy launch assembles x / y / batch / edge_index / CSR / CSC
  static — one fixed batch reused every step (upper bound: no collation cost at all)

Reports ms/step and edges/s (convolved edges of the batch / step time) for each, plus collation-only times.
"""
from __future__ import annotations

import argparse
import dataclasses
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from hgin import HetroGIN  # noqa: E402
from hgin.data import CONFIGS, REL_LN, REL_LP, REL_NL, REL_PL, collate, scaled_config, synthetic_graph  # noqa: E402
from hgin.store import GraphStore  # noqa: E402
from hgin.train import train_step  # noqa: E402

CONV = (REL_PL, REL_LP, REL_LN, REL_NL)


def schema(name):
    if name == "cfg1":      # reference 7/7/3 layout, config.json flags, H=8 (BASELINE configs[0] per graph)
        return CONFIGS["cfg1"]
    if name == "w128":      # cfg2 schema (F=H=128, divided/bl features) at 1/1000 size per graph
        return scaled_config(CONFIGS["cfg2"], 1e-3, name="cfg2/1000")
    raise ValueError(name)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--graphs", type=int, default=512)
    ap.add_argument("--batch", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--schema", default="cfg1")
    args = ap.parse_args()
    dev = torch.device("cuda")
    base = schema(args.schema)
    rng = np.random.default_rng(0)
    graphs = []
    for i in range(args.graphs):     # per-graph sizes vary (0.5x .. 1.5x), like the GNNet topologies
        cfg = scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}")
        graphs.append(synthetic_graph(cfg, seed=i))
    t0 = time.perf_counter()
    store = GraphStore.build(graphs, device=dev)
    torch.cuda.synchronize()
    build_s = time.perf_counter() - t0
    n_batches = args.warmup + args.steps
    order = [rng.choice(args.graphs, args.batch, replace=False).tolist() for _ in range(n_batches)]
    conv_edges = [sum(int(store.edge_off[r][g + 1] - store.edge_off[r][g]) for r in CONV for g in ids)
                  for ids in order]

    torch.manual_seed(1997)
    kw = base.model_kwargs({"link": base.f_link, "path": base.f_path, "node": base.f_node})
    results = {}

    def run(variant):
        torch.manual_seed(1997)
        # the ctor mutates input_channels (models.py:261-269): a fresh dict per model
        model = HetroGIN(**{**kw, "input_channels": dict(kw["input_channels"])}).to(dev)
        opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
        fixed = store.collate(order[0]) if variant == "static" else None

        def batch_for(ids):
            if variant == "device":
                return store.collate(ids)
            if variant == "host":
                return collate([graphs[g] for g in ids]).to(dev, non_blocking=False)
            return fixed

        for i in range(args.warmup):
            train_step(model, opt, batch_for(order[i]))
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.warmup, n_batches):
            train_step(model, opt, batch_for(order[i]))
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t) / args.steps
        edges = np.mean(conv_edges[args.warmup:]) if variant != "static" else conv_edges[0]
        # collation alone (host: collate + H2D + CSR/CSC sort; device: batched copy)
        from hgin import ops
        torch.cuda.synchronize()
        t = time.perf_counter()
        for i in range(args.warmup, n_batches):
            b = batch_for(order[i])
            if variant == "host":
                for r, e in b.edge_index.items():
                    g = ops.relation_graph(e, b.x[r[0]].shape[0], b.x[r[2]].shape[0])
                    g.csc
        torch.cuda.synchronize()
        ct = (time.perf_counter() - t) / args.steps
        results[variant] = {"ms_per_step": round(dt * 1e3, 4), "edges_per_s": round(edges / dt, 1),
                            "collate_ms": round(ct * 1e3, 4) if variant != "static" else 0.0}

    for v in ("static", "device", "host"):
        run(v)

    # hipGraph: padded static batch, captured once, replayed per batch (hgin/graphs.py)
    from hgin.graphs import CapturedTrainStep
    torch.manual_seed(1997)
    model = HetroGIN(**{**kw, "input_channels": dict(kw["input_channels"])}).to(dev)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), capturable=True)
    step = CapturedTrainStep(model, opt, store, args.batch, warmup_ids=order[:args.warmup], warmup=args.warmup)
    torch.cuda.synchronize()
    t = time.perf_counter()
    for i in range(args.warmup, n_batches):
        step.step(order[i])
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t) / args.steps
    results["graph"] = {"ms_per_step": round(dt * 1e3, 4),
                        "edges_per_s": round(float(np.mean(conv_edges[args.warmup:])) / dt, 1),
                        "collate_ms": results["device"]["collate_ms"],
                        "note": "padded static batch (capacity = batch x largest graph), one replay per step"}
    out = {"workload": f"{args.graphs} {base.name}-schema graphs resident, shuffled batches of {args.batch} "
                       f"(sizes 0.5x-1.5x), hidden {base.hidden}, {base.layers} layers, fp32",
           "store_build_s": round(build_s, 3), "mean_conv_edges_per_batch": float(np.mean(conv_edges)),
           "steps": args.steps, "warmup": args.warmup, **results}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
