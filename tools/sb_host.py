"""Host-side cost of the fused small-batch step's per-batch work (the GPU part is ~0.09 ms: when the host takes
longer, the device idles between batches).  Times, per call and without device syncs inside the timed loops:
the batch plan + descriptor table (numpy), the whole collate_into (+ the copy launch), the graph replay call,
and step() — each over 50 calls, median of 5 repetitions.
    python tools/sb_host.py"""
import json
import os
import statistics
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from hgin import HetroGIN
    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    from hgin.smallbatch import SmallBatchStep
    from hgin.store import GraphStore
    dev = torch.device("cuda")
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(0)
    graphs = [synthetic_graph(scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=i)
              for i in range(256)]
    store = GraphStore.build(graphs, device=dev, normalize=True)
    order = [rng.choice(256, 8, replace=False).tolist() for _ in range(400)]
    torch.manual_seed(1997)
    model = HetroGIN(**base.model_kwargs({"link": base.f_link, "path": base.f_path, "node": base.f_node})).to(dev)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
    st = SmallBatchStep(model, opt, store, 8, warmup_ids=order[:5], warmup=5)
    pb = st.batch
    out = {}

    def timed(name, fn, n=50):
        reps = []
        for r in range(5):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for k in range(n):
                fn(order[(r * n + k) % len(order)])
            t1 = time.perf_counter()
            torch.cuda.synchronize()
            reps.append((t1 - t0) / n * 1e6)
        out[name] = round(statistics.median(reps), 2)

    def desc(ids):
        p = store.plan(ids)
        store._descriptors(p[0], pb.x, pb.batch, pb.y, pb.edge_index, pb.csr, pb.csc, pb.m_valid, pb.goff,
                           pb.batch_size)
    timed("plan_us", store.plan)
    timed("plan_descriptors_us", desc)
    timed("collate_into_us", lambda ids: store.collate_into(ids, pb))
    timed("graph_replay_us", lambda ids: st.graph.replay())
    timed("step_us", st.step)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
