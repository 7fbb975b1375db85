"""Where the real loop's fused and general paths part ways over many Adam steps (26.9126 vs 26.8914 after
205 batches).  Same store, same batch order, same initial parameters; four trajectories:

  fused_step          SmallBatchStep, Adam folded into its final kernel (bench extras.batches main figure)
  general_foreach     CapturedTrainStep + Adam(foreach)          (bench extras.batches general_path)
  general_fusedadam   CapturedTrainStep + Adam(fused=True)       (fused Adam: the fused step before round 5)
  oracle              oracle.pyg_cpu on the host-collated batches, torch CPU Adam

Prints one JSON line: the per-step relative loss differences of each GPU trajectory against the oracle at a few step
counts, and the fused-vs-general difference with the optimizer held equal.

    python tools/sb_drift.py [--steps 205]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from hgin import HetroGIN
    from hgin.data import CONFIGS, scaled_config, synthetic_graph
    from hgin.graphs import CapturedTrainStep
    from hgin.smallbatch import SmallBatchStep
    from hgin.store import GraphStore
    from oracle.pyg_cpu import OracleHetroGIN, train_step as oracle_step
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=205)
    ap.add_argument("--graphs", type=int, default=256)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(0)
    graphs = [synthetic_graph(scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=i)
              for i in range(args.graphs)]
    store = GraphStore.build(graphs, device=dev, normalize=True)
    warm = [rng.choice(args.graphs, 8, replace=False).tolist()]
    order = [rng.choice(args.graphs, 8, replace=False).tolist() for _ in range(args.steps)]
    ic = lambda: {"link": base.f_link, "path": base.f_path, "node": base.f_node}   # noqa: E731

    def model():
        torch.manual_seed(1997)
        return HetroGIN(**base.model_kwargs(ic())).to(dev)

    traj = {}
    for name in ("fused_step", "general_foreach", "general_fusedadam"):
        m = model()
        opt = torch.optim.Adam(m.parameters(), lr=1e-3, capturable=True,
                               **({"fused": True} if name.endswith("fusedadam") else {}))
        cls = SmallBatchStep if name.startswith("fused") else CapturedTrainStep
        st = cls(m, opt, store, 8, warmup_ids=warm, warmup=1)   # one warm-up Adam step on warm[0]
        traj[name] = [float(st.step(ids)) for ids in order]
        del st, m, opt
        torch.cuda.empty_cache()
    torch.manual_seed(1997)
    ref = OracleHetroGIN(**base.model_kwargs(ic()))
    opt = torch.optim.Adam(ref.parameters(), lr=1e-3)

    def host(ids):
        b = store.collate(ids).to("cpu")
        return oracle_step(ref, opt, b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y)
    host(warm[0])
    traj["oracle"] = [float(host(ids)) for ids in order]
    at = [k for k in (1, 5, 10, 20, 50, 100, 150, 200, args.steps) if k <= args.steps]
    o = np.array(traj["oracle"])
    rel = lambda a, b: [float(abs(a[k - 1] - b[k - 1]) / abs(b[k - 1])) for k in at]   # noqa: E731
    out = {"steps": args.steps, "at_step": at,
           "vs_oracle": {k: rel(np.array(v), o) for k, v in traj.items() if k != "oracle"},
           "fused_vs_general_same_adam": rel(np.array(traj["fused_step"]), np.array(traj["general_fusedadam"])),
           "general_foreach_vs_fusedadam": rel(np.array(traj["general_foreach"]), np.array(traj["general_fusedadam"])),
           "final_loss": {k: v[-1] for k, v in traj.items()}}
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
