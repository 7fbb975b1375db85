"""The fused small-batch step alone (bench.py extras.batches' main figure), a rocprofv3 target:
    rocprofv3 --kernel-trace --stats -- python3 tools/sb_prof.py [--steps 200] [--gat]
(tools/sb_busy.py turns the kernel trace into kernel-busy vs wall time per batch)
Prints the ms per batch (HIP events)."""
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
    from hgin.smallbatch import SmallBatchStep
    from hgin.store import GraphStore
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--model", default="{}", help='HetroGIN keyword overrides as JSON, e.g. {"mlp_bn": true}')
    ap.add_argument("--eval", type=int, default=0, help="> 0: SmallBatchEval at this batch size instead")
    ap.add_argument("--gat", action="store_true", help="HetroGAT (config.json MODEL GAT: HEADS 16, hidden 8, 1 layer)")
    ap.add_argument("--n-parts", type=int, default=None, help="SmallBatchStep n_parts override (A/B)")
    args = ap.parse_args()
    dev = torch.device("cuda")
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(0)
    graphs = [synthetic_graph(scaled_config(base, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=i)
              for i in range(256)]
    store = GraphStore.build(graphs, device=dev, normalize=True)
    order = [rng.choice(256, 8, replace=False).tolist() for _ in range(5 + args.steps)]
    torch.manual_seed(1997)
    kw = dict(base.model_kwargs({"link": base.f_link, "path": base.f_path, "node": base.f_node}),
              **json.loads(args.model))
    if args.gat:
        from hgin import HetroGAT
        kw.update(heads=16, node_embedding_size=8, message_passing_layers=1)
        model = HetroGAT(**kw).to(dev)
    else:
        model = HetroGIN(**kw).to(dev)
    if args.eval:
        from hgin.smallbatch import SmallBatchEval
        model.eval()
        order = [ids[:args.eval] for ids in order]
        st = SmallBatchEval(model, store, args.eval, warmup_ids=order[:5], warmup=5)
    else:
        opt = torch.optim.Adam(lr=1e-3, params=model.parameters())
        st = SmallBatchStep(model, opt, store, 8, warmup_ids=order[:5], warmup=5, n_parts=args.n_parts)
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for ids in order[5:]:
        st.step(ids)
    e.record()
    torch.cuda.synchronize()
    print(json.dumps({"model": json.loads(args.model), "gat": args.gat, "n_parts": st.n_parts,
                      "ms_per_batch": s.elapsed_time(e) / args.steps}), flush=True)


if __name__ == "__main__":
    main()
