"""What one rank of an N-GPU cfg4 run computes, timed alone on one GPU: rank 0's share of the 8 components
(rank_components(cfg4, 0, N)) trained with the bench's eager step, N = 1, 2, 4, 8.  t(1) / t(N) bounds the strong
scaling of `bench.py --gpus N` from above (the N-rank run adds one RCCL all-reduce of ~1.4 MB per step).

    python tools/rank_share_bench.py [cfg4|cfg5] [steps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gnn-link-prediction_amd")]

import dataclasses  # noqa: E402

import torch  # noqa: E402

from hgin import HetroGIN  # noqa: E402
from hgin.data import CONFIGS, rank_components  # noqa: E402
from hgin.train import train_step  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "cfg4"
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
    cfg = CONFIGS[name]
    if cfg.components == 1:
        cfg = dataclasses.replace(cfg, components=8)
    base = None
    for W in (1, 2, 4, 8):
        g, ids = rank_components(cfg, 0, W, device="cuda", n_components=8)
        torch.manual_seed(1997)
        model = HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).cuda()
        opt = torch.optim.Adam(model.parameters(), lr=1e-3, foreach=True)
        for _ in range(3):
            train_step(model, opt, g)
        torch.cuda.synchronize()
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(steps + 1)]
        ev[0].record()
        for i in range(steps):
            train_step(model, opt, g)
            ev[i + 1].record()
        torch.cuda.synchronize()
        ts = sorted(ev[i].elapsed_time(ev[i + 1]) for i in range(steps))
        med = ts[len(ts) // 2]
        base = base or med
        print(f"{name} N={W}: rank 0 holds components {ids}: {med:8.3f} ms/step (median of {steps}); "
              f"t(1)/t(N) = {base / med:5.2f}", flush=True)
        del g, model, opt
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
