"""Data-parallel path (hgin.dist.GradAllReducer) with world_size 2 over gloo on CPU.

Each rank holds one whole graph component (the reference's batch-of-graphs unit, dataset.py:26/242) and
computes gradients with the CPU oracle; after the all-reduce every rank must hold
  (a) exactly the mean of the per-rank gradients, and
  (b) for the (linear-in-paths) MAPE loss, the gradient of the collated two-component batch.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import fixture_model_kwargs  # noqa: F401  (puts the repo on sys.path for spawned ranks)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _model(cfg):
    from oracle.pyg_cpu import OracleHetroGIN
    torch.manual_seed(1997)
    return OracleHetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}))


def _grads(model, graph, sqrt_loss):
    from oracle.pyg_cpu import mape
    model.zero_grad(set_to_none=True)
    out = model(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"])
    lv = mape(out, graph.y.reshape(-1, 1))
    (torch.sqrt(lv) if sqrt_loss else lv).backward()
    return {n: (p.grad.clone() if p.grad is not None else None) for n, p in model.named_parameters()}


def _worker(rank, world, port, outdir, sqrt_loss):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.dist import GradAllReducer
    cfg = CONFIGS["cfg1"]
    model = _model(cfg)
    _grads(model, synthetic_graph(cfg, seed=100 + rank), sqrt_loss)
    GradAllReducer(model.parameters()).sync()
    torch.save({n: p.grad for n, p in model.named_parameters()}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("sqrt_loss", [True, False])
def test_grad_allreduce_two_ranks(sqrt_loss):
    from hgin.data import CONFIGS, collate, synthetic_graph
    torch.set_num_threads(1)
    cfg = CONFIGS["cfg1"]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, sqrt_loss), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    per_rank = [_grads(_model(cfg), synthetic_graph(cfg, seed=100 + r), sqrt_loss) for r in range(2)]
    union = _grads(_model(cfg), collate([synthetic_graph(cfg, seed=100), synthetic_graph(cfg, seed=101)]),
                   sqrt_loss)
    for n in r0:
        assert (r0[n] is None) == (per_rank[0][n] is None), n       # dead relations stay None on every rank
        if r0[n] is None:
            assert r1[n] is None
            continue
        assert torch.equal(r0[n], r1[n]), n                           # ranks agree bitwise
        mean = (per_rank[0][n] + per_rank[1][n]) * 0.5
        assert torch.allclose(r0[n], mean, rtol=1e-6, atol=1e-9), n
        if not sqrt_loss:   # MAPE is a mean over paths: equal-size components -> DP grad == batch grad
            assert torch.allclose(r0[n], union[n], rtol=1e-4, atol=1e-7), n
