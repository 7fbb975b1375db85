"""Data-parallel path (hgin.train.train_step + hgin.dist.GradAllReducer) with world_size 2 over gloo on CPU.

Each rank holds whole graph components (the reference's batch-of-graphs unit, dataset.py:26/242) and runs
train_step on them with the CPU oracle model.  The ranks together must train exactly as one device holding
the collated batch (train.py:40-44: sqrt(mape) over every path of the batch): after the step every rank
holds the single-device gradient of the union and the union's loss value, for equal AND unequal splits of
the paths over the ranks (hgin/dist.py).
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


def _components(cfg, seeds, scales):
    from hgin.data import collate, scaled_config, synthetic_graph
    return collate([synthetic_graph(scaled_config(cfg, s, name=f"c{s}"), seed=sd) for sd, s in zip(seeds, scales)])


# rank -> (component seeds, component size factors); "unequal" gives the ranks different path counts
SPLITS = {"equal": {0: ([100], [1.0]), 1: ([101], [1.0])},
          "unequal": {0: ([100, 102], [1.0, 0.5]), 1: ([101], [1.5])}}


def _worker(rank, world, port, outdir, split):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from hgin.data import CONFIGS
    from hgin.dist import GradAllReducer
    from hgin.train import train_step
    cfg = CONFIGS["cfg1"]
    model = _model(cfg)
    opt = torch.optim.SGD(model.parameters(), lr=0.0)
    seeds, scales = SPLITS[split][rank]
    lv = train_step(model, opt, _components(cfg, seeds, scales), reducer=GradAllReducer(model.parameters()))
    torch.save({"loss": lv, "grads": {n: p.grad for n, p in model.named_parameters()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("split", sorted(SPLITS))
def test_two_ranks_train_as_one_batch(split):
    from hgin.data import CONFIGS
    from oracle.pyg_cpu import mape
    torch.set_num_threads(1)
    cfg = CONFIGS["cfg1"]
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _free_port(), d, split), nprocs=2, join=True)
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    seeds = SPLITS[split][0][0] + SPLITS[split][1][0]
    scales = SPLITS[split][0][1] + SPLITS[split][1][1]
    union = _components(cfg, seeds, scales)
    model = _model(cfg)
    out = model(union.x_dict(), union.edge_index_dict(), union.batch["path"])
    lv = mape(out, union.y.reshape(-1, 1))
    torch.sqrt(lv).backward()
    lv = float(lv.detach())
    assert abs(float(r0["loss"]) - lv) <= 1e-5 * lv
    assert torch.equal(r0["loss"], r1["loss"])
    for n, p in model.named_parameters():
        g0, g1 = r0["grads"][n], r1["grads"][n]
        assert (g0 is None) == (p.grad is None), n                     # dead relations stay None on every rank
        if g0 is None:
            assert g1 is None
            continue
        assert torch.equal(g0, g1), n                                   # ranks agree bitwise
        err = float((g0.double() - p.grad.double()).norm())
        assert err <= 1e-5 * float(p.grad.double().norm()) + 1e-9, (n, err)


def test_single_rank_reducer_is_identity_semantics():
    """world 1 (no process group): the reducer path equals the plain sqrt(mape) backward."""
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.dist import GradAllReducer
    from hgin.train import train_step
    from oracle.pyg_cpu import mape
    cfg = CONFIGS["cfg1"]
    g = synthetic_graph(cfg, seed=7)
    m1, m2 = _model(cfg), _model(cfg)
    lv = train_step(m1, torch.optim.SGD(m1.parameters(), lr=0.0), g, reducer=GradAllReducer(m1.parameters()))
    out = m2(g.x_dict(), g.edge_index_dict(), g.batch["path"])
    lv2 = mape(out, g.y.reshape(-1, 1))
    torch.sqrt(lv2).backward()
    assert abs(float(lv) - float(lv2.detach())) <= 1e-6 * float(lv2.detach())
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        assert (p.grad is None) == (q.grad is None), n
        if p.grad is not None:
            err = float((p.grad.double() - q.grad.double()).norm())
            assert err <= 1e-5 * float(q.grad.double().norm()) + 1e-9, (n, err)
