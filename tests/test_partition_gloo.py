"""Connected-graph variant (hgin/partition.py): a 1D destination-range partition trained over
gloo on CPU with world sizes 2 and 3 (3 leaves short last row blocks: the padded all-gather / reduce-scatter).

The layers run on the CPU oracle model (the HIP kernels need the GPU; tests/test_gpu_dist.py runs the same
partition through libhgin.so).  What is checked here is the partition itself: the per-rank edge sets, the
all-gather of source embeddings, the reduce-scatter adjoint in the backward and the loss / gradient
combination.  After one step every rank must hold the single-device gradient of the whole graph and its loss.
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


def _cfg(n_path=301):
    import dataclasses

    from hgin.data import CONFIGS, scaled_config
    # cfg2 schema (divided / bl features: no column slicing), odd counts so world 3 pads its last blocks
    c = scaled_config(CONFIGS["cfg2"], 0.0005, name="cfg2-tiny")
    return dataclasses.replace(c, n_path=n_path, n_link=151, n_node=52, f_path=16, f_link=12, f_node=8, hidden=16,
                               layers=3)


def _graph(n_path=301):
    from hgin.data import synthetic_graph
    return synthetic_graph(_cfg(n_path), seed=5)


def _model():
    from oracle.pyg_cpu import OracleHetroGIN
    cfg = _cfg()
    torch.manual_seed(1997)
    return OracleHetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}))


def _worker(rank, world, port, outdir, n_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.set_num_threads(1)
    from hgin.partition import DstRangePartition, train_step
    g = _graph(n_path)
    part = DstRangePartition({t: g.num_nodes(t) for t in g.x})
    local = part.local_graph(g)
    model = _model()
    lv = train_step(model, torch.optim.SGD(model.parameters(), lr=0.0), part, local)
    torch.save({"loss": lv, "grads": {n: p.grad for n, p in model.named_parameters()},
                "edges": {"__".join(r): e for r, e in local.edge_index.items()},
                "rows": {t: part.rows(t) for t in g.x}}, os.path.join(outdir, f"rank{rank}.pt"))
    dist.destroy_process_group()


@pytest.mark.parametrize("world,n_path", [(2, 301), (3, 301), (3, 4)])
def test_dst_range_partition_trains_as_one_graph(world, n_path):
    """(3, 4): chunks of 2 paths, so rank 2 owns none — it still runs the (empty) readout, so every rank sends
    the same gradient layout and holds every readout gradient (zero contribution from it)."""
    from oracle.pyg_cpu import mape
    torch.set_num_threads(1)
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _free_port(), d, n_path), nprocs=world, join=True)
        rs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    g = _graph(n_path)
    # the ranks' edge sets: every edge exactly once, at the rank owning its destination, in the original order
    for rel, e in g.edge_index.items():
        key = "__".join(rel)
        parts = []
        for r in rs:
            lo, hi = r["rows"][rel[2]]
            el = r["edges"][key].clone()
            assert el.numel() == 0 or (int(el[1].min()) >= 0 and int(el[1].max()) < hi - lo)
            el[1] += lo
            parts.append(el)
        owner = torch.cat(parts, 1)
        expect = torch.cat([e[:, (e[1] >= r["rows"][rel[2]][0]) & (e[1] < r["rows"][rel[2]][1])] for r in rs], 1)
        assert torch.equal(owner, expect), key
        assert owner.size(1) == e.size(1), key
    model = _model()
    out = model(g.x_dict(), g.edge_index_dict(), g.batch["path"])
    lv = mape(out, g.y.reshape(-1, 1))
    torch.sqrt(lv).backward()
    lv = float(lv.detach())
    for r in rs:
        assert torch.equal(r["loss"], rs[0]["loss"])
        assert abs(float(r["loss"]) - lv) <= 1e-5 * lv
    for n, p in model.named_parameters():
        g0 = rs[0]["grads"][n]
        assert (g0 is None) == (p.grad is None), n
        if g0 is None:
            continue
        for r in rs[1:]:
            assert torch.equal(r["grads"][n], g0), n      # one all-reduce: every rank holds the same sum
        err = float((g0.double() - p.grad.double()).norm())
        # 4 paths: the scalar slope / eps gradients are short sums of cancelling terms, split differently over
        # the ranks than on one device (fp32 summation order): 1e-4 of the norm there, 1e-5 otherwise
        tol = 1e-5 if n_path > 100 else 1e-4
        assert err <= tol * float(p.grad.double().norm()) + 1e-9, (n, err)


def test_partition_rows_and_exchange_bytes():
    from hgin.partition import DstRangePartition
    n = {"path": 10, "link": 7, "node": 0}
    rows = [DstRangePartition(n, rank=r, world=3).rows("path") for r in range(3)]
    assert rows == [(0, 4), (4, 8), (8, 10)]
    assert [DstRangePartition(n, rank=r, world=3).rows("link") for r in range(3)] == [(0, 3), (3, 6), (6, 7)]
    assert DstRangePartition(n, rank=2, world=3).rows("node") == (0, 0)
    p = DstRangePartition(n, rank=0, world=3)
    assert p.exchange_bytes({"path": 8, "link": 4}, 4) == 2 * (4 * 8 + 3 * 4) * 4
    with pytest.raises(ValueError):
        DstRangePartition(n, rank=3, world=3)


def test_single_rank_partition_is_the_plain_step():
    """world 1 (no process group): the partition is the whole graph and the step is the plain sqrt(MAPE) step."""
    from hgin.partition import DstRangePartition, train_step
    from oracle.pyg_cpu import mape
    torch.set_num_threads(1)
    g = _graph()
    part = DstRangePartition({t: g.num_nodes(t) for t in g.x})
    assert part.world == 1
    m1, m2 = _model(), _model()
    lv = train_step(m1, torch.optim.SGD(m1.parameters(), lr=0.0), part, part.local_graph(g))
    out = m2(g.x_dict(), g.edge_index_dict(), g.batch["path"])
    lv2 = mape(out, g.y.reshape(-1, 1))
    torch.sqrt(lv2).backward()
    assert abs(float(lv) - float(lv2.detach())) <= 1e-6 * float(lv2.detach())
    for (n, p), (_, q) in zip(m1.named_parameters(), m2.named_parameters()):
        if p.grad is not None:
            err = float((p.grad.double() - q.grad.double()).norm())
            assert err <= 1e-5 * float(q.grad.double().norm()) + 1e-9, (n, err)
