"""The multi-rank HIP path (hgin.train.train_step + hgin.dist.GradAllReducer over libhgin.so) with two ranks.

The box has one GPU, so both ranks share it and talk over gloo (RCCL refuses two ranks on one device); the
step's arithmetic is the RCCL run's.  Each rank holds half the components of a cfg2-schema graph
(hgin.data.rank_components); after one step both ranks must hold the single-device gradient of the union
and its loss value (hgin/dist.py), within fp32 summation-order tolerance (the GEMM weight-gradient
reductions run over different row counts).

The connected-graph variant (hgin/partition.py: destination-range rows per rank, per-layer all-gather of
source embeddings, reduce-scatter of their gradients) runs the same check on one connected graph.
"""
import os
import socket
import tempfile

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from conftest import fixture_model_kwargs  # noqa: F401  (puts the repo on sys.path for spawned ranks)

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _cfg(feat):
    import dataclasses

    from hgin.data import CONFIGS, scaled_config
    return dataclasses.replace(scaled_config(CONFIGS["cfg2"], 0.04, name="cfg2-small"), feat_dtype=feat)


def _model(cfg):
    from hgin import HetroGIN
    torch.manual_seed(1997)
    return HetroGIN(**cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})).to("cuda")


def _worker(rank, world, port, outdir, feat):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hgin.data import rank_components
    from hgin.dist import GradAllReducer
    from hgin.train import train_step
    cfg = _cfg(feat)
    graph, _ = rank_components(cfg, rank, world, device="cuda", n_components=4)
    model = _model(cfg)
    lv = train_step(model, torch.optim.SGD(model.parameters(), lr=0.0), graph,
                    reducer=GradAllReducer(model.parameters()))
    torch.save({"loss": lv.cpu(), "grads": {n: (p.grad.cpu() if p.grad is not None else None)
                                             for n, p in model.named_parameters()}},
               os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("feat", ["f32", "bf16"])
def test_two_ranks_equal_single_device(feat):
    from hgin.data import rank_components
    from hgin.train import mape
    cfg = _cfg(feat)
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_worker, args=(r, 2, port, d, feat)) for r in range(2)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
            assert p.exitcode == 0, p.exitcode
        r0 = torch.load(os.path.join(d, "rank0.pt"), weights_only=True)
        r1 = torch.load(os.path.join(d, "rank1.pt"), weights_only=True)
    union, _ = rank_components(cfg, 0, 1, device="cuda", n_components=4)
    model = _model(cfg)
    _, lv = model.forward_loss(union.x_dict(), union.edge_index_dict(), union.batch["path"], union.y)
    torch.sqrt(lv).backward()
    lv = float(lv)
    assert torch.equal(r0["loss"], r1["loss"])
    assert abs(float(r0["loss"]) - lv) <= 1e-5 * lv
    # bf16 storage: the ranks' activations / gradient tensors round differently per row block only through
    # the GEMM reduction splits; the bound stays at the fp32-accumulation level
    tol = 1e-4 if feat == "f32" else 5e-3
    g_scale = max(float(p.grad.double().norm()) for p in model.parameters() if p.grad is not None)
    for n, p in model.named_parameters():
        g0, g1 = r0["grads"][n], r1["grads"][n]
        assert (g0 is None) == (p.grad is None), n
        if g0 is None:
            continue
        assert torch.equal(g0, g1), n
        err = float((g0.double() - p.grad.double().cpu()).norm())
        assert err <= tol * float(p.grad.double().norm()) + 1e-6 * g_scale, (n, err)


def _part_worker(rank, world, port, outdir, feat):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from hgin.data import synthetic_graph
    from hgin.partition import DstRangePartition, forward_loss, train_step
    cfg = _cfg(feat)
    g = synthetic_graph(cfg, seed=3, device="cuda")
    res = {}
    for overlap in (True, False):    # the overlapped schedule (default) and the serial one: bitwise equal
        part = DstRangePartition({t: g.num_nodes(t) for t in g.x}, overlap=overlap)
        local = part.local_graph(g)
        model = _model(cfg)
        with torch.no_grad():
            out, _ = forward_loss(model, part, local)
        lv = train_step(model, torch.optim.SGD(model.parameters(), lr=0.0), part, local)
        res[overlap] = {"loss": lv.cpu(), "out": out.float().cpu(), "rows": part.rows("path"),
                        "grads": {n: (p.grad.cpu() if p.grad is not None else None)
                                  for n, p in model.named_parameters()}}
    a, b = res[True], res[False]
    assert torch.equal(a["out"], b["out"]) and torch.equal(a["loss"], b["loss"])
    for n, ga in a["grads"].items():
        gb = b["grads"][n]
        assert (ga is None) == (gb is None) and (ga is None or torch.equal(ga, gb)), n
    torch.save(a, os.path.join(outdir, f"rank{rank}.pt"))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("feat,world", [("f32", 2), ("bf16", 2), ("f32", 3)])
def test_dst_range_partition_equals_single_device(feat, world):
    """The ranks each own a block of every node type of ONE connected graph (world 3: short, padded last blocks):
    the forward output rows are bit-identical to the single-device forward (same edges per destination row, same
    order), the loss and the gradients equal the single-device ones within fp32 summation-order tolerance."""
    from hgin.data import synthetic_graph
    cfg = _cfg(feat)
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        port = _free_port()
        procs = [ctx.Process(target=_part_worker, args=(r, world, port, d, feat)) for r in range(world)]
        for p in procs:
            p.start()
        for p in procs:
            p.join(timeout=240)
            assert p.exitcode == 0, p.exitcode
        rs = [torch.load(os.path.join(d, f"rank{r}.pt"), weights_only=True) for r in range(world)]
    g = synthetic_graph(cfg, seed=3, device="cuda")
    model = _model(cfg)
    out, lv = model.forward_loss(g.x_dict(), g.edge_index_dict(), g.batch["path"], g.y)
    torch.sqrt(lv).backward()
    lv = float(lv)
    full_out = out.detach().float().cpu()
    for r in rs:
        lo, hi = r["rows"]
        assert torch.equal(r["out"], full_out[lo:hi])
    for r in rs[1:]:
        assert torch.equal(rs[0]["loss"], r["loss"])
    assert abs(float(rs[0]["loss"]) - lv) <= 1e-5 * lv
    tol = 1e-4 if feat == "f32" else 5e-3
    g_scale = max(float(p.grad.double().norm()) for p in model.parameters() if p.grad is not None)
    for n, p in model.named_parameters():
        g0 = rs[0]["grads"][n]
        assert (g0 is None) == (p.grad is None), n
        if g0 is None:
            continue
        for r in rs[1:]:
            assert torch.equal(g0, r["grads"][n]), n
        err = float((g0.double() - p.grad.double().cpu()).norm())
        assert err <= tol * float(p.grad.double().norm()) + 1e-6 * g_scale, (n, err)


def _rccl_worker(outdir):
    """World size 1 over RCCL: the process group comes up before any other GPU work of this child; then the
    component-DP step (GradAllReducer's all-reduce) and the dst-range partition's all-gather / reduce-scatter
    (overlapped on the communication stream) run their collectives on the "nccl" (= RCCL) backend."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=os.environ["HGIN_TEST_PORT"])
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1)
    assert dist.get_backend() == "nccl"
    from hgin.data import synthetic_graph
    from hgin.dist import GradAllReducer
    from hgin.partition import DstRangePartition
    from hgin.partition import train_step as part_step
    from hgin.train import train_step
    cfg = _cfg("f32")
    g = synthetic_graph(cfg, seed=3, device="cuda")
    res = {}
    for mode in ("plain", "reducer", "partition"):
        model = _model(cfg)
        opt = torch.optim.SGD(model.parameters(), lr=0.0)
        if mode == "plain":
            lv = train_step(model, opt, g)
        elif mode == "reducer":
            red = GradAllReducer(model.parameters())
            lv = train_step(model, opt, g, reducer=red)
            red.check()
        else:
            part = DstRangePartition({t: g.num_nodes(t) for t in g.x})
            lv = part_step(model, opt, part, part.local_graph(g))
        torch.cuda.synchronize()
        res[mode] = {"loss": lv.cpu(), "grads": {n: (p.grad.cpu() if p.grad is not None else None)
                                                 for n, p in model.named_parameters()}}
    torch.save(res, os.path.join(outdir, "rccl.pt"))
    dist.destroy_process_group()


def test_rccl_world1_collectives_equal_plain_step():
    """The "nccl" backend on the hardware: one train_step through GradAllReducer (one RCCL all-reduce of
    [grads | presence | S | m]) and one through the dst-range partition (RCCL all-gathers / reduce-scatters)
    equal the reducer-free step: loss within 1e-6, gradients within 1e-5 of their norm (the reducer
    back-propagates S = m * mape and rescales, the plain step sqrt(mape): different roundings of the same
    gradient)."""
    with tempfile.TemporaryDirectory() as d:
        ctx = mp.get_context("spawn")
        os.environ["HGIN_TEST_PORT"] = str(_free_port())
        p = ctx.Process(target=_rccl_worker, args=(d,))
        p.start()
        p.join(timeout=240)
        assert p.exitcode == 0, p.exitcode
        res = torch.load(os.path.join(d, "rccl.pt"), weights_only=True)
    base = res["plain"]
    for mode in ("reducer", "partition"):
        r = res[mode]
        assert abs(float(r["loss"]) - float(base["loss"])) <= 1e-6 * float(base["loss"]), mode
        for n, g0 in base["grads"].items():
            g1 = r["grads"][n]
            assert (g0 is None) == (g1 is None), (mode, n)
            if g0 is not None:
                err = float((g1.double() - g0.double()).norm())
                assert err <= 1e-5 * float(g0.double().norm()) + 1e-9, (mode, n, err)
