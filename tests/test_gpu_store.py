"""§8 F1/F2 on the GPU: device batch collation out of an HBM-resident GraphStore.

The checker is oracle/collate_np.py (an independent numpy restatement of PyG's Batch.from_data_list,
dataset.py:239-244) on the host plus the C oracle's stable CSR build (oracle/hgin_oracle.c) of the collated
edge_index — every collated array must be bit-identical, including the CSR / CSC the store assembles without
sorting.
"""
import dataclasses

import numpy as np
import pytest
import torch

from hgin import HetroGIN, ops
from hgin.data import CONFIGS, REL_PN, HeteroGraph, scaled_config, synthetic_graph
from hgin.store import GraphStore, normalize_reference
from oracle import c_oracle as co
from oracle import collate_np


def oracle_collate(graphs) -> HeteroGraph:
    c = collate_np.collate([collate_np.from_graph(g) for g in graphs])
    return HeteroGraph({t: torch.from_numpy(v) for t, v in c["x"].items()},
                       {r: torch.from_numpy(e) for r, e in c["edge_index"].items()}, torch.from_numpy(c["y"]),
                       {t: torch.from_numpy(b) for t, b in c["batch"].items()})

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graphs(n, seed=0, empty_rel_at=None):
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        cfg = scaled_config(base, float(rng.uniform(0.05, 0.4)), name=f"g{i}")
        cfg = dataclasses.replace(cfg, e_pn=max(1, cfg.e_ln))
        g = synthetic_graph(cfg, seed=seed * 1000 + i)
        if empty_rel_at is not None and i == empty_rel_at:
            g.edge_index[REL_PN] = torch.empty(2, 0, dtype=torch.long)
        out.append(g)
    return out


def _check_batch(b: HeteroGraph, ref: HeteroGraph):
    for t in ref.x:
        assert torch.equal(b.x[t].cpu(), ref.x[t]), t
        assert torch.equal(b.batch[t].cpu(), ref.batch[t]), t
    assert torch.equal(b.y.cpu(), ref.y)
    for r, e in ref.edge_index.items():
        assert torch.equal(b.edge_index[r].cpu(), e), r
        n_s, n_d = ref.x[r[0]].shape[0], ref.x[r[2]].shape[0]
        rg = ops.relation_graph(b.edge_index[r], n_s, n_d)
        for key_row, c, n_rows, n_cols in ((1, rg._csr, n_d, n_s), (0, rg._csc, n_s, n_d)):
            assert c is not None, "collate must attach prebuilt CSR / CSC"
            rp, col, perm, st = co.csr_build(e.numpy(), key_row, n_rows, n_cols)
            assert st == 0
            assert np.array_equal(c.rowptr.cpu().numpy(), rp), (r, key_row)
            assert np.array_equal(c.col.cpu().numpy(), col), (r, key_row)
            assert np.array_equal(c.perm.cpu().numpy(), perm), (r, key_row)


@pytest.mark.parametrize("ids", [[0], [3, 1, 4, 1, 5, 9, 2, 6], list(range(12)), [11, 0, 7]])
def test_collate_bit_exact(ids):
    graphs = _graphs(12, seed=1, empty_rel_at=4)
    store = GraphStore.build(graphs, device=DEV)
    b = store.collate(ids)
    torch.cuda.synchronize()
    _check_batch(b, oracle_collate([graphs[i] for i in ids]))


def test_collate_store_csr_matches_fresh_build():
    graphs = _graphs(6, seed=2)
    store = GraphStore.build(graphs, device=DEV)
    big = oracle_collate(graphs)
    for r, e in big.edge_index.items():
        n_s, n_d = big.x[r[0]].shape[0], big.x[r[2]].shape[0]
        rp, col, perm, _ = co.csr_build(e.numpy(), 1, n_d, n_s)
        assert np.array_equal(store.csr[r].rowptr.cpu().numpy(), rp)
        assert np.array_equal(store.csr[r].perm.cpu().numpy(), perm)


def test_collate_model_output_identical():
    graphs = _graphs(10, seed=3)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    ids = [7, 2, 9, 0, 4, 4, 1, 8]
    b = store.collate(ids)
    ref = oracle_collate([graphs[i] for i in ids]).to(DEV)     # fresh tensors -> CSR / CSC built by sorting
    out_b = model(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    out_r = model(ref.x_dict(), ref.edge_index_dict(), ref.batch["path"])
    assert torch.equal(out_b, out_r)
    g_b = torch.autograd.grad(out_b.sum(), list(model.parameters()), allow_unused=True)
    g_r = torch.autograd.grad(out_r.sum(), list(model.parameters()), allow_unused=True)
    for a, c in zip(g_b, g_r):
        assert (a is None) == (c is None)
        if a is not None:
            assert torch.equal(a, c)


def test_save_load_roundtrip(tmp_path):
    graphs = _graphs(5, seed=4)
    store = GraphStore.build(graphs, device=DEV, normalize=True)
    path = str(tmp_path / "store.pt")
    store.save(path)
    loaded = GraphStore.load(path, device=DEV)
    ids = [4, 0, 2]
    a, b = store.collate(ids), loaded.collate(ids)
    torch.cuda.synchronize()
    for t in a.x:
        assert torch.equal(a.x[t], b.x[t])
    for r in a.edge_index:
        assert torch.equal(a.edge_index[r], b.edge_index[r])
    # normalisation applied once at build, exactly as dataset.py:33-58 does per sample
    ref = oracle_collate([HeteroGraph(normalize_reference(g.x), g.edge_index, g.y, g.batch) for g in [graphs[i] for i in ids]])
    _check_batch(b, ref)


def test_collate_rejects_bad_ids():
    store = GraphStore.build(_graphs(3, seed=5), device=DEV)
    with pytest.raises(IndexError):
        store.collate([0, 3])
    with pytest.raises(ValueError):
        store.collate([])


def test_padded_batch_matches_exact_batch():
    """collate_into a static padded batch: valid rows equal the exact collation, padding rows isolated, and
    the fused loss / gradients over it equal the exact batch's (padding masked out)."""
    graphs = _graphs(9, seed=6)
    store = GraphStore.build(graphs, device=DEV)
    pb = store.padded_batch(4)
    ids = [3, 8, 0]
    store.collate_into(ids, pb)
    ref = store.collate(ids)
    torch.cuda.synchronize()
    assert int(pb.m_valid) == ref.y.numel()
    for t in ref.x:
        n = ref.x[t].shape[0]
        assert torch.equal(pb.x[t][:n], ref.x[t])
    for r, e in ref.edge_index.items():
        E = e.shape[1]
        assert torch.equal(pb.edge_index[r][:, :E], e)
        for c_pad, c_ref in ((pb.csr[r], ops.relation_graph(e, ref.x[r[0]].shape[0], ref.x[r[2]].shape[0])._csr),
                             (pb.csc[r], ops.relation_graph(e, ref.x[r[0]].shape[0], ref.x[r[2]].shape[0])._csc)):
            n = c_ref.rowptr.numel()
            assert torch.equal(c_pad.rowptr[:n], c_ref.rowptr)
            assert bool((c_pad.rowptr[n:] == E).all())                # padding rows: empty
            assert torch.equal(c_pad.col[:E], c_ref.col)
    cfg = CONFIGS["cfg1"]
    losses, grads = [], []
    for b in (pb, ref):
        torch.manual_seed(1997)
        model = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
        m_valid = getattr(b, "m_valid", None)
        _, lv = model.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y, m_valid)
        torch.sqrt(lv).backward()
        losses.append(float(lv))
        grads.append({n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None})
    assert abs(losses[0] - losses[1]) <= 1e-6 * abs(losses[1])
    scale = max(float(g.norm()) for g in grads[1].values())
    for n in grads[1]:
        assert float((grads[0][n] - grads[1][n]).norm()) <= 1e-5 * float(grads[1][n].norm()) + 1e-7 * scale, n


def test_captured_train_step_matches_eager():
    """hipGraph-captured padded steps vs eager exact-batch steps on the same batch sequence."""
    from hgin.graphs import CapturedTrainStep
    from hgin.train import train_step
    graphs = _graphs(12, seed=7)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    seq = [[0, 5, 9], [3, 1, 11], [7, 2, 4], [10, 6, 8], [2, 9, 0]]
    torch.manual_seed(1997)
    m1 = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3, capturable=True)
    step = CapturedTrainStep(m1, o1, store, batch_size=3, warmup_ids=seq[:3], warmup=3)
    cap_losses = [float(step.step(ids)) for ids in seq[3:]]
    torch.manual_seed(1997)
    m2 = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    for ids in seq[:3]:
        train_step(m2, o2, store.collate(ids))
    eager_losses = [float(train_step(m2, o2, store.collate(ids))) for ids in seq[3:]]
    assert np.allclose(cap_losses, eager_losses, rtol=1e-4, atol=0), (cap_losses, eager_losses)
    # the parameters' change over the 5 steps, relative to its own size (an absolute bound would be met by any
    # gradient: Adam moves a weight by at most ~lr per step)
    torch.manual_seed(1997)
    p0 = [p.detach().clone() for p in HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).parameters()]
    for (n, p1), (_, p2), q in zip(m1.named_parameters(), m2.named_parameters(), p0):
        d1, d2 = (p1.detach() - q.to(DEV)).double(), (p2.detach() - q.to(DEV)).double()
        assert float((d1 - d2).norm()) <= 5e-2 * float(d2.norm()) + 1e-7, n
    # and the gradients of the last captured replay equal an eager exact-batch backward on the same batch
    # and parameters (the replay rewrites .grad in place; Adam ran after it)
    ids = seq[-1]
    g_cap = {n: p.grad.detach().clone() for n, p in m1.named_parameters() if p.grad is not None}
    torch.manual_seed(1997)
    m3 = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    with torch.no_grad():
        for p3, p2 in zip(m3.parameters(), m2.parameters()):
            p3.copy_(p2)
    step2 = CapturedTrainStep(m3, torch.optim.Adam(m3.parameters(), lr=0.0, capturable=True), store, batch_size=3,
                              warmup_ids=[ids], warmup=1)
    step2.step(ids)
    m4 = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    with torch.no_grad():
        for p4, p2 in zip(m4.parameters(), m2.parameters()):
            p4.copy_(p2)
    b = store.collate(ids)
    _, lv = m4.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y)
    torch.sqrt(lv).backward()
    for (n, p3), (_, p4) in zip(m3.named_parameters(), m4.named_parameters()):
        assert (p3.grad is None) == (p4.grad is None), n
        if p4.grad is not None:
            err = float((p3.grad - p4.grad).double().norm())
            assert err <= 1e-5 * float(p4.grad.double().norm()) + 1e-9, (n, err)
    assert g_cap


def test_captured_train_step_global_feats_matches_eager():
    """GLOBAL_FEATS (models.py:347-352) in the captured padded step: the padding path rows carry the graph id
    batch_size (collate_into), so the per-graph [mean | max] pooling of the real graphs is the exact batch's; one
    replay's loss and gradients equal an eager exact-batch backward on the same parameters."""
    from hgin.graphs import CapturedTrainStep
    graphs = _graphs(10, seed=17)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    kw = lambda: dict(cfg.model_kwargs({"link": 7, "path": 7, "node": 3}), global_feats=True, bl_features=True)  # noqa: E731
    ids = [6, 2, 9]
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = CapturedTrainStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=4,
                             warmup_ids=[[1, 4, 7, 3], ids], warmup=2)
    lv = float(step.step(ids))
    torch.manual_seed(1997)
    m2 = HetroGIN(**kw()).to(DEV)
    b = store.collate(ids)
    _, lv2 = m2.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y)
    torch.sqrt(lv2).backward()
    assert abs(lv - float(lv2)) <= 1e-5 * abs(float(lv2)), (lv, float(lv2))
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert (p1.grad is None) == (p2.grad is None), n
        if p2.grad is not None:
            err = float((p1.grad - p2.grad).double().norm())
            assert err <= 1e-5 * float(p2.grad.double().norm()) + 1e-9, (n, err)


def test_captured_train_step_mlp_bn_matches_eager():
    """MLP_BN (models.py:303-313, training-mode BatchNorm1d in the readout) in the captured padded step: the batch
    statistics over the first m_valid rows only (models._masked_batch_norm), so one replay's loss, gradients and
    running statistics equal an eager exact-batch step's (torch's BatchNorm) on the same parameters."""
    from hgin.graphs import CapturedTrainStep
    graphs = _graphs(10, seed=29)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    kw = lambda: dict(cfg.model_kwargs({"link": 7, "path": 7, "node": 3}), mlp_bn=True)  # noqa: E731
    ids = [8, 1, 4]
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = CapturedTrainStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=4,
                             warmup_ids=[[2, 5, 7, 0]], warmup=1)
    torch.manual_seed(1997)
    m2 = HetroGIN(**kw()).to(DEV)
    with torch.no_grad():   # the warm-up and the capture moved m1's running statistics: start m2 from them
        for b1, b2 in zip(m1.buffers(), m2.buffers()):
            b2.copy_(b1)
    lv = float(step.step(ids))
    b = store.collate(ids)
    _, lv2 = m2.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y)
    torch.sqrt(lv2).backward()
    assert abs(lv - float(lv2)) <= 1e-5 * abs(float(lv2)), (lv, float(lv2))
    # (the bias of the Linear ahead of a BatchNorm has an exactly-zero gradient in exact arithmetic: both sides hold
    # rounding noise there, so the bound has an absolute part scaled by the largest gradient)
    scale = max(float(p.grad.double().norm()) for p in m2.parameters() if p.grad is not None)
    for (n, p1), (_, p2) in zip(m1.named_parameters(), m2.named_parameters()):
        assert (p1.grad is None) == (p2.grad is None), n
        if p2.grad is not None:
            err = float((p1.grad - p2.grad).double().norm())
            assert err <= 1e-5 * float(p2.grad.double().norm()) + 1e-7 * scale, (n, err)
    for (n, b1), (_, b2) in zip(m1.named_buffers(), m2.named_buffers()):
        assert torch.allclose(b1.double(), b2.double(), rtol=1e-5, atol=1e-7), n


def test_captured_train_step_with_dropout_draws_fresh_masks():
    """dropout > 0 (models.py:358-359) in the captured step: replays of the same batch at lr 0 give different losses
    (a fresh mask per replay, as eager steps draw), their mean within the spread of eager dropout steps on the exact
    batch, and finite gradients."""
    from hgin.graphs import CapturedTrainStep
    from hgin.train import train_step
    graphs = _graphs(8, seed=23)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    kw = lambda: dict(cfg.model_kwargs({"link": 7, "path": 7, "node": 3}), dropout=0.2)  # noqa: E731  (a fresh dict:
    ids = [3, 5, 0]                                                                      # HetroGIN mutates it)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = CapturedTrainStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=3,
                             warmup_ids=[ids], warmup=2)
    cap = [float(step.step(ids)) for _ in range(8)]
    assert len(set(cap)) > 1, cap
    assert all(p.grad is None or bool(torch.isfinite(p.grad).all()) for p in m1.parameters())
    torch.manual_seed(1997)
    m2 = HetroGIN(**kw()).to(DEV)
    o2 = torch.optim.Adam(m2.parameters(), lr=0.0)
    eager = [float(train_step(m2, o2, store.collate(ids))) for _ in range(8)]
    lo, hi = min(eager), max(eager)
    span = hi - lo
    assert lo - 2 * span <= float(np.mean(cap)) <= hi + 2 * span, (cap, eager)


def test_store_build_normalize_equals_reference_fixture():
    """GraphStore.build(normalize=True) holds exactly the features the reference's own normalize
    (dataset.py:33-58, executed by tests/golden/make_golden_normalize.py) produces for the same collated graphs."""
    from conftest import load_fixture
    from hgin.data import CONFIGS, synthetic_graph
    from hgin.store import GraphStore
    fx = load_fixture("normalize_ref")
    graphs = [synthetic_graph(CONFIGS["cfg1"], seed=s) for s in fx["meta"]["graph_seeds"]]
    st = GraphStore.build(graphs, device="cuda", normalize=True)
    for t in ("path", "link", "node"):
        n = st.x[t].shape[0]
        assert torch.equal(st.x[t].cpu(), fx[f"out.x.{t}"][:n]), t


@pytest.mark.parametrize("mlp_bn,global_feats", [(False, False), (True, False), (False, True)])
def test_captured_eval_step_matches_eager(mlp_bn, global_feats):
    """train.py's test() loop (model.eval(), forward + MAPE per batch) as captured replays: every batch's loss and the
    predictions of its paths equal an eager no-grad forward on the exact batch (BatchNorm in eval mode reads its
    running statistics: row-independent), and the device accumulators give test()'s two averages."""
    from hgin.graphs import CapturedEvalStep
    from hgin.train import mape
    graphs = _graphs(12, seed=9)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    torch.manual_seed(1997)
    kw = dict(cfg.model_kwargs({"link": 7, "path": 7, "node": 3}), mlp_bn=mlp_bn)
    if global_feats:   # (the pooled GLOBAL_FEATS columns come with the raw-feature layout, models.py:347-352)
        kw.update(global_feats=True, bl_features=True)
    model = HetroGIN(**kw).to(DEV)
    if mlp_bn:   # non-trivial running statistics
        for m in model.modules():
            if isinstance(m, torch.nn.BatchNorm1d):
                m.running_mean.uniform_(-0.5, 0.5)
                m.running_var.uniform_(0.5, 2.0)
    model.eval()
    seq = [[4], [0, 7, 2], [11, 3, 9], [6, 1, 10], [8]]
    ev = CapturedEvalStep(model, store, batch_size=3, warmup_ids=seq[:2], warmup=2)
    losses, n_paths = [], 0
    for ids in seq:
        lv = float(ev.step(ids))
        b = store.collate(ids)
        n = int(b.y.numel())
        got = ev.out[:n].detach().clone()
        with torch.no_grad():
            out = model(b.x_dict(), b.edge_index_dict(), b.batch["path"])
            want = float(mape(out, b.y.reshape(-1, 1)))
        assert abs(lv - want) <= 1e-6 * abs(want), (ids, lv, want)
        assert torch.allclose(got.reshape(-1), out.reshape(-1), rtol=1e-6, atol=1e-6), ids
        losses.append(want)
        n_paths += n
    avg, mape_w = ev.result(n_paths)
    assert abs(avg - np.mean(losses)) <= 1e-5 * abs(np.mean(losses))
    w = sum(l * int(store.collate(ids).y.numel()) for l, ids in zip(losses, seq)) / n_paths
    assert abs(mape_w - w) <= 1e-5 * abs(w)
    model.train()
    with pytest.raises(ValueError, match="eval"):
        CapturedEvalStep(model, store, batch_size=3, warmup_ids=seq[:1])
