"""The fused small-batch train step (hgin/smallbatch.py, csrc/hgin_smallbatch.hip): the reference's real loop
(dataset.py:26, :239-244; train.py:25-44) in 3 L + 1 launches + Adam per batch.

* Against the CPU oracle (oracle/pyg_cpu.py, itself pinned bit-for-bit to the reference-executed fixtures), on the
  batch collated on the host and checked against oracle/collate_np.py (the numpy restatement of PyG's
  ``Batch.from_data_list``): loss within 1e-5 relative and every gradient within 1e-4 of its norm at L = 1, 2, 3; a
  five-step Adam trajectory within 1e-4 relative per loss (train.py:31-44 = oracle.pyg_cpu.train_step).
* Against the general path — eager exact-batch steps through the per-op HIP kernels (hgin.train.train_step): loss
  values within 1e-5 relative, the gradients within 1e-5 of their norm (the fused kernels re-associate the GEMM-shaped
  sums and apply the sqrt-MAPE scale after the reduction), parameters after several Adam steps within 1e-3 of their
  total change; bitwise run-to-run."""
import numpy as np
import pytest
import torch

from hgin import HetroGIN
from hgin.data import CONFIGS, scaled_config, synthetic_graph
from hgin.store import GraphStore

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _store(n, seed, base="cfg1", normalize=True):
    rng = np.random.default_rng(seed)
    cfg = CONFIGS[base]
    graphs = [synthetic_graph(scaled_config(cfg, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=seed * 100 + i)
              for i in range(n)]
    return GraphStore.build(graphs, device=DEV, normalize=normalize), cfg


def _model(cfg, layers=None):
    torch.manual_seed(1997)
    kw = cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})
    if layers:
        kw["message_passing_layers"] = layers
    return HetroGIN(**kw).to(DEV)


def _oracle_twin(model, cfg, layers=None):
    """OracleHetroGIN with the same constructor arguments and the HIP model's parameters (on the host)."""
    from oracle.pyg_cpu import OracleHetroGIN
    kw = cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})
    if layers:
        kw["message_passing_layers"] = layers
    ref = OracleHetroGIN(**kw)
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return ref


def _host_batch(store, ids):
    """The batch on the host, pinned to the numpy restatement of PyG's collation of the same graphs."""
    from oracle import collate_np
    b = store.collate(ids).to("cpu")
    want = collate_np.collate([collate_np.from_graph(store.collate([i]).to("cpu")) for i in ids])
    for t in b.x:
        assert torch.equal(b.x[t], torch.from_numpy(want["x"][t])), t
        assert torch.equal(b.batch[t], torch.from_numpy(want["batch"][t])), t
    for r in b.edge_index:
        assert torch.equal(b.edge_index[r], torch.from_numpy(want["edge_index"][r])), r
    assert torch.equal(b.y, torch.from_numpy(want["y"]))
    return b


@pytest.mark.parametrize("readout", ["mfma", "scalar"])
@pytest.mark.parametrize("layers", [1, 2, 3])
def test_fused_step_vs_oracle(layers, readout, monkeypatch):
    """One fused step (Adam at lr 0) against the CPU oracle's forward / sqrt-MAPE backward on the host-collated batch;
    the readout on the 32-row MFMA tiles (default) and on the 8-row scalar tiles (HGIN_SB_MFMA=0)."""
    from hgin.smallbatch import SmallBatchStep
    if readout == "scalar":
        monkeypatch.setenv("HGIN_SB_MFMA", "0")
    from oracle.pyg_cpu import mape
    store, cfg = _store(10, seed=11)
    ids = [2, 8, 5, 0]
    m1 = _model(cfg, layers)
    ref = _oracle_twin(m1, cfg, layers)
    o1 = torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True)
    step = SmallBatchStep(m1, o1, store, batch_size=5, warmup_ids=[ids], warmup=1)
    assert step.args.ro_wlds == (2 if readout == "mfma" else 1)
    lv = float(step.step(ids))
    torch.cuda.synchronize()
    b = _host_batch(store, ids)
    out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    lv_ref = mape(out, b.y.reshape(-1, 1))
    torch.sqrt(lv_ref).backward()
    assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (lv, float(lv_ref))
    for (n, p), (n2, q) in zip(m1.named_parameters(), ref.named_parameters()):
        assert n == n2
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((p.grad.detach().cpu() - want).double().norm())
        assert d <= 1e-4 * float(want.double().norm()) + 1e-9, (n, d, float(want.norm()))


@pytest.mark.parametrize("variant", ["hidden128", "global_feats", "global_feats_no_concat"])
def test_fused_step_vs_oracle_variants(variant):
    """Model variants through the fused step, against the CPU oracle as above: hidden 128 (config.json's
    EMBEDDING_SIZE widened: the k <= 128 GEMMs at their widest) and GLOBAL_FEATS (models.py:347-352: each path row
    also reads its graph's [mean | max] of the sliced path features, pooled per step from the batch's raw rows; the
    padding rows pool as a graph of their own), with and without CONCAT_PATH."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN, mape
    over = {"hidden128": dict(node_embedding_size=128),
            "global_feats": dict(global_feats=True, bl_features=True),
            "global_feats_no_concat": dict(global_feats=True, bl_features=True, concat_path=False)}[variant]
    store, cfg = _store(8, seed=19)
    ids = [1, 6, 3]
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      **over)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    ref = OracleHetroGIN(**kw())
    ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=4,
                          warmup_ids=[[0, 2]], warmup=1)
    lv = float(step.step(ids))
    torch.cuda.synchronize()
    b = _host_batch(store, ids)
    out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    lv_ref = mape(out, b.y.reshape(-1, 1))
    torch.sqrt(lv_ref).backward()
    assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (lv, float(lv_ref))
    for (n, p), (n2, q) in zip(m1.named_parameters(), ref.named_parameters()):
        assert n == n2
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((p.grad.detach().cpu() - want).double().norm())
        assert d <= 1e-4 * float(want.double().norm()) + 1e-9, (n, d, float(want.norm()))


def test_fused_trajectory_vs_oracle():
    """Five shuffled batches with Adam(lr=1e-3) (train.py:31-44): the fused step's loss trajectory against
    oracle.pyg_cpu.train_step on the host-collated batches, within 1e-4 relative per step."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import train_step as oracle_step
    store, cfg = _store(12, seed=13)
    seq = [[1, 6, 10], [4, 0, 11], [8, 3, 5], [9, 7, 2], [3, 10, 1]]
    m1 = _model(cfg)
    ref = _oracle_twin(m1, cfg)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3, capturable=True)
    step = SmallBatchStep(m1, o1, store, batch_size=3, warmup_ids=[seq[0]], warmup=1)
    o2 = torch.optim.Adam(ref.parameters(), lr=1e-3)
    hb = {tuple(ids): _host_batch(store, ids) for ids in seq}

    def oracle(ids):
        b = hb[tuple(ids)]
        return float(oracle_step(ref, o2, b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y))
    oracle(seq[0])   # the warm-up's Adam step
    for k, ids in enumerate(seq):
        got, want = float(step.step(ids)), oracle(ids)
        assert abs(got - want) <= 1e-4 * abs(want), (k, got, want)


@pytest.mark.parametrize("layers", [2, 1, 3])
def test_fused_step_gradients_and_loss_equal_general_path(layers):
    from hgin.smallbatch import SmallBatchStep
    from hgin import _lib
    store, cfg = _store(10, seed=3)
    ids = [4, 1, 7, 9]
    m1 = _model(cfg, layers)
    o1 = torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True)   # lr 0: the parameters stay put
    step = SmallBatchStep(m1, o1, store, batch_size=5, warmup_ids=[ids], warmup=1)
    with _lib.trace_launches() as tr:
        lv = float(step.step(ids))
        torch.cuda.synchronize()
    g1 = {n: p.grad.detach().clone() for n, p in m1.named_parameters()}
    m2 = _model(cfg, layers)
    b = store.collate(ids)
    _, lv2 = m2.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y)
    torch.sqrt(lv2).backward()
    assert abs(lv - float(lv2)) <= 1e-5 * abs(float(lv2)), (lv, float(lv2))
    for n, p in m2.named_parameters():
        want = p.grad if p.grad is not None else torch.zeros_like(p)
        d = float((g1[n] - want).double().norm())
        assert d <= 1e-5 * float(want.double().norm()) + 1e-9, (n, d, float(want.norm()))
    # run to run: a second replay of the same batch is bitwise identical
    step.step(ids)
    torch.cuda.synchronize()
    for n, p in m1.named_parameters():
        assert torch.equal(p.grad, g1[n]), n


def test_fused_steps_train_like_the_general_path():
    """Five shuffled batches with Adam(lr=1e-3): the same loss trajectory and parameter changes as eager steps."""
    from hgin.smallbatch import SmallBatchStep
    from hgin.train import train_step
    store, cfg = _store(12, seed=5)
    seq = [[0, 5, 9], [3, 1, 11], [7, 2, 4], [10, 6, 8], [2, 9, 0]]
    m1 = _model(cfg)
    p0 = [p.detach().clone() for p in m1.parameters()]
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3, capturable=True)
    step = SmallBatchStep(m1, o1, store, batch_size=3, warmup_ids=[seq[0]], warmup=1)
    # the warm-up ran one Adam step on seq[0]: the eager twin does the same first
    m2 = _model(cfg)
    o2 = torch.optim.Adam(m2.parameters(), lr=1e-3)
    train_step(m2, o2, store.collate(seq[0]))
    fused = [float(step.step(ids)) for ids in seq]
    eager = [float(train_step(m2, o2, store.collate(ids))) for ids in seq]
    assert np.allclose(fused, eager, rtol=1e-4, atol=0), (fused, eager)
    for (n, p1), p2, q in zip(m1.named_parameters(), m2.parameters(), p0):
        d1, d2 = (p1.detach() - q).double(), (p2.detach() - q).double()
        assert float((d1 - d2).norm()) <= 1e-3 * float(d2.norm()) + 1e-8, n


def test_supports_and_refusals():
    from hgin.smallbatch import SmallBatchStep
    cfg = CONFIGS["cfg1"]
    # (HetroGIN mutates its input_channels dict, as the reference does: a fresh one per model)
    kw = lambda **o: dict(cfg.model_kwargs({"link": 7, "path": 7, "node": 3}), **o)   # noqa: E731
    assert SmallBatchStep.supports(HetroGIN(**kw()))
    assert SmallBatchStep.supports(HetroGIN(**kw(global_feats=True, bl_features=True)))
    assert not SmallBatchStep.supports(HetroGIN(**kw(dropout=0.1)))
    assert not SmallBatchStep.supports(HetroGIN(**kw(mlp_bn=True)))
    assert SmallBatchStep.supports(HetroGIN(**kw(node_embedding_size=128)))
    assert not SmallBatchStep.supports(HetroGIN(**kw(node_embedding_size=256)))
