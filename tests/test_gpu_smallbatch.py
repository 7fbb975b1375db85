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


def _g(p):
    """A fused-step parameter's gradient; the dead convs' parameters keep .grad None, as in the reference."""
    return p.grad.detach() if p.grad is not None else torch.zeros_like(p.detach())


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
    the readout on the 32-row MFMA tiles (default) and on the 8-row scalar tiles (readout="scalar")."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import mape
    store, cfg = _store(10, seed=11)
    ids = [2, 8, 5, 0]
    m1 = _model(cfg, layers)
    ref = _oracle_twin(m1, cfg, layers)
    o1 = torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True)
    step = SmallBatchStep(m1, o1, store, batch_size=5, warmup_ids=[ids], warmup=1,
                          readout="auto" if readout == "mfma" else "scalar")
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
        assert (p.grad is None) == (q.grad is None), n   # the dead convs' parameters: no gradient on either side
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((_g(p).cpu() - want).double().norm())
        assert d <= 1e-4 * float(want.double().norm()) + 1e-9, (n, d, float(want.norm()))


@pytest.mark.parametrize("variant", ["hidden128", "hidden64", "hidden96_L3", "global_feats", "global_feats_no_concat",
                                     "mlp_bn",
                                     "mlp_bn_global_feats", "mlp_bn_3hid", "mlp_bn_global_feats_h128_L3"])
def test_fused_step_vs_oracle_variants(variant):
    """Model variants through the fused step, against the CPU oracle as above: hidden 128 (config.json's
    EMBEDDING_SIZE widened: the k <= 128 GEMMs at their widest), GLOBAL_FEATS (models.py:347-352: each path row
    also reads its graph's [mean | max] of the sliced path features, pooled per step from the batch's raw rows; the
    padding rows pool as a graph of their own) with and without CONCAT_PATH, and MLP_BN (models.py:303-313:
    training-mode BatchNorm1d over the batch's rows between each hidden Linear and the PReLU; the k_sb_bn_* launches)
    — its running statistics and num_batches_tracked against the oracle's BatchNorm after the same step too.  With
    BatchNorm the hidden Linears' biases have a zero gradient in exact arithmetic (the normalisation removes them), so
    the gradient bound adds 1e-6 of the largest gradient norm."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN, mape
    over = {"hidden128": dict(node_embedding_size=128),
            "hidden64": dict(node_embedding_size=64),   # (the MFMA tiles' k-split path: two column blocks)
            "hidden96_L3": dict(node_embedding_size=96, message_passing_layers=3),
            "global_feats": dict(global_feats=True, bl_features=True),
            "global_feats_no_concat": dict(global_feats=True, bl_features=True, concat_path=False),
            "mlp_bn": dict(mlp_bn=True),
            "mlp_bn_global_feats": dict(mlp_bn=True, global_feats=True, bl_features=True),
            "mlp_bn_3hid": dict(mlp_bn=True, mlp_layers=[64, 48, 16]),
            "mlp_bn_global_feats_h128_L3": dict(mlp_bn=True, global_feats=True, bl_features=True,
                                                node_embedding_size=128, message_passing_layers=3)}[variant]
    store, cfg = _store(8, seed=19)
    ids = [1, 6, 3]
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      **over)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=4,
                          warmup_ids=[[0, 2]], warmup=1)
    torch.cuda.synchronize()
    # the readout: MFMA tiles, their weights in LDS where they fit (2) or through the caches (4); MLP_BN's launches (3)
    assert step.args.ro_wlds in ((3,) if "mlp_bn" in variant else (4,) if variant == "hidden128" else
                                 (2, 4) if variant.startswith("hidden") else (2,))
    ref = OracleHetroGIN(**kw())   # (after the warm-up step, which advanced MLP_BN's running statistics)
    ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
    lv = float(step.step(ids))
    torch.cuda.synchronize()
    b = _host_batch(store, ids)
    out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    lv_ref = mape(out, b.y.reshape(-1, 1))
    torch.sqrt(lv_ref).backward()
    assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (lv, float(lv_ref))
    gmax = max(float(q.grad.double().norm()) for q in ref.parameters() if q.grad is not None)
    slack = 1e-6 * gmax if "mlp_bn" in variant else 1e-9
    for (n, p), (n2, q) in zip(m1.named_parameters(), ref.named_parameters()):
        assert n == n2
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((_g(p).cpu() - want).double().norm())
        assert d <= 1e-4 * float(want.double().norm()) + slack, (n, d, float(want.norm()))
    for (n, u), (n2, v) in zip(m1.named_buffers(), ref.named_buffers()):
        assert n == n2
        if v.dtype == torch.int64:
            assert torch.equal(u.cpu(), v), n
        else:
            assert torch.allclose(u.cpu(), v, rtol=1e-5, atol=1e-6), (n, float((u.cpu() - v).abs().max()))
    # bitwise run to run (fixed-order sums everywhere, BatchNorm's merges included): the same batch again
    g1 = [_g(p).clone() for p in m1.parameters()]
    assert float(step.step(ids)) == lv
    torch.cuda.synchronize()
    for g, p in zip(g1, m1.parameters()):
        assert torch.equal(g, _g(p))


def test_fused_step_vs_reference_fixture_global_bn():
    """The reference-executed fixture tests/golden/collate2_global_bn.pt (models.py run on two graphs collated
    PyG-style, GLOBAL_FEATS + MLP_BN: tests/golden/make_golden.py) through the fused step.  The two graphs are
    regenerated by the committed generator (seeds 4 and 5) and their device collation is bit-identical to the
    fixture's inputs; then one step (Adam at lr 0): the loss within 1e-5 relative, every gradient within 1e-4 of its
    norm plus 1e-6 of the largest (the BatchNorm-fed Linear biases are zero in exact arithmetic: rounding noise on
    both sides), the reference's gradient-free (dead) relations exactly zero."""
    import dataclasses

    from conftest import fixture_model_kwargs, fixture_state_dict, load_fixture
    from hgin.smallbatch import SmallBatchStep
    fx = load_fixture("collate2_global_bn")
    cfg = dataclasses.replace(CONFIGS["cfg1"], bl_features=True)
    store = GraphStore.build([synthetic_graph(cfg, seed=4), synthetic_graph(cfg, seed=5)], device=DEV,
                             normalize=False)
    b = store.collate([0, 1]).to("cpu")
    for t in ("path", "link", "node"):
        assert torch.equal(b.x[t], fx[f"in.x.{t}"]), t
    for r in fx["meta"]["relations"]:
        assert torch.equal(b.edge_index[tuple(r.split("__"))], fx[f"in.ei.{r}"]), r
    assert torch.equal(b.y, fx["in.y"]) and torch.equal(b.batch["path"], fx["in.batch"])
    model = HetroGIN(**fixture_model_kwargs(fx))
    model.load_state_dict(fixture_state_dict(fx))
    model = model.to(DEV)
    step = SmallBatchStep(model, torch.optim.Adam(model.parameters(), lr=0.0, capturable=True), store, batch_size=2,
                          warmup_ids=[[1, 0]], warmup=1)
    assert step.args.ro_wlds == 3 and step.args.pool_w == 8
    lv = float(step.step([0, 1]))
    torch.cuda.synchronize()
    want = float(fx["loss_value"])
    assert abs(lv - want) <= 1e-5 * abs(want), (lv, want)
    no_grad = set(fx["meta"]["no_grad_params"])
    g_scale = max(float(fx["grad." + n].double().norm()) for n, _ in model.named_parameters() if n not in no_grad)
    for n, p in model.named_parameters():
        g = _g(p).cpu()
        if n in no_grad:
            assert not g.any(), n
            continue
        ref = fx["grad." + n]
        err = float((g.double() - ref.double()).norm())
        assert err <= 1e-4 * float(ref.double().norm()) + 1e-6 * g_scale, (n, err, float(ref.norm()))


def test_fused_step_dropout_masks_and_gradients(monkeypatch):
    """DROPOUT (models.py:358-359, here p = 0.3): the fused step hashes its masks per step — each layer's dropped
    fraction within 0.05 of p over the batch's rows, and a second replay of the same batch draws new masks (another
    loss at lr 0).  Given one step's masks — read back from its layer outputs, where a dropped element is an exact
    zero — the CPU oracle with F.dropout applying those masks gives the same loss (1e-5 relative) and gradients (1e-4
    of their norm) on the host-collated batch."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN, mape
    p = 0.3
    store, cfg = _store(8, seed=23)
    ids = [2, 5, 7]
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      dropout=p)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=3,
                          warmup_ids=[[0, 1]], warmup=1)
    ref = OracleHetroGIN(**kw())
    ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
    lv = float(step.step(ids))
    torch.cuda.synchronize()
    grads = [_g(q).cpu().clone() for q in m1.parameters()]
    act = step.act.detach().cpu().clone()
    a = step.args
    b = _host_batch(store, ids)
    types = ("path", "link", "node")
    n = {t: b.x[t].shape[0] for t in types}
    assert len(set(n.values())) == 3
    masks = {}
    for l in range(a.L):
        for ti, t in enumerate(types):
            o = a.act_off[l][ti]
            masks[(l, t)] = act[o:o + n[t] * a.H].view(n[t], a.H) != 0
            frac = 1.0 - float(masks[(l, t)].float().mean())
            assert abs(frac - p) < 0.05, (l, t, frac)
    calls = {}

    def replay_masks(x, p=0.5, training=True, inplace=False):
        t = next(t for t in types if n[t] == x.shape[0])
        l = calls.get(t, 0)
        calls[t] = l + 1
        return x * (masks[(l, t)].to(x.dtype) * (1.0 / (1.0 - p)))
    monkeypatch.setattr(torch.nn.functional, "dropout", replay_masks)
    out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    lv_ref = mape(out, b.y.reshape(-1, 1))
    torch.sqrt(lv_ref).backward()
    assert calls == {t: a.L for t in types}
    assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (lv, float(lv_ref))
    for g, (nm, q) in zip(grads, ref.named_parameters()):
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((g - want).double().norm())
        assert d <= 1e-4 * float(want.double().norm()) + 1e-9, (nm, d, float(want.norm()))
    lv2 = float(step.step(ids))
    torch.cuda.synchronize()
    assert lv2 != lv and not torch.equal(step.act.detach().cpu(), act)


@pytest.mark.parametrize("variant", ["default", "mlp_bn_global_feats"])
def test_fused_step_ragged_batches_vs_oracle(variant):
    """The epoch's ragged batches (the last DataLoader batch is short: dataset.py:239-244): one captured step of
    capacity 4 replayed on 1, 4, 2 and 3 graphs, each step (Adam at lr 0) against the CPU oracle on its host-collated
    batch — loss 1e-5, gradients 1e-4 of their norm (+1e-6 of the largest with MLP_BN)."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN, mape
    store, cfg = _store(10, seed=31)
    over = {} if variant == "default" else dict(mlp_bn=True, global_feats=True, bl_features=True)
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      **over)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0, capturable=True), store, batch_size=4,
                          warmup_ids=[[0, 1, 2, 3]], warmup=1)
    for ids in ([5], [1, 2, 3, 4], [7, 0], [9, 6, 8]):
        torch.cuda.synchronize()
        ref = OracleHetroGIN(**kw())
        ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
        lv = float(step.step(ids))
        torch.cuda.synchronize()
        b = _host_batch(store, ids)
        out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
        lv_ref = mape(out, b.y.reshape(-1, 1))
        torch.sqrt(lv_ref).backward()
        assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (ids, lv, float(lv_ref))
        gmax = max(float(q.grad.double().norm()) for q in ref.parameters() if q.grad is not None)
        slack = 1e-6 * gmax if over else 1e-9
        for (n, p), q in zip(m1.named_parameters(), ref.parameters()):
            want = q.grad if q.grad is not None else torch.zeros_like(q)
            d = float((_g(p).cpu() - want).double().norm())
            assert d <= 1e-4 * float(want.double().norm()) + slack, (ids, n, d, float(want.norm()))


@pytest.mark.parametrize("variant", ["default", "global_feats_dropout", "mlp_bn"])
def test_fused_eval_vs_oracle_and_captured(variant):
    """SmallBatchEval (train.py:70-113 test() / :322-348 evaluate() on the fused kernels) in eval mode: per batch the
    loss within 1e-5 relative and the predictions within 1e-5 of the CPU oracle's eval-mode forward on the host-collated
    batch (dropout off; MLP_BN's BatchNorm on its running statistics); result()'s running sums equal
    CapturedEvalStep's within 1e-5; after a SmallBatchStep on the same model has folded its parameters into a flat
    buffer (and taken an Adam step, which also moves MLP_BN's running statistics), the evaluation re-captures and
    follows the new parameters."""
    from hgin.graphs import CapturedEvalStep
    from hgin.smallbatch import SmallBatchEval, SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN, mape
    store, cfg = _store(10, seed=29)
    over = {"default": {}, "global_feats_dropout": dict(global_feats=True, bl_features=True, dropout=0.2),
            "mlp_bn": dict(mlp_bn=True)}[variant]
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      **over)
    torch.manual_seed(1997)
    m = HetroGIN(**kw()).to(DEV).eval()
    ev = SmallBatchEval(m, store, batch_size=4, warmup_ids=[[0, 1]], warmup=1)
    seq = [[2, 5, 7], [1, 9], [3, 4, 6, 8]]

    def check(ref):
        n_paths = 0
        for ids in seq:
            lv = float(ev.step(ids))
            torch.cuda.synchronize()
            b = _host_batch(store, ids)
            with torch.no_grad():
                out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
            lv_ref = float(mape(out, b.y.reshape(-1, 1)))
            assert abs(lv - lv_ref) <= 1e-5 * abs(lv_ref), (ids, lv, lv_ref)
            n = out.shape[0]
            n_paths += n
            assert torch.allclose(ev.out_pred[:n].cpu(), out.reshape(-1), rtol=1e-5, atol=1e-5), ids
        return n_paths

    ref = OracleHetroGIN(**kw())
    ref.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    ref.eval()
    n_paths = check(ref)
    avg, mp = ev.result(n_paths)
    ce = CapturedEvalStep(m, store, 4, warmup_ids=[[0, 1]], warmup=1)
    for ids in seq:
        ce.step(ids)
    avg2, mp2 = ce.result(n_paths)
    assert abs(avg - avg2) <= 1e-5 * abs(avg2) and abs(mp - mp2) <= 1e-5 * abs(mp2), (avg, avg2, mp, mp2)
    # a training step folds the parameters elsewhere and moves them: the evaluation follows
    m.train()
    st = SmallBatchStep(m, torch.optim.Adam(m.parameters(), lr=1e-2), store, batch_size=4, warmup_ids=[[0, 1]],
                        warmup=1)
    st.step([3, 8])
    m.eval()
    torch.cuda.synchronize()
    ref.load_state_dict({k: v.detach().cpu() for k, v in m.state_dict().items()})
    ev.reset()
    n_paths = check(ref)
    # CapturedEvalStep follows the re-allocation too (it re-captures on a moved parameter pointer)
    avg, mp = ev.result(n_paths)
    ce.reset()
    for ids in seq:
        ce.step(ids)
    avg2, mp2 = ce.result(n_paths)
    assert abs(avg - avg2) <= 1e-5 * abs(avg2) and abs(mp - mp2) <= 1e-5 * abs(mp2), (avg, avg2, mp, mp2)


@pytest.mark.parametrize("variant", ["default", "mlp_bn_global_feats", "weight_decay"])
def test_fused_trajectory_vs_oracle(variant):
    """Five shuffled batches with Adam(lr=1e-3) (train.py:31-44): the fused step's loss trajectory against
    oracle.pyg_cpu.train_step on the host-collated batches, within 1e-4 relative per step.  ``weight_decay``: config.json's
    WEIGHT_DECAY (train.py:142) at 1e-2, the folded Adam's L2 term (csrc/hgin_smallbatch.hip adam_update) against
    torch's Adam, and the parameters after the last step within 1e-4 of their change.  With GLOBAL_FEATS + MLP_BN the
    BatchNorm running statistics after the last step too, each within 1e-4 of its norm.  The Linear biases ahead of a
    BatchNorm have an exactly-zero true gradient (the normalisation removes them); their rounding-noise gradients become
    +-lr Adam steps of either sign on either side, and they shift the batch mean of z and so running_mean by the same
    amount.  That shift is taken out on both sides before comparing: running_mean - sum_j mom (1 - mom)^(K - j) b_j,
    with b_j each side's own bias at step j (running_var does not see a shift)."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN
    from oracle.pyg_cpu import train_step as oracle_step
    store, cfg = _store(12, seed=13)
    seq = [[1, 6, 10], [4, 0, 11], [8, 3, 5], [9, 7, 2], [3, 10, 1]]
    over = dict(mlp_bn=True, global_feats=True, bl_features=True) if variant == "mlp_bn_global_feats" else {}
    wd = 1e-2 if variant == "weight_decay" else 0.0
    kw = lambda: dict(cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node}),  # noqa: E731
                      **over)
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    ref = OracleHetroGIN(**kw())
    ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
    p0 = [p.detach().cpu().clone() for p in ref.parameters()]
    bn_lin = lambda mod: [seq_[0] for seq_ in mod.readout[:-1] if len(seq_) == 3]  # noqa: E731 (Linear ahead of a BN)
    shift = {"fused": [], "ref": []}   # per step: the pre-BatchNorm biases the step's forward uses
    snap = lambda: (shift["fused"].append([l.bias.detach().cpu().clone() for l in bn_lin(m1)]),  # noqa: E731
                    shift["ref"].append([l.bias.detach().clone() for l in bn_lin(ref)]))
    snap()   # (the warm-up step's)
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3, weight_decay=wd, capturable=True)
    step = SmallBatchStep(m1, o1, store, batch_size=3, warmup_ids=[seq[0]], warmup=1)
    assert step.folded
    o2 = torch.optim.Adam(ref.parameters(), lr=1e-3, weight_decay=wd)
    hb = {tuple(ids): _host_batch(store, ids) for ids in seq}

    def oracle(ids):
        b = hb[tuple(ids)]
        return float(oracle_step(ref, o2, b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y))
    oracle(seq[0])   # the warm-up's Adam step
    for k, ids in enumerate(seq):
        torch.cuda.synchronize()
        snap()
        got, want = float(step.step(ids)), oracle(ids)
        assert abs(got - want) <= 1e-4 * abs(want), (k, got, want)
    torch.cuda.synchronize()
    if wd:
        for (n, p), q, q0 in zip(m1.named_parameters(), ref.parameters(), p0):
            d = float((p.detach().cpu() - q.detach()).double().norm())
            assert d <= 1e-4 * float((q.detach() - q0).double().norm()) + 1e-9, (n, d)
    bns = [mod for mod in ref.modules() if isinstance(mod, torch.nn.BatchNorm1d)]
    K = len(shift["ref"])

    def unshifted(rm, side, i, mom):
        out = rm.double().clone()
        for j in range(K):
            out -= mom * (1.0 - mom) ** (K - 1 - j) * shift[side][j][i].double()
        return out
    i_bn = {}
    for (n, u), (n2, v) in zip(m1.named_buffers(), ref.named_buffers()):
        assert n == n2
        if v.dtype == torch.int64:
            assert torch.equal(u.cpu(), v), n
            continue
        if n.endswith("running_mean"):
            i = i_bn.setdefault(n, len(i_bn))
            mom = bns[i].momentum
            u, v = unshifted(u.cpu(), "fused", i, mom), unshifted(v, "ref", i, mom)
        d = float((u.cpu().double() - v.double()).norm())
        assert d <= 1e-4 * float(v.double().norm()) + 1e-7, (n, d, float(v.norm()))


def test_folded_adam_follows_the_optimizer():
    """The folded Adam follows its torch optimizer between steps: a new lr in the param group (what an LR
    scheduler writes) re-captures the step with it, and ``opt.load_state_dict`` of an earlier state is copied into the
    flat moments / step count — each against oracle.pyg_cpu.train_step with torch's Adam given the same changes at the
    same steps: losses within 1e-4 relative."""
    import copy

    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import OracleHetroGIN
    from oracle.pyg_cpu import train_step as oracle_step
    store, cfg = _store(12, seed=37)
    seq = [[1, 6, 10], [4, 0, 11], [8, 3, 5], [9, 7, 2], [3, 10, 1], [2, 5, 8], [0, 11, 7]]
    kw = lambda: cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})  # noqa: E731
    torch.manual_seed(1997)
    m1 = HetroGIN(**kw()).to(DEV)
    ref = OracleHetroGIN(**kw())
    ref.load_state_dict({k: v.detach().cpu() for k, v in m1.state_dict().items()})
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3)
    step = SmallBatchStep(m1, o1, store, batch_size=3, warmup_ids=[seq[0]], warmup=1)
    o2 = torch.optim.Adam(ref.parameters(), lr=1e-3)
    hb = {tuple(ids): _host_batch(store, ids) for ids in seq}

    def oracle(ids):
        b = hb[tuple(ids)]
        return float(oracle_step(ref, o2, b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y))
    oracle(seq[0])
    saved = None
    for k, ids in enumerate(seq):
        if k == 2:   # the scheduler's write
            for o in (o1, o2):
                o.param_groups[0]["lr"] = 3e-3
        if k == 3:
            torch.cuda.synchronize()
            saved = (copy.deepcopy(o1.state_dict()), copy.deepcopy(o2.state_dict()))
        if k == 5:
            o1.load_state_dict(saved[0])
            o2.load_state_dict(saved[1])
        got, want = float(step.step(ids)), oracle(ids)
        assert abs(got - want) <= 1e-4 * abs(want), (k, got, want)
    assert step.args.lr == pytest.approx(3e-3)


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
    g1 = {n: _g(p).clone() for n, p in m1.named_parameters()}
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
        assert torch.equal(_g(p), g1[n]), n


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
    assert SmallBatchStep.supports(HetroGIN(**kw(mlp_bn=True)))
    assert SmallBatchStep.supports(HetroGIN(**kw(dropout=0.1)))
    assert SmallBatchStep.supports(HetroGIN(**kw(node_embedding_size=128)))
    assert not SmallBatchStep.supports(HetroGIN(**kw(node_embedding_size=256)))
