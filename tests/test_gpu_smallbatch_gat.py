"""The fused small-batch step for HetroGAT (train.py:120-125 builds it for MODEL == "GAT"; config.json: HEADS 16,
NODE_EMBEDDING_SIZE 8, MP_LAYERS 1): k_sb_gat_fwd / the readout / k_sb_gat_bwd / k_sb_final (csrc/hgin_smallbatch.hip).

* Against the reference-executed fixture tests/golden/gat_cfg1_h16.pt (models.py's HetroGAT run over the shim's PyG
  2.0.2 GATConv; its graph regenerated and collated bit-identically): loss within 1e-5 relative, every gradient within
  1e-4 of its norm and None exactly where the reference's is (the three relations that cannot reach the readout), the
  first Adam step within 1e-6 of lr on every entry whose gradient is not at rounding level.
* Against the CPU oracle (oracle.pyg_cpu.OracleHetroGAT, pinned bit for bit to both GAT fixtures by
  tests/test_oracle_golden.py) on host-collated batches of several graphs: loss 1e-5, gradients 1e-4 of their norm,
  BatchNorm running statistics 1e-5, for config.json's shape and the switches (MLP_BN, GLOBAL_FEATS, CONCAT_PATH off,
  other heads x widths), ragged batches from one capture, a five-step Adam trajectory (1e-4 per loss) and the
  evaluation loop (SmallBatchEval, 1e-5).
The fused step folds the projections into the attention (a_s = x_s . W_s^T att_s, out = W_s (sum alpha x_s) + b): the
same sums in another association, so fp32 tolerances, not bit-identity."""
import numpy as np
import pytest
import torch

from hgin import HetroGAT
from hgin.data import CONFIGS, scaled_config, synthetic_graph
from hgin.store import GraphStore

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _store(n, seed):
    rng = np.random.default_rng(seed)
    cfg = CONFIGS["cfg1"]
    graphs = [synthetic_graph(scaled_config(cfg, float(rng.uniform(0.5, 1.5)), name=f"g{i}"), seed=seed * 100 + i)
              for i in range(n)]
    return GraphStore.build(graphs, device=DEV, normalize=True), cfg


def _kw(cfg, **over):
    kw = cfg.model_kwargs({"link": cfg.f_link, "path": cfg.f_path, "node": cfg.f_node})
    kw.update(heads=16, node_embedding_size=8, message_passing_layers=1)
    kw.update(over)
    return kw


def _g(p):
    return p.grad.detach() if p.grad is not None else torch.zeros_like(p.detach())


def _host_batch(store, ids):
    """The batch on the host, pinned to the numpy restatement of PyG's collation of the same graphs."""
    from oracle import collate_np
    b = store.collate(ids).to("cpu")
    want = collate_np.collate([collate_np.from_graph(store.collate([i]).to("cpu")) for i in ids])
    for t in b.x:
        assert torch.equal(b.x[t], torch.from_numpy(want["x"][t])), t
    for r in b.edge_index:
        assert torch.equal(b.edge_index[r], torch.from_numpy(want["edge_index"][r])), r
    assert torch.equal(b.y, torch.from_numpy(want["y"]))
    return b


def _oracle(model, kw):
    """OracleHetroGAT with the HIP model's (materialised) parameters and buffers."""
    from oracle.pyg_cpu import OracleHetroGAT
    dims = {}
    for key, conv in model.convs[0].convs.items():
        s, _, d = key.split("__")
        dims[s], dims[d] = conv.lin_src.weight.shape[1], conv.lin_dst.weight.shape[1]
    ref = OracleHetroGAT(dims, kw["node_embedding_size"], kw["heads"], kw["dropout"], kw["concat_path"],
                         kw["bl_features"], kw["divided_features"], kw["global_feats"], list(kw["mlp_layers"]),
                         kw["act"], kw["mlp_head_act"], kw["mlp_bn"])
    ref.load_state_dict({k: v.detach().cpu() for k, v in model.state_dict().items()})
    return ref


def _check_grads(model, ref, slack_rel=0.0):
    gmax = max(float(q.grad.double().norm()) for q in ref.parameters() if q.grad is not None)
    bad = []
    for (n, p), (n2, q) in zip(model.named_parameters(), ref.named_parameters()):
        assert n == n2
        assert (p.grad is None) == (q.grad is None), n
        want = q.grad if q.grad is not None else torch.zeros_like(q)
        d = float((_g(p).cpu() - want).double().norm())
        if not d <= 1e-4 * float(want.double().norm()) + slack_rel * gmax + 1e-9:
            bad.append((n, d, float(want.norm())))
    assert not bad, bad


def test_fused_gat_step_vs_reference_fixture():
    from conftest import load_fixture
    from hgin.smallbatch import SmallBatchStep
    fx = load_fixture("gat_cfg1_h16")
    m = fx["meta"]
    cfg = CONFIGS["cfg1"]
    store = GraphStore.build([synthetic_graph(cfg, seed=11)], device=DEV, normalize=False)
    b = store.collate([0]).to("cpu")
    for t in ("path", "link", "node"):
        assert torch.equal(b.x[t], fx[f"in.x.{t}"]), t
    for r in m["relations"]:
        assert torch.equal(b.edge_index[tuple(r.split("__"))], fx[f"in.ei.{r}"]), r
    assert torch.equal(b.y, fx["in.y"])
    kw = _kw(cfg, node_embedding_size=m["hidden"], heads=m["heads"], concat_path=m["concat_path"],
             bl_features=m["bl_features"], divided_features=m["divided_features"], mlp_layers=list(m["mlp_layers"]))
    model = HetroGAT(**kw)
    sd = {k[3:]: v for k, v in fx.items() if k.startswith("sd.")}
    model.load_state_dict(sd)   # (materialises the lazy projections)
    model = model.to(DEV)
    opt = torch.optim.Adam(model.parameters(), lr=0.0)
    step = SmallBatchStep(model, opt, store, batch_size=1, warmup_ids=[[0]], warmup=1)
    assert step.folded and step.gat and step.args.gat_heads == 16 and step.args.gat_c == 8
    lv = float(step.step([0]))   # (a hipGraph replay: the launch trace records the capture, not the replays)
    torch.cuda.synchronize()
    want = float(fx["loss_value"])
    assert abs(lv - want) <= 1e-5 * abs(want), (lv, want)
    for n, p in model.named_parameters():
        ref = fx["grad." + n]
        if ref.numel() == 0:   # the reference's None: a relation that cannot reach the readout
            assert p.grad is None, n
            continue
        err = float((_g(p).cpu().double() - ref.double()).norm())
        assert err <= 1e-4 * float(ref.double().norm()) + 1e-9, (n, err, float(ref.norm()))
    # the first Adam step (lr 1e-3) from the same parameters: fresh moments, the new lr re-captures the step
    p0 = {n: p.detach().cpu().clone() for n, p in model.named_parameters()}
    step.mflat.zero_()
    step.vflat.zero_()
    step.adam_step.zero_()
    opt.param_groups[0]["lr"] = 1e-3
    step.step([0])
    torch.cuda.synchronize()
    for n, p in model.named_parameters():
        got = p.detach().cpu()
        ref_step, g_ref = fx["step." + n], fx["grad." + n]
        if g_ref.numel() == 0:   # not stepped (no gradient), as torch's Adam
            assert torch.equal(got, p0[n]), n
            continue
        big = g_ref.abs() > 1e-4 * float(g_ref.abs().max())   # (near-zero gradients: Adam's +-lr on rounding noise)
        assert (got[big] - ref_step[big]).abs().max() <= 1e-6, n
        assert ((got - ref_step).abs() <= 2e-3 + 1e-6).all(), n


@pytest.mark.parametrize("variant", ["default", "mlp_bn", "global_feats", "no_concat", "heads4_c16", "heads32_c4",
                                     "dropout"])
def test_fused_gat_step_vs_oracle(variant, monkeypatch):
    """One fused step (Adam at lr 0) against OracleHetroGAT's forward and sqrt-MAPE backward on the host-collated batch;
    dropout (p 0.3) by replaying the step's own masks (read back from its layer outputs) through the oracle."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import mape
    over = {"default": {}, "mlp_bn": dict(mlp_bn=True), "global_feats": dict(global_feats=True, bl_features=True),
            "no_concat": dict(concat_path=False), "heads4_c16": dict(heads=4, node_embedding_size=16),
            "heads32_c4": dict(heads=32, node_embedding_size=4), "dropout": dict(dropout=0.3)}[variant]
    store, cfg = _store(8, seed=41)
    ids = [1, 6, 3]
    kw = _kw(cfg, **over)
    torch.manual_seed(1997)
    m1 = HetroGAT(**dict(kw, input_channels=dict(kw["input_channels"]))).to(DEV)
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0), store, batch_size=4, warmup_ids=[[0, 2]],
                          warmup=1)
    torch.cuda.synchronize()
    # GATConv's bias starts at 0 (reset_parameters): a destination row without edges (path rows past the link count get
    # no self loop) then outputs exactly 0, which the dropout replay below would read as dropped — nonzero biases keep
    # every kept element nonzero (written through the parameters, which are views of the step's flat buffer)
    with torch.no_grad():
        for conv in m1.convs[0].convs.values():
            conv.bias.uniform_(-0.1, 0.1)
    ref = _oracle(m1, kw)   # (after the warm-up step, which advanced MLP_BN's running statistics)
    lv = float(step.step(ids))
    torch.cuda.synchronize()
    b = _host_batch(store, ids)
    if kw["dropout"] > 0:
        act = step.act.detach().cpu().clone()
        a = step.args
        n = {t: b.x[t].shape[0] for t in ("path", "link", "node")}
        masks = {}
        for ti, t in enumerate(("path", "link", "node")):
            o = a.act_off[0][ti]
            masks[n[t]] = act[o:o + n[t] * a.H].view(n[t], a.H) != 0
            assert abs((1.0 - float(masks[n[t]].float().mean())) - kw["dropout"]) < 0.05, t
        monkeypatch.setattr(torch.nn.functional, "dropout",
                            lambda x, p=0.5, training=True, inplace=False: x * (masks[x.shape[0]].to(x.dtype) /
                                                                               (1.0 - p)))
    out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    lv_ref = mape(out, b.y.reshape(-1, 1))
    torch.sqrt(lv_ref).backward()
    assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (lv, float(lv_ref))
    _check_grads(m1, ref, 1e-6 if kw["mlp_bn"] else 0.0)
    for (n, u), (n2, v) in zip(m1.named_buffers(), ref.named_buffers()):
        assert n == n2
        if v.dtype == torch.int64:
            assert torch.equal(u.cpu(), v), n
        else:
            assert torch.allclose(u.cpu(), v, rtol=1e-5, atol=1e-6), (n, float((u.cpu() - v).abs().max()))
    if kw["dropout"] == 0:   # bitwise run to run
        g1 = [_g(p).clone() for p in m1.parameters()]
        assert float(step.step(ids)) == lv
        torch.cuda.synchronize()
        for g, p in zip(g1, m1.parameters()):
            assert torch.equal(g, _g(p))


def test_fused_gat_ragged_batches_vs_oracle():
    """One capture of capacity 4 replayed on 1, 4, 2 and 3 graphs (the epoch's short last batch), each against the
    oracle: loss 1e-5, gradients 1e-4 of their norm."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import mape
    store, cfg = _store(10, seed=43)
    kw = _kw(cfg)
    torch.manual_seed(1997)
    m1 = HetroGAT(**dict(kw, input_channels=dict(kw["input_channels"]))).to(DEV)
    step = SmallBatchStep(m1, torch.optim.Adam(m1.parameters(), lr=0.0), store, batch_size=4,
                          warmup_ids=[[0, 1, 2, 3]], warmup=1)
    for ids in ([5], [1, 2, 3, 4], [7, 0], [9, 6, 8]):
        torch.cuda.synchronize()
        ref = _oracle(m1, kw)
        lv = float(step.step(ids))
        torch.cuda.synchronize()
        b = _host_batch(store, ids)
        out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
        lv_ref = mape(out, b.y.reshape(-1, 1))
        torch.sqrt(lv_ref).backward()
        assert abs(lv - float(lv_ref)) <= 1e-5 * abs(float(lv_ref)), (ids, lv, float(lv_ref))
        _check_grads(m1, ref)


@pytest.mark.parametrize("variant", ["default", "mlp_bn"])
def test_fused_gat_trajectory_vs_oracle(variant):
    """Five shuffled batches with Adam(lr=1e-3) (train.py:31-44) against oracle.pyg_cpu.train_step: each loss within
    1e-4 relative."""
    from hgin.smallbatch import SmallBatchStep
    from oracle.pyg_cpu import train_step as oracle_step
    store, cfg = _store(12, seed=47)
    seq = [[1, 6, 10], [4, 0, 11], [8, 3, 5], [9, 7, 2], [3, 10, 1]]
    kw = _kw(cfg, **({"mlp_bn": True} if variant == "mlp_bn" else {}))
    torch.manual_seed(1997)
    m1 = HetroGAT(**dict(kw, input_channels=dict(kw["input_channels"]))).to(DEV)
    hb = {tuple(ids): _host_batch(store, ids) for ids in seq}
    o1 = torch.optim.Adam(m1.parameters(), lr=1e-3)
    # the oracle twin from the parameters the fused step's warm-up starts from (materialised on the warm-up batch)
    from hgin.smallbatch import _materialize
    _materialize(m1, store, seq[0])
    ref = _oracle(m1, kw)
    step = SmallBatchStep(m1, o1, store, batch_size=3, warmup_ids=[seq[0]], warmup=1)
    o2 = torch.optim.Adam(ref.parameters(), lr=1e-3)

    def oracle(ids):
        b = hb[tuple(ids)]
        return float(oracle_step(ref, o2, b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y))
    oracle(seq[0])   # the warm-up's Adam step
    for k, ids in enumerate(seq):
        got, want = float(step.step(ids)), oracle(ids)
        assert abs(got - want) <= 1e-4 * abs(want), (k, got, want)


def test_fused_gat_eval_vs_oracle():
    """SmallBatchEval (train.py:70-113 test() / :322-348 evaluate()) on the GAT kernels in eval mode: per batch the
    loss and the predictions within 1e-5 of the oracle's eval-mode forward; the running sums equal the per-batch
    losses' (avg) and the path-weighted MAPE."""
    from hgin.smallbatch import SmallBatchEval
    from oracle.pyg_cpu import mape
    store, cfg = _store(10, seed=53)
    kw = _kw(cfg)
    torch.manual_seed(1997)
    m = HetroGAT(**dict(kw, input_channels=dict(kw["input_channels"]))).to(DEV).eval()
    ev = SmallBatchEval(m, store, batch_size=4, warmup_ids=[[0, 1]], warmup=1)
    ref = _oracle(m, kw).eval()
    lvs, n_paths, wsum = [], 0, 0.0
    for ids in ([2, 5, 7], [1, 9], [3, 4, 6, 8]):
        lv = float(ev.step(ids))
        torch.cuda.synchronize()
        b = _host_batch(store, ids)
        with torch.no_grad():
            out = ref(b.x_dict(), b.edge_index_dict(), b.batch["path"])
        lv_ref = float(mape(out, b.y.reshape(-1, 1)))
        assert abs(lv - lv_ref) <= 1e-5 * abs(lv_ref), (ids, lv, lv_ref)
        nn = out.shape[0]
        assert torch.allclose(ev.out_pred[:nn].cpu(), out.reshape(-1), rtol=1e-5, atol=1e-5), ids
        lvs.append(lv_ref)
        n_paths += nn
        wsum += lv_ref * nn
    avg, mp = ev.result(n_paths)
    assert abs(avg - np.mean(lvs)) <= 1e-5 * abs(avg) and abs(mp - wsum / n_paths) <= 1e-5 * abs(mp)
