"""The CPU oracle (oracle/pyg_cpu.py) against the golden vectors made by executing the reference's own
models.py (tests/golden/make_golden.py).  Everything is compared bit-for-bit: same torch CPU ops."""
import pytest
import torch

from conftest import (CASES, assert_state_dict_digests, fixture_inputs, fixture_model_kwargs, is_compact,
                      load_fixture)
from oracle.pyg_cpu import OracleHetroGIN, mape, propagate_sum


@pytest.fixture(autouse=True)
def _one_thread():
    n = torch.get_num_threads()
    torch.set_num_threads(1)
    yield
    torch.set_num_threads(n)


@pytest.mark.parametrize("case", CASES)
def test_oracle_reproduces_reference(case):
    fx = load_fixture(case)
    torch.manual_seed(fx["meta"]["seed_model"])
    kw = fixture_model_kwargs(fx)
    model = OracleHetroGIN(**kw)
    assert kw["input_channels"] == fx["meta"]["input_channels_after_ctor"]
    sd = model.state_dict()
    if is_compact(fx):
        assert_state_dict_digests(fx, sd)
    else:
        assert list(sd) == [k[3:] for k in fx if k.startswith("sd.")]
        for k, v in sd.items():
            assert torch.equal(v, fx["sd." + k]), k
    x, ei, batch, y = fixture_inputs(fx)
    model.set_record(True)
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0)
    opt.zero_grad()
    out = model(dict(x), ei, batch)
    assert torch.equal(out, fx["out"])
    # per-relation aggregates (propagate results) in layer / relation order
    for li, conv in enumerate(model.convs):
        for key, layer in conv.convs.items():
            agg, k = layer.conv.trace[0], f"agg.{li}.{key}"
            if is_compact(fx):   # sampled rows bit-exact, whole-tensor float64 sums to rounding
                assert torch.equal(agg[fx["rows." + k]], fx[k]), (li, key)
                assert torch.allclose(_sums(agg), fx["sums." + k], rtol=1e-12, atol=0), (li, key)
            else:
                assert torch.equal(agg, fx[k]), (li, key)
    lv = mape(out, y.reshape(-1, 1))
    assert torch.equal(lv, fx["loss_value"])
    torch.sqrt(lv).backward()
    for n, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros(0)
        assert torch.equal(g, fx["grad." + n]), n
    if is_compact(fx):
        return                       # compact fixtures carry no Adam step (the full-size cases pin it)
    opt.step()
    for n, p in model.named_parameters():
        assert torch.equal(p, fx["step." + n]), n


def _sums(t):
    d = t.detach().double()
    return torch.stack([d.sum(), d.abs().sum(), (d * d).sum()])


def test_propagate_equals_sequential_edge_order():
    """scatter_add_ on CPU == per-destination sequential sum in original edge order."""
    g = torch.Generator().manual_seed(7)
    n_src, n_dst, E, F = 500, 300, 20000, 5
    ei = torch.stack([torch.randint(0, n_src, (E,), generator=g), torch.randint(0, n_dst, (E,), generator=g)])
    x = torch.randn(n_src, F, generator=g)
    ref = propagate_sum(x, ei, n_dst)
    order = torch.sort(ei[1], stable=True).indices
    out = torch.zeros(n_dst, F)
    for e in order.tolist():
        out[ei[1, e]] += x[ei[0, e]]
    assert torch.equal(ref, out)


@pytest.mark.parametrize("case", ["gat_cfg1_h16", "gat_w16_h4"])
def test_oracle_gat_reproduces_reference(case):
    """OracleHetroGAT (the fused GAT step's checker) against the reference's HetroGAT executed over the shim's GATConv
    (tests/golden/make_golden.py ``gat``): output, loss, every gradient (None for the dead relations) and the Adam step,
    bit for bit."""
    from oracle.pyg_cpu import OracleHetroGAT
    fx = load_fixture(case)
    m = fx["meta"]
    sd = {k[3:]: v for k, v in fx.items() if k.startswith("sd.")}
    dims = {}
    for key in m["relations"]:
        s, _, d = key.split("__")
        if f"convs.0.convs.{key}.lin_src.weight" not in sd:   # (carried in the data, no conv: models.py:413-418)
            continue
        dims[s] = sd[f"convs.0.convs.{key}.lin_src.weight"].shape[1]
        dims[d] = sd[f"convs.0.convs.{key}.lin_dst.weight"].shape[1]
    model = OracleHetroGAT(dims, node_embedding_size=m["hidden"], heads=m["heads"], dropout=0.0,
                           concat_path=m["concat_path"], bl_features=m["bl_features"],
                           divided_features=m["divided_features"], global_feats=False, mlp_layers=list(m["mlp_layers"]),
                           act="torch.nn.PReLU()", mlp_head_act=None, mlp_bn=False)
    assert list(model.state_dict()) == list(sd)
    model.load_state_dict(sd)
    x = {t: fx[f"in.x.{t}"].clone() for t in ("path", "link", "node")}
    ei = {tuple(r.split("__")): fx[f"in.ei.{r}"] for r in m["relations"]}
    opt = torch.optim.Adam(lr=1e-3, params=model.parameters(), weight_decay=0)
    out = model(x, ei, fx["in.batch"])
    assert torch.equal(out, fx["out"]), float((out - fx["out"]).abs().max())
    lv = mape(out, fx["in.y"].reshape(-1, 1))
    assert torch.equal(lv, fx["loss_value"])
    torch.sqrt(lv).backward()
    for n, p in model.named_parameters():
        g = p.grad if p.grad is not None else torch.zeros(0)
        assert torch.equal(g, fx["grad." + n]), n
    opt.step()
    for n, p in model.named_parameters():
        assert torch.equal(p.detach(), fx["step." + n]), n
