"""HetroGAT host-side checks (no GPU): the oracle's GATConv relation restatement reproduces the reference-executed
fixtures bit for bit (attention and aggregate), and the drop-in's constructor matches the reference's parameter
names, order and constructor-time initial values under train.py's seed (the lazy (-1, -1) projections materialise at
the first forward, on the device: checked in tests/test_gpu_gat.py)."""
import pytest
import torch

from conftest import load_fixture

CASES = ["gat_cfg1_h16", "gat_w16_h4"]


def _kwargs(fx):
    m = fx["meta"]
    ic = {"link": fx["in.x.link"].shape[1], "path": fx["in.x.path"].shape[1], "node": fx["in.x.node"].shape[1]}
    return dict(input_channels=ic, node_embedding_size=m["hidden"], message_passing_layers=m["layers"], dropout=0.0,
                heads=m["heads"], concat_path=m["concat_path"], bl_features=m["bl_features"],
                divided_features=m["divided_features"], global_feats=False, mlp_layers=list(m["mlp_layers"]),
                act="torch.nn.PReLU()", mlp_head_act=None, mlp_bn=False)


def _sliced(fx):
    """models.py:482-493 feature slicing of the fixture inputs."""
    m = fx["meta"]
    x = {t: fx[f"in.x.{t}"] for t in ("path", "link", "node")}
    if not m["divided_features"]:
        x["path"] = torch.cat([x["path"][:, 0:3], x["path"][:, 6].reshape(-1, 1)], axis=1)
        x["link"] = torch.cat([x["link"][:, 0:3], x["link"][:, 4:7]], axis=1)
        if not m["bl_features"]:
            x["path"], x["link"] = x["path"][:, 0:3], x["link"][:, 0:3]
    elif not m["bl_features"]:
        x["path"], x["link"] = x["path"][:, 0:6], x["link"][:, 0:3]
    return x


@pytest.mark.parametrize("case", CASES)
def test_oracle_gat_relation_matches_reference(case):
    from oracle.pyg_cpu import gat_relation
    fx = load_fixture(case)
    x = _sliced(fx)
    H = fx["meta"]["heads"]
    for key in ("path__uses__link", "link__includes__path", "link__connects__node", "node__has__link"):
        src, _, dst = key.split("__")
        pre = f"sd.convs.0.convs.{key}."
        xs = torch.nn.functional.linear(x[src], fx[pre + "lin_src.weight"]).view(x[src].size(0), H, -1)
        xd = torch.nn.functional.linear(x[dst], fx[pre + "lin_dst.weight"]).view(x[dst].size(0), H, -1)
        alpha, agg = gat_relation(xs, xd, fx[f"in.ei.{key}"], fx[pre + "att_src"], fx[pre + "att_dst"])
        assert torch.equal(alpha, fx[f"alpha.0.{key}"]), key
        assert torch.equal(agg, fx[f"agg.0.{key}"]), key


def test_constructor_matches_reference_initialisation():
    from hgin import HetroGAT
    fx = load_fixture("gat_cfg1_h16")
    torch.manual_seed(fx["meta"]["seed_model"])
    kw = _kwargs(fx)
    ic = dict(kw["input_channels"])
    model = HetroGAT(**kw)
    assert kw["input_channels"] == ic          # HetroGAT reads input_channels; it does not mutate it (models.py:396)
    assert [n for n, _ in model.named_parameters()] == fx["meta"]["param_names_before_forward"]
    sd = model.state_dict()
    for k, v in sd.items():
        if k.endswith("lin_src.weight") or k.endswith("lin_dst.weight"):
            assert isinstance(v, torch.nn.parameter.UninitializedParameter), k   # lazy until the first forward
            continue
        assert torch.equal(v, fx["sd." + k]), k   # constructor-time RNG draws in the reference's order


def test_captured_padded_steps_refuse_gat_self_loops():
    """The captured padded steps (hgin/graphs.py) refuse HetroGAT: GATConv's bipartite self loops (i, i) for
    i < min(N_src, N_dst) would be counted on the padded capacities, giving real rows a loop from a padding source row;
    HetroGIN passes the same check (the fused step takes HetroGAT on real row counts)."""
    from hgin import HetroGAT, HetroGIN
    from hgin.graphs import _check_no_bipartite_loops
    fx = load_fixture("gat_cfg1_h16")
    kw = _kwargs(fx)
    with pytest.raises(ValueError, match="self loops"):
        _check_no_bipartite_loops(HetroGAT(**kw))
    gin_kw = {k: v for k, v in kw.items() if k != "heads"}
    _check_no_bipartite_loops(HetroGIN(**gin_kw))
