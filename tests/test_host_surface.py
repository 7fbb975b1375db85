"""Host-side mirror of models.py: constructor, init RNG parity, state_dict layout, no CPU fallback,
PyG input checks, dead-relation analysis, synthetic data + collation."""
import dataclasses

import pytest
import torch

import models as dropin_models
from conftest import (CASES, assert_state_dict_digests, fixture_model_kwargs, fixture_state_dict, is_compact,
                      load_fixture)
from hgin import GINConv, GINLayer, HetroGAT, HetroGIN, ops
from hgin.data import CONFIGS, REL_LP, REL_PL, collate, scaled_config, synthetic_graph
from hgin.models import make_activation


def test_dropin_module_exports_reference_names():
    assert dropin_models.HetroGIN is HetroGIN
    assert dropin_models.GINLayer is GINLayer and dropin_models.GINConv is GINConv
    assert dropin_models.HetroGAT is HetroGAT and issubclass(HetroGAT, torch.nn.Module)   # train.py:120-125


@pytest.mark.parametrize("case", CASES)
def test_init_and_state_dict_match_reference(case):
    """Same seed -> the reference's exact parameter values (double Linear init via reset, models.py:162-199)."""
    fx = load_fixture(case)
    torch.manual_seed(fx["meta"]["seed_model"])
    kw = fixture_model_kwargs(fx)
    model = HetroGIN(**kw)
    assert kw["input_channels"] == fx["meta"]["input_channels_after_ctor"]  # mutated like the reference
    sd = model.state_dict()
    if is_compact(fx):
        assert_state_dict_digests(fx, sd)
    else:
        assert list(sd) == [k[3:] for k in fx if k.startswith("sd.")]
        for k, v in sd.items():
            assert torch.equal(v, fx["sd." + k]), k
    # a reference checkpoint loads strictly (train.py:327)
    model.load_state_dict(fixture_state_dict(fx), strict=True)


def test_forward_refuses_cpu_tensors():
    """Host-resident call (train.py:322-348 evaluate) without a HIP device: raises, never a CPU fallback.
    With a device the call runs there (tests/test_gpu_model.py::test_evaluate_host_resident_call)."""
    if torch.cuda.is_available():
        pytest.skip("a HIP device is visible: host-resident calls run on it")
    fx = load_fixture("cfg1_L2")
    model = HetroGIN(**fixture_model_kwargs(fx))
    x = {t: fx[f"in.x.{t}"] for t in ("path", "link", "node")}
    ei = {tuple(r.split("__")): fx[f"in.ei.{r}"] for r in fx["meta"]["relations"]}
    with pytest.raises(RuntimeError, match="no CPU fallback"):
        model(x, ei, fx["in.batch"])


def test_edge_index_checks_match_pyg():
    with pytest.raises(AssertionError):
        ops.check_edge_index(torch.zeros(2, 5, dtype=torch.int32))
    with pytest.raises(AssertionError):
        ops.check_edge_index(torch.zeros(3, 5, dtype=torch.long))
    with pytest.raises(AssertionError):
        ops.check_edge_index(torch.zeros(10, dtype=torch.long))


def test_dead_relations_match_survey():
    fx = load_fixture("cfg1_L2")
    model = HetroGIN(**fixture_model_kwargs(fx))
    dead = model.prune_dead(True)
    assert sorted(dead) == sorted(["1:path__uses__link", "1:link__connects__node", "1:node__has__link",
                                   "0:link__connects__node"])
    # matches the params that get no gradient in the reference's own backward
    no_grad = {n.split(".mlp.")[0].split(".conv.")[0] for n in fx["meta"]["no_grad_params"]}
    assert no_grad == {f"convs.{d.split(':')[0]}.convs.{d.split(':')[1]}" for d in dead}
    model.prune_dead(False)
    assert all(not c.skip for c in model.convs)


def test_activation_whitelist():
    assert isinstance(make_activation("torch.nn.PReLU()"), torch.nn.PReLU)
    with pytest.raises(ValueError):
        make_activation("__import__('os').system('true')")


def test_synthetic_graph_schema():
    cfg = scaled_config(CONFIGS["cfg2"], 1e-4)
    g = synthetic_graph(cfg, seed=3)
    assert list(g.edge_index) == [("path", "uses", "link"), ("link", "includes", "path"),
                                  ("link", "connects", "node"), ("node", "has", "link"),
                                  ("path", "is_connected", "node")]
    assert torch.equal(g.edge_index[REL_LP], g.edge_index[REL_PL].flip(0))
    assert g.x["path"].shape == (cfg.n_path, cfg.f_path)
    assert (g.y >= 0.5).all() and (g.y < 1.5).all()
    assert cfg.conv_edges == 2 * cfg.e_pl + 2 * cfg.e_ln
    assert torch.equal(synthetic_graph(cfg, seed=3).x["link"], g.x["link"])  # seeded


def test_collate_offsets():
    cfg = CONFIGS["cfg1"]
    a, b = synthetic_graph(cfg, seed=1), synthetic_graph(cfg, seed=2)
    c = collate([a, b])
    for et, e in c.edge_index.items():
        Ea = a.edge_index[et].size(1)
        assert torch.equal(e[:, :Ea], a.edge_index[et])
        off = torch.tensor([[a.num_nodes(et[0])], [a.num_nodes(et[2])]])
        assert torch.equal(e[:, Ea:], b.edge_index[et] + off)
    assert torch.equal(c.batch["path"], torch.cat([torch.zeros(cfg.n_path), torch.ones(cfg.n_path)]).long())


def test_config_sizes():
    c2, c3 = CONFIGS["cfg2"], CONFIGS["cfg3"]
    assert c2.nodes == 1_000_000 and c2.graph_edges == 10_000_000
    assert c3.nodes == 10_000_000 and c3.graph_edges == 100_000_000
    assert CONFIGS["cfg1"].nodes == 1000 and CONFIGS["cfg1"].graph_edges == 5000
