"""The independent PyG-collation restatement (oracle/collate_np.py) against the product's host collation
(hgin.data.collate).  PyG itself is not importable here, so the collation semantics are
"parity unpinned" beyond these two independent restatements agreeing."""
import dataclasses

import numpy as np
import pytest
import torch

from conftest import load_fixture
from hgin.data import CONFIGS, REL_PN, collate, scaled_config, synthetic_graph
from oracle import collate_np


def _graphs(n, seed):
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        cfg = dataclasses.replace(scaled_config(CONFIGS["cfg1"], float(rng.uniform(0.02, 0.5)), name=f"g{i}"),
                                  e_pn=int(rng.integers(0, 40)), with_np=bool(i % 2))
        g = synthetic_graph(dataclasses.replace(cfg, with_np=True), seed=seed * 100 + i)
        if i == 2:
            g.edge_index[REL_PN] = torch.empty(2, 0, dtype=torch.long)     # an empty relation in the middle
        out.append(g)
    return out


@pytest.mark.parametrize("n,seed", [(1, 0), (2, 1), (8, 2), (13, 3)])
def test_oracle_collate_equals_host_collate(n, seed):
    graphs = _graphs(n, seed)
    a = collate(graphs)
    b = collate_np.collate([collate_np.from_graph(g) for g in graphs])
    for t in a.x:
        assert np.array_equal(a.x[t].numpy(), b["x"][t]), t
        assert np.array_equal(a.batch[t].numpy(), b["batch"][t]), t
    assert list(a.edge_index) == list(b["edge_index"])
    for r in a.edge_index:
        assert a.edge_index[r].dtype == torch.long
        assert np.array_equal(a.edge_index[r].numpy(), b["edge_index"][r]), r
    assert np.array_equal(a.y.numpy(), b["y"])


def test_fixture_inputs_are_still_the_oracle_collation():
    """Regression guard, NOT a parity pin: tests/golden/make_golden.py built collate2_global_bn's inputs with
    collate_np itself (two cfg1 graphs, seeds 4 and 5), so this only checks that neither the generator nor
    collate_np drifted since the fixture was made (the reference's models.py then ran on exactly these inputs)."""
    fx = load_fixture("collate2_global_bn")
    cfg = dataclasses.replace(CONFIGS["cfg1"], bl_features=True)
    c = collate_np.collate([collate_np.from_graph(synthetic_graph(cfg, seed=s)) for s in (4, 5)])
    for t in ("path", "link", "node"):
        assert np.array_equal(fx[f"in.x.{t}"].numpy(), c["x"][t]), t
    for r in fx["meta"]["relations"]:
        assert np.array_equal(fx[f"in.ei.{r}"].numpy(), c["edge_index"][tuple(r.split("__"))]), r
    assert np.array_equal(fx["in.batch"].numpy(), c["batch"]["path"])
    assert np.array_equal(fx["in.y"].numpy(), c["y"])
