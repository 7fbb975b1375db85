"""Golden vectors for the feature normalisation by EXECUTING the reference's own ``GNN21Dataset.normalize``
(``dataset.py:33-58``) — run in the build container only:

    python tests/golden/make_golden_normalize.py      # writes tests/golden/normalize_ref.pt

``dataset.py`` imports PyG (absent here): ``tests/golden/pyg_shim`` provides the one symbol its
import needs (``torch_geometric.data.Dataset``, a bare base class).  ``normalize`` is called unbound on a
HeteroData-like mapping (``data["link"].x`` / ``data["path"].x``), which is all it touches.  Inputs: the raw
7 / 7 / 3 feature layout (``dataset.py:90-106``) of 4 synthetic cfg1 graphs collated PyG-style (the store
normalises the collated features once), plus a block of extreme values.  ``sys.dont_write_bytecode`` keeps
/root/reference untouched.
"""
from __future__ import annotations

import importlib.util
import os
import sys
from types import SimpleNamespace

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REFERENCE = "/root/reference"
sys.path.insert(0, os.path.join(HERE, "pyg_shim"))
sys.path.insert(0, os.path.join(REPO, "gnn-link-prediction_amd"))
sys.path.insert(0, REPO)

import torch  # noqa: E402

from hgin.data import CONFIGS, collate, synthetic_graph  # noqa: E402

GRAPH_SEEDS = (11, 12, 13, 14)


def load_reference_dataset():
    sys.path.insert(0, REFERENCE)          # dataset.py imports datanetAPI and models by module name
    try:
        spec = importlib.util.spec_from_file_location("reference_dataset", os.path.join(REFERENCE, "dataset.py"))
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
    finally:
        sys.path.remove(REFERENCE)
    return mod


def inputs():
    big = collate([synthetic_graph(CONFIGS["cfg1"], seed=s) for s in GRAPH_SEEDS])
    x = {t: v.clone() for t, v in big.x.items()}
    g = torch.Generator().manual_seed(99)
    # extremes: large / tiny / negative / exactly-the-mean values in every normalised column
    ext_l = torch.cat([torch.full((1, 7), 1e30), torch.full((1, 7), -3.5), torch.full((1, 7), 1e-30),
                       torch.rand(5, 7, generator=g) * 1000])
    ext_l[3, :6] = torch.tensor([0.3546671, 0.16771736017268535, 0.09862498490722958, 0.05104, 0.35411, 0.00066])
    ext_p = torch.cat([torch.full((1, 7), -1e30), torch.full((1, 7), 2.0), torch.rand(6, 7, generator=g) - 0.5])
    x["link"] = torch.cat([x["link"], ext_l])
    x["path"] = torch.cat([x["path"], ext_p])
    return x


def main():
    ds = load_reference_dataset()
    x = inputs()
    data = {t: SimpleNamespace(x=v.clone()) for t, v in x.items()}
    out = ds.GNN21Dataset.normalize(None, data)
    fx = {"meta": {"reference": "dataset.py:33-58 GNN21Dataset.normalize executed via tests/golden/pyg_shim",
                   "graph_seeds": list(GRAPH_SEEDS), "layout": "raw 7/7/3 (dataset.py:90-106)"}}
    for t in x:
        fx[f"in.x.{t}"] = x[t]
        fx[f"out.x.{t}"] = out[t].x.clone()
    torch.save(fx, os.path.join(HERE, "normalize_ref.pt"))
    print("wrote", os.path.join(HERE, "normalize_ref.pt"))


if __name__ == "__main__":
    main()
