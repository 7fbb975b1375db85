"""Golden fixtures for the queueing-theory baseline by EXECUTING the reference's own
``QTBaseline`` (``models.py:15-158``) over the PyG shim (torch_scatter.scatter = zeros().scatter_add_).

    python tests/golden/make_golden_qt.py        # build container only; writes tests/golden/qt_<case>.pt

Inputs are synthetic RouteNet-shaped samples (``hgin/qt_data.py``: same vertex / edge insertion rules as
``generateFiles.py:26-101``).  Each fixture: ``in.edge_index``, ``in.edge_type``, ``in.type``, ``in.P``,
``in.L`` and the reference's outputs ``out.delay`` ([n_paths]) and ``out.feats`` ([n_links, 3] =
[L, rhos, pi_0]); weights_only-loadable.
"""
from __future__ import annotations

import os
import sys

sys.dont_write_bytecode = True
HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(HERE, "pyg_shim"))
sys.path.insert(0, os.path.join(REPO, "gnn-link-prediction_amd"))

import torch  # noqa: E402

from hgin.qt_data import collate_routes, route_sample  # noqa: E402
from make_golden import load_reference_models  # noqa: E402

CASES = {
    "qt_n6": lambda: route_sample(6, seed=1),
    "qt_n12_f2": lambda: route_sample(12, seed=2, flows_per_pair=2),
    "qt_batch3": lambda: collate_routes([route_sample(5, seed=10), route_sample(8, seed=11), route_sample(7, seed=12)]),
}


def _clip_keeps_integer_dtype():
    """The reference targets torch ~1.10 (PyG 2.0.2 era), where ``torch.clip(long, 0., 1.)`` stayed long;
    torch >= 1.13 promotes it to float and ``separate_edge_timesteps`` (models.py:21-26) then fails on its
    long index_put.  Restore the old semantics for integer inputs in this generator process only."""
    orig = torch.clip

    def clip(input, min=None, max=None, *, out=None):
        res = orig(input, min, max) if out is None else orig(input, min, max, out=out)
        if not input.is_floating_point() and res.is_floating_point():
            res = res.to(input.dtype)
        return res

    torch.clip = clip


def main():
    _clip_keeps_integer_dtype()
    ref = load_reference_models()
    for name, make in CASES.items():
        s = make()
        out, feats = ref.QTBaseline()(s)
        fx = {"meta": {"case": name, "num_nodes": s.num_nodes, "source": "reference models.py QTBaseline over "
                       "tests/golden/pyg_shim"},
              "in.edge_index": s.edge_index, "in.edge_type": s.edge_type, "in.type": s.type, "in.P": s.P,
              "in.L": s.L, "out.delay": out, "out.feats": feats}
        torch.save(fx, os.path.join(HERE, f"{name}.pt"))
        print(name, s.num_nodes, int(s.edge_index.shape[1]), tuple(out.shape), tuple(feats.shape),
              float(out.abs().max()), float(feats.abs().max()))


if __name__ == "__main__":
    main()
