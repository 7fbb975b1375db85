"""§8 F4 on the GPU: hgin.qt.QTBaseline against the reference's own QTBaseline outputs (fixtures) and the
CPU oracle.  Integer preparation (positions, the (position, edge)-ordered CSR) and the traffic sums are
bit-exact; the M/M/1/B powers use the device powf, so the outputs are compared within 1e-4 relative."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN
from hgin import _lib, ops
from hgin.qt import QTBaseline, plan
from hgin.qt_data import collate_routes, route_sample
from oracle.qt_cpu import edge_positions, position_groups, qt_baseline, traffic_sum

pytestmark = pytest.mark.gpu
DEV = "cuda"
QT_CASES = ["qt_n6", "qt_n12_f2", "qt_batch3"]


def _fx(case):
    return torch.load(os.path.join(GOLDEN, f"{case}.pt"), weights_only=True)


@pytest.mark.parametrize("case", QT_CASES)
def test_qt_vs_reference_fixture(case):
    fx = _fx(case)

    class D:
        pass

    d = D()
    d.edge_index, d.edge_type, d.type, d.P, d.L = (fx["in.edge_index"], fx["in.edge_type"], fx["in.type"],
                                                   fx["in.P"], fx["in.L"])
    delay, feats = QTBaseline()(d)
    assert delay.device.type == "cpu" and delay.shape == fx["out.delay"].shape and feats.shape == fx["out.feats"].shape
    assert torch.allclose(delay, fx["out.delay"], rtol=1e-4, atol=1e-7)
    assert torch.allclose(feats, fx["out.feats"], rtol=1e-4, atol=1e-7)


@pytest.mark.parametrize("n_nodes,seed", [(6, 1), (15, 3), (30, 4)])
def test_qt_plan_and_traffic_bit_exact(n_nodes, seed):
    s = route_sample(n_nodes, seed=seed)
    pl = plan(s.edge_index, s.edge_type, s.type, DEV)
    sel = s.edge_type == 0
    src, dst = s.edge_index[0, sel], s.edge_index[1, sel]
    pos = edge_positions(src)
    assert torch.equal(pl.pos.cpu().long(), pos)
    groups = position_groups(pos)
    # rows of the CSR list each destination's edges by (position, edge id)
    order = torch.cat(groups) if groups else torch.zeros(0, dtype=torch.long)
    d_sorted = torch.sort(dst[order], stable=True)
    assert torch.equal(pl.csr.col.cpu().long(), order[d_sorted.indices])
    # one traffic pass with arbitrary blocking probabilities: bit-exact against the reference's loop
    g = torch.Generator().manual_seed(seed)
    n = s.num_nodes
    a = torch.zeros(n)
    a[s.type == 0] = s.P[:, 1]
    bp = torch.rand(n, generator=g)
    ref = traffic_sum(src, dst, groups, a, bp)
    val = torch.empty(max(src.numel(), 1), device=DEV)
    t = torch.empty(n, device=DEV)
    a_d, bp_d = a.to(DEV), bp.to(DEV)
    st = ops._stream(a_d)
    _lib.call("hgin_qt_traffic", ops._p(pl.run_ptr), int(pl.run_src.numel()), ops._p(pl.run_src), ops._p(pl.dst),
              ops._p(a_d), ops._p(bp_d), ops._p(val), st)
    _lib.call("hgin_qt_link_sum", ops._p(pl.csr.rowptr), ops._p(pl.csr.col), ops._p(pl.pos), ops._p(val), n,
              ops._p(t), st)
    assert torch.equal(t.cpu(), ref)


def test_qt_large_batch_vs_oracle():
    s = collate_routes([route_sample(int(k), seed=100 + i) for i, k in enumerate(np.random.default_rng(0).integers(20, 40, 16))])
    delay, feats = QTBaseline()(s)
    r_delay, r_feats = qt_baseline(s.edge_index, s.edge_type, s.type, s.P, s.L)
    assert torch.allclose(delay, r_delay, rtol=1e-4, atol=1e-7)
    assert torch.allclose(feats, r_feats, rtol=1e-4, atol=1e-7)
