"""The queueing-theory baseline oracle (oracle/qt_cpu.py) against the reference's own QTBaseline outputs
(tests/golden/qt_*.pt, produced by tests/golden/make_golden_qt.py) — bit for bit."""
import os

import pytest
import torch

from conftest import GOLDEN
from oracle.qt_cpu import edge_positions, qt_baseline

QT_CASES = ["qt_n6", "qt_n12_f2", "qt_batch3"]


def _fx(case):
    return torch.load(os.path.join(GOLDEN, f"{case}.pt"), weights_only=True)


@pytest.mark.parametrize("case", QT_CASES)
def test_qt_oracle_bit_exact(case):
    fx = _fx(case)
    delay, feats = qt_baseline(fx["in.edge_index"], fx["in.edge_type"], fx["in.type"], fx["in.P"], fx["in.L"])
    assert torch.equal(delay, fx["out.delay"])
    assert torch.equal(feats, fx["out.feats"])


def test_edge_positions():
    src = torch.tensor([3, 3, 3, 1, 1, 7, 3, 3])
    assert edge_positions(src).tolist() == [0, 1, 2, 0, 1, 0, 0, 1]
    assert edge_positions(torch.zeros(0, dtype=torch.long)).numel() == 0
