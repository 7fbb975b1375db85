"""C oracle (oracle/hgin_oracle.c) self-checks: published Philox KATs, stable CSR vs numpy, aggregate vs the
reference CPU op (scatter_add_) bit-for-bit, sampler / decoder definitions."""
import numpy as np
import pytest
import torch

from oracle import c_oracle as co
from oracle.pyg_cpu import propagate_sum


def test_philox_known_answers():
    # Random123 kat_vectors, philox4x32_10
    assert list(co.philox4x32_10([0, 0, 0, 0], [0, 0])) == [0x6627e8d5, 0xe169c58d, 0xbc57ac4c, 0x9b00dbd8]
    assert list(co.philox4x32_10([0xffffffff] * 4, [0xffffffff] * 2)) == [0x408f276d, 0x41c83b0e, 0xa20bc7c6,
                                                                           0x6d5451fd]
    assert list(co.philox4x32_10([0x243f6a88, 0x85a308d3, 0x13198a2e, 0x03707344], [0xa4093822, 0x299f31d0])) == \
        [0xd16cfe09, 0x94fdcceb, 0x5001e420, 0x24126ea1]


@pytest.mark.parametrize("E,n_rows,n_cols", [(0, 5, 5), (1, 1, 1), (1000, 37, 50), (50000, 3000, 70), (7, 100, 3)])
@pytest.mark.parametrize("key_row", [0, 1])
def test_csr_stable(E, n_rows, n_cols, key_row):
    rng = np.random.default_rng(E + n_rows)
    kr = rng.integers(0, n_rows, E)
    oc = rng.integers(0, n_cols, E)
    ei = np.stack([oc, kr]) if key_row == 1 else np.stack([kr, oc])
    rowptr, col, perm, st = co.csr_build(ei, key_row, n_rows, n_cols)
    assert st == 0
    order = np.argsort(ei[key_row], kind="stable")
    assert np.array_equal(perm, order)
    assert np.array_equal(col, ei[1 - key_row][order])
    assert np.array_equal(rowptr, np.searchsorted(ei[key_row][order], np.arange(n_rows + 1), side="left"))


def test_csr_out_of_range_flags():
    ei = np.array([[0, 1, 5], [0, 9, 1]])
    _, _, _, st = co.csr_build(ei, 1, 4, 6)  # dst 9 >= 4
    assert st & 1
    _, _, _, st = co.csr_build(ei, 1, 10, 3)  # src 5 >= 3
    assert st == 2


@pytest.mark.parametrize("F", [1, 3, 8, 33])
def test_aggregate_matches_scatter_add(F):
    g = torch.Generator().manual_seed(F)
    n_src, n_dst, E = 400, 250, 6000
    ei = torch.stack([torch.randint(0, n_src, (E,), generator=g), torch.randint(0, n_dst, (E,), generator=g)])
    x = torch.randn(n_src, F, generator=g)
    xd = torch.randn(n_dst, F, generator=g)
    eps = 0.3125
    rowptr, col, perm, _ = co.csr_build(ei.numpy(), 1, n_dst, n_src)
    agg = propagate_sum(x, ei, n_dst)
    assert np.array_equal(co.aggregate(rowptr, col, x.numpy(), None, 0.0, 0), agg.numpy())
    epst = torch.tensor([eps])
    add = agg + (1 + epst) * xd
    assert np.array_equal(co.aggregate(rowptr, col, x.numpy(), xd.numpy(), eps, 1), add.numpy())
    cat = torch.cat((agg, (1 + epst) * xd), 1)
    assert np.array_equal(co.aggregate(rowptr, col, x.numpy(), xd.numpy(), eps, 2), cat.numpy())


def test_neg_sample_definition():
    s = co.neg_sample(1234, 6, 10, 1000)
    for i in range(10):
        c = 6 + i
        x = co.philox4x32_10([c >> 2, 0, 0, 0], [1234, 0])[c & 3]
        assert s[i] == (int(x) * 1000) >> 32
    assert ((s >= 0) & (s < 1000)).all()


def test_dot_decoder_bwd_definition():
    rng = np.random.default_rng(0)
    n_src, n_dst, n, F = 30, 40, 500, 6
    src, dst = rng.integers(0, n_src, n), rng.integers(0, n_dst, n)
    zd = rng.standard_normal((n_dst, F)).astype(np.float32)
    g = rng.standard_normal(n).astype(np.float32)
    rowptr, col, perm, _ = co.csr_build(np.stack([src, dst]), 0, n_src, n_dst)
    gz = co.dot_decode_bwd(rowptr, col, perm, g, zd)
    ref = torch.zeros(n_src, F).index_add_(0, torch.from_numpy(src), torch.from_numpy(g)[:, None] *
                                           torch.from_numpy(zd)[dst])
    assert np.array_equal(gz, ref.numpy())
