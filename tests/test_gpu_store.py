"""§8 F1/F2 on the GPU: device batch collation out of an HBM-resident GraphStore.

The checker is hgin.data.collate (the PyG Batch.from_data_list restatement, dataset.py:239-244) on the host
plus the C oracle's stable CSR build (oracle/hgin_oracle.c) of the collated edge_index — every collated array
must be bit-identical, including the CSR / CSC the store assembles without sorting.
"""
import dataclasses

import numpy as np
import pytest
import torch

from hgin import HetroGIN, ops
from hgin.data import CONFIGS, REL_PN, HeteroGraph, collate, scaled_config, synthetic_graph
from hgin.store import GraphStore, normalize_reference
from oracle import c_oracle as co

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _graphs(n, seed=0, empty_rel_at=None):
    base = CONFIGS["cfg1"]
    rng = np.random.default_rng(seed)
    out = []
    for i in range(n):
        cfg = scaled_config(base, float(rng.uniform(0.05, 0.4)), name=f"g{i}")
        cfg = dataclasses.replace(cfg, e_pn=max(1, cfg.e_ln))
        g = synthetic_graph(cfg, seed=seed * 1000 + i)
        if empty_rel_at is not None and i == empty_rel_at:
            g.edge_index[REL_PN] = torch.empty(2, 0, dtype=torch.long)
        out.append(g)
    return out


def _check_batch(b: HeteroGraph, ref: HeteroGraph):
    for t in ref.x:
        assert torch.equal(b.x[t].cpu(), ref.x[t]), t
        assert torch.equal(b.batch[t].cpu(), ref.batch[t]), t
    assert torch.equal(b.y.cpu(), ref.y)
    for r, e in ref.edge_index.items():
        assert torch.equal(b.edge_index[r].cpu(), e), r
        n_s, n_d = ref.x[r[0]].shape[0], ref.x[r[2]].shape[0]
        rg = ops.relation_graph(b.edge_index[r], n_s, n_d)
        for key_row, c, n_rows, n_cols in ((1, rg._csr, n_d, n_s), (0, rg._csc, n_s, n_d)):
            assert c is not None, "collate must attach prebuilt CSR / CSC"
            rp, col, perm, st = co.csr_build(e.numpy(), key_row, n_rows, n_cols)
            assert st == 0
            assert np.array_equal(c.rowptr.cpu().numpy(), rp), (r, key_row)
            assert np.array_equal(c.col.cpu().numpy(), col), (r, key_row)
            assert np.array_equal(c.perm.cpu().numpy(), perm), (r, key_row)


@pytest.mark.parametrize("ids", [[0], [3, 1, 4, 1, 5, 9, 2, 6], list(range(12)), [11, 0, 7]])
def test_collate_bit_exact(ids):
    graphs = _graphs(12, seed=1, empty_rel_at=4)
    store = GraphStore.build(graphs, device=DEV)
    b = store.collate(ids)
    torch.cuda.synchronize()
    _check_batch(b, collate([graphs[i] for i in ids]))


def test_collate_store_csr_matches_fresh_build():
    graphs = _graphs(6, seed=2)
    store = GraphStore.build(graphs, device=DEV)
    big = collate(graphs)
    for r, e in big.edge_index.items():
        n_s, n_d = big.x[r[0]].shape[0], big.x[r[2]].shape[0]
        rp, col, perm, _ = co.csr_build(e.numpy(), 1, n_d, n_s)
        assert np.array_equal(store.csr[r].rowptr.cpu().numpy(), rp)
        assert np.array_equal(store.csr[r].perm.cpu().numpy(), perm)


def test_collate_model_output_identical():
    graphs = _graphs(10, seed=3)
    store = GraphStore.build(graphs, device=DEV)
    cfg = CONFIGS["cfg1"]
    torch.manual_seed(1997)
    model = HetroGIN(**cfg.model_kwargs({"link": 7, "path": 7, "node": 3})).to(DEV)
    ids = [7, 2, 9, 0, 4, 4, 1, 8]
    b = store.collate(ids)
    ref = collate([graphs[i] for i in ids]).to(DEV)     # fresh tensors -> CSR / CSC built by sorting
    out_b = model(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    out_r = model(ref.x_dict(), ref.edge_index_dict(), ref.batch["path"])
    assert torch.equal(out_b, out_r)
    g_b = torch.autograd.grad(out_b.sum(), list(model.parameters()), allow_unused=True)
    g_r = torch.autograd.grad(out_r.sum(), list(model.parameters()), allow_unused=True)
    for a, c in zip(g_b, g_r):
        assert (a is None) == (c is None)
        if a is not None:
            assert torch.equal(a, c)


def test_save_load_roundtrip(tmp_path):
    graphs = _graphs(5, seed=4)
    store = GraphStore.build(graphs, device=DEV, normalize=True)
    path = str(tmp_path / "store.pt")
    store.save(path)
    loaded = GraphStore.load(path, device=DEV)
    ids = [4, 0, 2]
    a, b = store.collate(ids), loaded.collate(ids)
    torch.cuda.synchronize()
    for t in a.x:
        assert torch.equal(a.x[t], b.x[t])
    for r in a.edge_index:
        assert torch.equal(a.edge_index[r], b.edge_index[r])
    # normalisation applied once at build, exactly as dataset.py:33-58 does per sample
    ref = collate([HeteroGraph(normalize_reference(g.x), g.edge_index, g.y, g.batch) for g in [graphs[i] for i in ids]])
    _check_batch(b, ref)


def test_collate_rejects_bad_ids():
    store = GraphStore.build(_graphs(3, seed=5), device=DEV)
    with pytest.raises(IndexError):
        store.collate([0, 3])
    with pytest.raises(ValueError):
        store.collate([])
