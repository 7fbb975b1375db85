"""Host-side pieces of the §8 F1/F2 graph store (no GPU): descriptor layout vs the C ABI struct, the batch
plan, and the reference normalisation restatement (dataset.py:33-58)."""
import ctypes

import numpy as np
import pytest
import torch

from hgin.store import DESC_DTYPE, NORMALIZATION, GraphStore, PaddedBatch, _DescPlan, normalize_reference


class _CopyDesc(ctypes.Structure):      # include/hgin.h: hgin_copy_desc
    _fields_ = [("src", ctypes.c_void_p), ("dst", ctypes.c_void_p), ("count", ctypes.c_int64),
                ("add", ctypes.c_int64), ("kind", ctypes.c_int32), ("reserved", ctypes.c_int32)]


def test_descriptor_layout_matches_c_struct():
    assert DESC_DTYPE.itemsize == ctypes.sizeof(_CopyDesc)
    for name, *_ in _CopyDesc._fields_:
        assert DESC_DTYPE.fields[name][1] == getattr(_CopyDesc, name).offset, name


def test_copy_kinds_match_header():
    import re
    import os
    from conftest import ROOT
    hdr = open(os.path.join(ROOT, "include", "hgin.h")).read()
    from hgin import store
    for name, val in (("HGIN_COPY_F32", store.COPY_F32), ("HGIN_COPY_I32_ADD", store.COPY_I32_ADD),
                      ("HGIN_COPY_I64_ADD", store.COPY_I64_ADD), ("HGIN_FILL_I64", store.FILL_I64),
                      ("HGIN_FILL_I32", store.FILL_I32), ("HGIN_COPY_B16", store.COPY_B16)):
        m = re.search(rf"#define\s+{name}\s+(\d+)", hdr)
        assert m and int(m.group(1)) == val, name


def _offset_store(node_counts, edge_counts):
    node_off = {t: np.concatenate([[0], np.cumsum(c)]).astype(np.int64) for t, c in node_counts.items()}
    edge_off = {r: np.concatenate([[0], np.cumsum(c)]).astype(np.int64) for r, c in edge_counts.items()}
    x = {t: torch.zeros(int(o[-1]), 2) for t, o in node_off.items()}
    ei = {r: torch.zeros(2, int(o[-1]), dtype=torch.long) for r, o in edge_off.items()}
    return GraphStore(x, torch.zeros(int(node_off["path"][-1])), ei, node_off, edge_off, {}, {})


def test_plan_offsets():
    rel = ("path", "uses", "link")
    st = _offset_store({"path": [3, 5, 2], "link": [1, 4, 0]}, {rel: [6, 0, 9]})
    ids, nodes, edges, b_node, b_edge = st.plan([2, 0, 2])
    assert list(nodes["path"]) == [2, 3, 2] and list(b_node["path"]) == [0, 2, 5, 7]
    assert list(b_node["link"]) == [0, 0, 1, 1]
    assert list(edges[rel]) == [9, 6, 9] and list(b_edge[rel]) == [0, 9, 15, 24]
    with pytest.raises(IndexError):
        st.plan([3])
    with pytest.raises(IndexError):
        st.plan([-1])
    with pytest.raises(ValueError):
        st.plan([])


def test_normalize_reference_columns():
    torch.manual_seed(0)
    x = {"link": torch.rand(5, 7), "path": torch.rand(4, 7), "node": torch.rand(3, 3)}
    out = normalize_reference(x)
    assert torch.equal(out["node"], x["node"])
    assert torch.equal(out["link"][:, 6], x["link"][:, 6])
    assert torch.equal(out["path"][:, 4:], x["path"][:, 4:])
    c, mean, std = NORMALIZATION["link"][2]
    assert torch.equal(out["link"][:, c], (x["link"][:, c] - mean) / std)
    assert not torch.equal(out["link"], x["link"])      # input untouched, output normalised


def test_normalize_reference_equals_reference_executed_fixture():
    """F2 pinned to the reference itself: tests/golden/normalize_ref.pt was made by executing dataset.py:33-58
    (GNN21Dataset.normalize) on collated cfg1 features plus extreme values; normalize_reference reproduces it
    bit for bit, every node type and column."""
    from conftest import load_fixture
    fx = load_fixture("normalize_ref")
    x = {t: fx[f"in.x.{t}"] for t in ("path", "link", "node")}
    out = normalize_reference(x)
    for t in x:
        assert torch.equal(out[t], fx[f"out.x.{t}"]), t
        assert torch.equal(x[t], fx[f"in.x.{t}"]), t           # the input dict is not modified


def _emulate_batched_copy(arr):
    """csrc/hgin_collate.hip's hgin_batched_copy restated on host memory (CPU tensors' addresses)."""
    from hgin import store
    size = {store.COPY_F32: 4, store.COPY_B16: 2, store.COPY_I32_ADD: 4, store.COPY_I64_ADD: 8,
            store.FILL_I64: 8, store.FILL_I32: 4}
    ctype = {4: ctypes.c_int32, 8: ctypes.c_int64, 2: ctypes.c_int16}
    for d in arr:
        n, k, add = int(d["count"]), int(d["kind"]), int(d["add"])
        if n == 0:
            continue
        ct = ctype[size[k]]
        dst = np.ctypeslib.as_array((ct * n).from_address(int(d["dst"])))
        if k in (store.FILL_I64, store.FILL_I32):
            dst[:] = add
            continue
        src = np.ctypeslib.as_array((ct * n).from_address(int(d["src"])))
        dst[:] = src + add if k in (store.COPY_I32_ADD, store.COPY_I64_ADD) else src


def test_batch_descriptors_fill_the_padded_batch():
    """The per-graph descriptor tables (GraphStore._template / _descriptors) against the collation they stand for:
    host tensors stand in for device buffers and the batched copy is emulated on them; every buffer of the padded
    batch equals the graphs' rows concatenated with the batch's index shifts (PyG's collate, hgin.data.collate)."""
    from hgin import ops
    rng = np.random.default_rng(0)
    types = ("path", "link", "node")
    rels = (("path", "uses", "link"), ("link", "includes", "path"), ("node", "has", "link"))
    G = 5
    nc = {t: rng.integers(0, 6, G) for t in types}
    nc["path"][0] = 3
    ec = {r: rng.integers(0, 9, G) for r in rels}
    node_off = {t: np.concatenate([[0], np.cumsum(c)]).astype(np.int64) for t, c in nc.items()}
    edge_off = {r: np.concatenate([[0], np.cumsum(c)]).astype(np.int64) for r, c in ec.items()}
    x = {t: torch.randn(int(node_off[t][-1]), 3) for t in types}
    y = torch.rand(int(node_off["path"][-1]))
    ei, csr, csc = {}, {}, {}
    for r in rels:
        s, _, d = r
        E = int(edge_off[r][-1])
        ei[r] = torch.randint(0, 50, (2, E))
        csr[r] = ops.Csr(torch.randint(0, 50, (int(node_off[d][-1]) + 1,), dtype=torch.int32),
                         torch.randint(0, 50, (E,), dtype=torch.int32), torch.randint(0, 50, (E,), dtype=torch.int32),
                         int(node_off[d][-1]), int(node_off[s][-1]))
        csc[r] = ops.Csr(torch.randint(0, 50, (int(node_off[s][-1]) + 1,), dtype=torch.int32),
                         torch.randint(0, 50, (E,), dtype=torch.int32), torch.randint(0, 50, (E,), dtype=torch.int32),
                         int(node_off[s][-1]), int(node_off[d][-1]))
    st = GraphStore(x, y, ei, node_off, edge_off, csr, csc)
    cap = 4
    cap_n = {t: int(cap * nc[t].max()) for t in types}
    cap_e = {r: int(cap * ec[r].max()) for r in rels}
    for ids in ([2, 0, 2], [4], [1, 3, 0, 2]):
        xo = {t: torch.full((cap_n[t], 3), -7.0) for t in types}
        bo = {t: torch.full((cap_n[t],), -7, dtype=torch.long) for t in types}
        yo = torch.full((cap_n["path"],), -7.0)
        eo = {r: torch.full((2, cap_e[r]), -7, dtype=torch.long) for r in rels}
        mk = lambda n, e: ops.Csr(torch.full((n + 1,), -7, dtype=torch.int32), torch.full((e,), -7, dtype=torch.int32),  # noqa: E731
                                  torch.full((e,), -7, dtype=torch.int32), n, 0)
        cro = {r: mk(cap_n[r[2]], cap_e[r]) for r in rels}
        cco = {r: mk(cap_n[r[0]], cap_e[r]) for r in rels}
        mv = torch.zeros(1, dtype=torch.int32)
        goff = torch.full((3 * (cap + 1),), -7, dtype=torch.int32)
        arr = st._descriptors(ids, xo, bo, yo, eo, cro, cco, mv, goff, cap)
        # collate_into's fast table (_DescPlan: output-side constants precomputed, written into a ring slot's
        # view): entry for entry the same table
        plan = _DescPlan(st, PaddedBatch(xo, eo, yo, bo, mv, cro, cco, cap, goff))
        view = np.zeros(plan.max_bytes // DESC_DTYPE.itemsize + 3, dtype=DESC_DTYPE)
        view["reserved"] = -1
        n, max_count = plan.fill(np.asarray(ids, dtype=np.int64), view)
        assert n == len(arr) and max_count == int(arr["count"].max())
        assert view[:n].tobytes() == arr.tobytes()
        _emulate_batched_copy(arr)
        b = {t: np.concatenate([[0], np.cumsum([nc[t][g] for g in ids])]) for t in types}
        be = {r: np.concatenate([[0], np.cumsum([ec[r][g] for g in ids])]) for r in rels}
        for t in types:
            n = int(b[t][-1])
            want = torch.cat([x[t][node_off[t][g]:node_off[t][g + 1]] for g in ids])
            assert torch.equal(xo[t][:n], want), t
            assert bo[t][:n].tolist() == [j for j, g in enumerate(ids) for _ in range(nc[t][g])]
            assert (xo[t][n:] == -7).all()
        assert torch.equal(yo[:int(b["path"][-1])], torch.cat([y[node_off["path"][g]:node_off["path"][g + 1]]
                                                                for g in ids]))
        assert mv.item() == b["path"][-1]
        for ti, t in enumerate(types):
            assert goff[ti * (cap + 1):(ti + 1) * (cap + 1)].tolist() == [int(b[t][min(j, len(ids))])
                                                                          for j in range(cap + 1)]
        for r in rels:
            s, _, d = r
            E = int(be[r][-1])
            seg = lambda g: slice(int(edge_off[r][g]), int(edge_off[r][g + 1]))  # noqa: E731
            sh = lambda t, j, g: int(b[t][j] - node_off[t][g])  # noqa: E731
            want_ei = torch.cat([ei[r][:, seg(g)] + torch.tensor([[sh(s, j, g)], [sh(d, j, g)]])
                                 for j, g in enumerate(ids)], 1)
            assert torch.equal(eo[r][:, :E], want_ei), r
            for out, src, shc, rt in ((cro[r], csr[r], s, d), (cco[r], csc[r], d, s)):
                assert out.col[:E].tolist() == [int(v) + sh(shc, j, g) for j, g in enumerate(ids)
                                                for v in src.col[seg(g)]]
                assert out.perm[:E].tolist() == [int(v) + int(be[r][j] - edge_off[r][g]) for j, g in enumerate(ids)
                                                 for v in src.perm[seg(g)]]
                n = int(b[rt][-1])
                assert out.rowptr[:n].tolist() == [int(v) + int(be[r][j] - edge_off[r][g])
                                                   for j, g in enumerate(ids)
                                                   for v in src.rowptr[node_off[rt][g]:node_off[rt][g + 1]]]
                assert (out.rowptr[n:] == E).all()
