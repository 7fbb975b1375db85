"""Host-side pieces of the §8 F1/F2 graph store (no GPU): descriptor layout vs the C ABI struct, the batch
plan, and the reference normalisation restatement (dataset.py:33-58)."""
import ctypes

import numpy as np
import pytest
import torch

from hgin.store import DESC_DTYPE, NORMALIZATION, GraphStore, normalize_reference


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
