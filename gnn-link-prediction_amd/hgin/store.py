"""HBM-resident graph store: device-side batch collation and the dict-of-tensors file
format (§8 F2).

Reference data path: every training step, ``torch_geometric.loader.DataLoader(batch_size=8,
shuffle=True)`` (``dataset.py:239-244``) unpickles 8 ``HeteroData`` samples (``dataset.py:146-167``,
``torch.load`` of PyG pickles + the always-on ``normalize``, ``dataset.py:33-58, :165``), collates them on
the host and ``sample.cuda()`` copies the batch (``train.py:28``); the GPU scatter kernels then start from
unsorted COO.

Here the whole dataset lives in HBM (288 GB holds the full GNNet set many times over) as ONE collated
store with global node ids, and each relation's stable CSR (by dst) and CSC (by src) are built once with
``hgin_csr_build``.  A graph's edges are a contiguous block of both sorted orders, so a batch's CSR / CSC is
the concatenation of store slices shifted by (batch offset - store offset) — bit-identical to sorting the
collated batch from scratch.  ``collate(ids)`` emits one "segment copy with shift" descriptor per array
slice (x rows, labels, batch vectors, edge_index, rowptr / col / perm of both directions) and executes all
of them in ONE ``hgin_batched_copy`` launch; the returned ``HeteroGraph`` already carries its CSR / CSC, so
the model never sorts.

File format (F2): ``GraphStore.save`` writes a flat dict of tensors (+ plain-value metadata) loadable with
``torch.load(weights_only=True)`` — no PyG pickles — including the sorted structures, so loading needs no
rebuild.  ``normalize=True`` applies the reference's always-on feature normalisation
(``dataset.py:33-58``) once, at store build, with the same fp32 operations.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
from torch import Tensor

from . import _lib, ops
from .data import EdgeType, HeteroGraph, collate

COPY_F32, COPY_I32_ADD, COPY_I64_ADD, FILL_I64, FILL_I32, COPY_B16 = 0, 1, 2, 3, 4, 5
_COPY_KIND = {4: COPY_F32, 2: COPY_B16}     # feature element size -> copy kind
DESC_DTYPE = np.dtype([("src", "<u8"), ("dst", "<u8"), ("count", "<i8"), ("add", "<i8"), ("kind", "<i4"),
                       ("reserved", "<i4")])
assert DESC_DTYPE.itemsize == 40   # sizeof(hgin_copy_desc)

# dataset.py:33-58 (column, mean, std) per node type of the raw 7/7/3 layout
NORMALIZATION = {
    "link": [(0, 0.3546671, 0.2083346), (1, 0.16771736017268535, 0.1974350417861857),
             (2, 0.09862498490722958, 0.179935315102362), (3, 0.05104, 0.06313), (4, 0.35411, 0.2075),
             (5, 0.00066, 0.00816)],
    "path": [(0, 0.6577772, 0.4192159), (1, 0.6578069, 0.4192953), (2, 0.6578076, 0.4193256),
             (3, 0.20152, 0.18457)],
}


def normalize_reference(x: Dict[str, Tensor]) -> Dict[str, Tensor]:
    """dataset.py:33-58 on a copy of the feature dict (same per-column fp32 tensor ops, same order)."""
    out = {t: v.clone() for t, v in x.items()}
    for t, cols in NORMALIZATION.items():
        if t not in out:
            continue
        for c, mean, std in cols:
            if c < out[t].shape[1]:
                out[t][:, c] = (out[t][:, c] - mean) / std
    return out


class GraphStore:
    def __init__(self, x: Dict[str, Tensor], y: Tensor, edge_index: Dict[EdgeType, Tensor],
                 node_off: Dict[str, np.ndarray], edge_off: Dict[EdgeType, np.ndarray],
                 csr: Dict[EdgeType, ops.Csr], csc: Dict[EdgeType, ops.Csr]):
        self.x, self.y, self.edge_index = x, y, edge_index
        self.node_off, self.edge_off = node_off, edge_off
        self.csr, self.csc = csr, csc
        self.types: List[str] = list(x.keys())
        self.relations: List[EdgeType] = list(edge_index.keys())
        self.device = y.device

    @property
    def num_graphs(self) -> int:
        return len(next(iter(self.node_off.values()))) - 1

    # ------------------------------------------------------------------------------------------ build
    @classmethod
    def build(cls, graphs: Sequence[HeteroGraph], device="cuda", normalize: bool = False) -> "GraphStore":
        if not graphs:
            raise ValueError("GraphStore.build: no graphs")
        big = collate(list(graphs))                    # PyG-style collation restated (hgin.data.collate)
        types = list(big.x.keys())
        node_off = {t: np.concatenate([[0], np.cumsum([g.num_nodes(t) for g in graphs])]).astype(np.int64)
                    for t in types}
        edge_off = {r: np.concatenate([[0], np.cumsum([int(g.edge_index[r].size(1)) for g in graphs])]).astype(
            np.int64) for r in big.edge_index}
        x = normalize_reference(big.x) if normalize else big.x
        x = {t: v.to(device).contiguous() for t, v in x.items()}
        y = big.y.to(device).contiguous()
        ei = {r: e.to(device).contiguous() for r, e in big.edge_index.items()}
        csr, csc = {}, {}
        for (s, rel, d), e in ei.items():
            n_s, n_d = int(node_off[s][-1]), int(node_off[d][-1])
            csr[(s, rel, d)] = ops.build_csr(e, 1, n_d, n_s)
            csc[(s, rel, d)] = ops.build_csr(e, 0, n_s, n_d, validate=False)
        return cls(x, y, ei, node_off, edge_off, csr, csc)

    # ------------------------------------------------------------------------------------ F2 format
    def state_dict(self) -> dict:
        sd = {"meta": {"format": "hgin-graph-store/1", "types": self.types,
                       "relations": ["__".join(r) for r in self.relations]}}
        for t in self.types:
            sd[f"x.{t}"] = self.x[t].cpu()
            sd[f"node_off.{t}"] = torch.from_numpy(self.node_off[t])
        sd["y"] = self.y.cpu()
        for r in self.relations:
            k = "__".join(r)
            sd[f"ei.{k}"] = self.edge_index[r].cpu()
            sd[f"edge_off.{k}"] = torch.from_numpy(self.edge_off[r])
            for name, c in (("csr", self.csr[r]), ("csc", self.csc[r])):
                sd[f"{name}.{k}.rowptr"] = c.rowptr.cpu()
                sd[f"{name}.{k}.col"] = c.col.cpu()
                sd[f"{name}.{k}.perm"] = c.perm.cpu()
        return sd

    def save(self, path: str) -> None:
        torch.save(self.state_dict(), path)

    @classmethod
    def load(cls, path: str, device="cuda") -> "GraphStore":
        sd = torch.load(path, weights_only=True)
        return cls.from_state_dict(sd, device)

    @classmethod
    def from_state_dict(cls, sd: dict, device="cuda") -> "GraphStore":
        meta = sd["meta"]
        if meta.get("format") != "hgin-graph-store/1":
            raise ValueError(f"not an hgin graph store: {meta.get('format')!r}")
        types = list(meta["types"])
        rels = [tuple(k.split("__")) for k in meta["relations"]]
        x = {t: sd[f"x.{t}"].to(device) for t in types}
        node_off = {t: sd[f"node_off.{t}"].numpy() for t in types}
        ei, edge_off, csr, csc = {}, {}, {}, {}
        for r in rels:
            k = "__".join(r)
            ei[r] = sd[f"ei.{k}"].to(device)
            edge_off[r] = sd[f"edge_off.{k}"].numpy()
            n_s, n_d = int(node_off[r[0]][-1]), int(node_off[r[2]][-1])
            csr[r] = ops.Csr(*(sd[f"csr.{k}.{f}"].to(device) for f in ("rowptr", "col", "perm")), n_d, n_s)
            csc[r] = ops.Csr(*(sd[f"csc.{k}.{f}"].to(device) for f in ("rowptr", "col", "perm")), n_s, n_d)
        return cls(x, sd["y"].to(device), ei, node_off, edge_off, csr, csc)

    # ------------------------------------------------------------------------------------- F1 collate
    def plan(self, ids: Sequence[int]):
        """Batch sizes and per-graph (store offset, batch offset) pairs — host-side, O(#graphs)."""
        ids = np.asarray(ids, dtype=np.int64)
        if ids.size == 0:
            raise ValueError("collate: empty batch")
        if ids.min() < 0 or ids.max() >= self.num_graphs:
            raise IndexError("collate: graph id out of range")
        nodes = {t: self.node_off[t][ids + 1] - self.node_off[t][ids] for t in self.types}
        edges = {r: self.edge_off[r][ids + 1] - self.edge_off[r][ids] for r in self.relations}
        b_node = {t: np.concatenate([[0], np.cumsum(n)]) for t, n in nodes.items()}
        b_edge = {r: np.concatenate([[0], np.cumsum(n)]) for r, n in edges.items()}
        return ids, nodes, edges, b_node, b_edge

    def collate(self, ids: Sequence[int]) -> HeteroGraph:
        """A new exactly-sized batch of the graphs ``ids`` (in that order), CSR / CSC attached."""
        ids, nodes, edges, b_node, b_edge = self.plan(ids)
        dev = self.device
        x_out = {t: torch.empty(int(b_node[t][-1]), self.x[t].shape[1], dtype=self.x[t].dtype, device=dev)
                 for t in self.types}
        batch_out = {t: torch.empty(int(b_node[t][-1]), dtype=torch.long, device=dev) for t in self.types}
        y_out = torch.empty(int(b_node["path"][-1]), dtype=self.y.dtype, device=dev)
        ei_out, csr_out, csc_out = {}, {}, {}
        for r in self.relations:
            s, _, d = r
            E = int(b_edge[r][-1])
            n_s, n_d = int(b_node[s][-1]), int(b_node[d][-1])
            ei_out[r] = torch.empty(2, E, dtype=torch.long, device=dev)
            csr_out[r] = ops.Csr(torch.empty(n_d + 1, dtype=torch.int32, device=dev),
                                 torch.empty(E, dtype=torch.int32, device=dev),
                                 torch.empty(E, dtype=torch.int32, device=dev), n_d, n_s)
            csc_out[r] = ops.Csr(torch.empty(n_s + 1, dtype=torch.int32, device=dev),
                                 torch.empty(E, dtype=torch.int32, device=dev),
                                 torch.empty(E, dtype=torch.int32, device=dev), n_s, n_d)
        self._launch(ids, nodes, edges, b_node, b_edge, x_out, batch_out, y_out, ei_out, csr_out, csc_out, None)
        for r in self.relations:
            s, _, d = r
            ops.attach_relation_graph(ei_out[r], int(b_node[s][-1]), int(b_node[d][-1]), csr_out[r], csc_out[r])
        return HeteroGraph(x_out, ei_out, y_out, batch_out)

    # ------------------------------------------------------------------- static-shape padded batches
    def padded_batch(self, batch_size: int) -> "PaddedBatch":
        """Static buffers able to hold any ``batch_size`` graphs of this store (capacity = batch_size x the
        largest graph, per node type and relation).  ``collate_into`` refills them in place, so a training
        step over them can be captured once into a hipGraph and replayed (hgin/graphs.py)."""
        dev = self.device
        cap_n = {t: int(batch_size * np.diff(self.node_off[t]).max()) for t in self.types}
        cap_e = {r: int(batch_size * np.diff(self.edge_off[r]).max()) for r in self.relations}
        x = {t: torch.zeros(cap_n[t], self.x[t].shape[1], dtype=self.x[t].dtype, device=dev) for t in self.types}
        batch = {t: torch.zeros(cap_n[t], dtype=torch.long, device=dev) for t in self.types}
        y = torch.ones(cap_n["path"], dtype=self.y.dtype, device=dev)
        ei, csr, csc = {}, {}, {}
        for r in self.relations:
            s, _, d = r
            E = cap_e[r]
            ei[r] = torch.zeros(2, E, dtype=torch.long, device=dev)
            csr[r] = ops.Csr(torch.zeros(cap_n[d] + 1, dtype=torch.int32, device=dev),
                             torch.zeros(E, dtype=torch.int32, device=dev),
                             torch.zeros(E, dtype=torch.int32, device=dev), cap_n[d], cap_n[s])
            csc[r] = ops.Csr(torch.zeros(cap_n[s] + 1, dtype=torch.int32, device=dev),
                             torch.zeros(E, dtype=torch.int32, device=dev),
                             torch.zeros(E, dtype=torch.int32, device=dev), cap_n[s], cap_n[d])
            ops.attach_relation_graph(ei[r], cap_n[s], cap_n[d], csr[r], csc[r])
        m_valid = torch.zeros(1, dtype=torch.int32, device=dev)
        # per-graph node offsets [path | link | node] x (batch_size + 1) (the fused small-batch step's graph ranges)
        goff = torch.zeros(3 * (batch_size + 1), dtype=torch.int32, device=dev)
        return PaddedBatch(x, ei, y, batch, m_valid, csr, csc, batch_size, goff)

    def collate_into(self, ids: Sequence[int], out: "PaddedBatch") -> "PaddedBatch":
        """Refill ``out`` with the graphs ``ids``: valid rows first; the CSR / CSC rows past the batch get
        empty ranges (padding vertices are isolated) and ``out.m_valid`` = the batch's path count, so the
        fused loss covers exactly the batch.  One batched-copy launch, no allocation, no host sync."""
        ids, nodes, edges, b_node, b_edge = self.plan(ids)
        if len(ids) > out.batch_size:
            raise ValueError(f"collate_into: {len(ids)} graphs > batch capacity {out.batch_size}")
        self._launch(ids, nodes, edges, b_node, b_edge, out.x, out.batch, out.y, out.edge_index, out.csr, out.csc,
                     out.m_valid, out.goff, out.batch_size)
        return out

    def _launch(self, ids, nodes, edges, b_node, b_edge, x_out, batch_out, y_out, ei_out, csr_out, csc_out,
                m_valid, goff=None, cap_graphs: int = 0) -> None:
        descs: List[tuple] = []

        def ptr(t: Tensor, elem_off: int) -> int:
            return t.data_ptr() + int(elem_off) * t.element_size()

        for t in self.types:
            F = self.x[t].shape[1]
            for j, g in enumerate(ids):
                n = int(nodes[t][j])
                if n == 0:
                    continue
                s_off, b_off = int(self.node_off[t][g]), int(b_node[t][j])
                descs.append((ptr(self.x[t], s_off * F), ptr(x_out[t], b_off * F), n * F, 0,
                              _COPY_KIND[self.x[t].element_size()]))
                descs.append((0, ptr(batch_out[t], b_off), n, j, FILL_I64))
        for j, g in enumerate(ids):
            n = int(nodes["path"][j])
            if n:
                descs.append((ptr(self.y, self.node_off["path"][g]), ptr(y_out, b_node["path"][j]), n, 0, COPY_F32))

        for r in self.relations:
            s, _, d = r
            E = int(b_edge[r][-1])
            n_s, n_d = int(b_node[s][-1]), int(b_node[d][-1])
            e, cr, cc = ei_out[r], csr_out[r], csc_out[r]
            e_cap = e.shape[1]                    # row stride of the [2, E] edge_index buffer
            se, sc, ss = self.edge_index[r], self.csr[r], self.csc[r]
            E_store = se.shape[1]
            for j, g in enumerate(ids):
                m = int(edges[r][j])
                es, eb = int(self.edge_off[r][g]), int(b_edge[r][j])
                ds_s, db_s = int(self.node_off[s][g]), int(b_node[s][j])
                ds_d, db_d = int(self.node_off[d][g]), int(b_node[d][j])
                nd, ns = int(nodes[d][j]), int(nodes[s][j])
                if m:
                    descs.append((ptr(se, es), ptr(e, eb), m, db_s - ds_s, COPY_I64_ADD))              # src row
                    descs.append((ptr(se, E_store + es), ptr(e, e_cap + eb), m, db_d - ds_d, COPY_I64_ADD))  # dst
                    descs.append((ptr(sc.col, es), ptr(cr.col, eb), m, db_s - ds_s, COPY_I32_ADD))
                    descs.append((ptr(sc.perm, es), ptr(cr.perm, eb), m, eb - es, COPY_I32_ADD))
                    descs.append((ptr(ss.col, es), ptr(cc.col, eb), m, db_d - ds_d, COPY_I32_ADD))
                    descs.append((ptr(ss.perm, es), ptr(cc.perm, eb), m, eb - es, COPY_I32_ADD))
                if nd:
                    descs.append((ptr(sc.rowptr, ds_d), ptr(cr.rowptr, db_d), nd, eb - es, COPY_I32_ADD))
                if ns:
                    descs.append((ptr(ss.rowptr, ds_s), ptr(cc.rowptr, db_s), ns, eb - es, COPY_I32_ADD))
            # rowptr[n .. capacity] = E: the last row's end, and empty rows for padding vertices
            descs.append((0, ptr(cr.rowptr, n_d), cr.rowptr.numel() - n_d, E, FILL_I32))
            descs.append((0, ptr(cc.rowptr, n_s), cc.rowptr.numel() - n_s, E, FILL_I32))
        if m_valid is not None:
            descs.append((0, ptr(m_valid, 0), 1, int(b_node["path"][-1]), FILL_I32))
        if goff is not None:   # graph j's rows of type t: [goff[t][j], goff[t][j + 1]); graphs past the batch: empty
            for ti, t in enumerate(("path", "link", "node")):
                if t not in b_node:
                    continue
                for j in range(cap_graphs + 1):
                    v = int(b_node[t][min(j, len(ids))])
                    descs.append((0, ptr(goff, ti * (cap_graphs + 1) + j), 1, v, FILL_I32))

        arr = np.zeros(len(descs), dtype=DESC_DTYPE)
        if descs:
            cols = list(zip(*descs))
            for name, vals in zip(("src", "dst", "count", "add", "kind"), cols):
                arr[name] = vals
        host = torch.from_numpy(arr.view(np.uint8)).pin_memory()
        dev_desc = host.to(self.device, non_blocking=True)
        max_count = int(arr["count"].max()) if len(arr) else 0
        _lib.call("hgin_batched_copy", ops._p(dev_desc), len(arr), max_count, ops._stream(dev_desc))


@dataclass
class PaddedBatch(HeteroGraph):
    """Static-capacity batch buffers (GraphStore.padded_batch): rows past the current batch are isolated
    padding vertices; ``m_valid`` (device int32) holds the current batch's path count for the fused loss."""
    m_valid: Tensor = None
    csr: Dict[EdgeType, ops.Csr] = None
    csc: Dict[EdgeType, ops.Csr] = None
    batch_size: int = 0
    goff: Tensor = None   # int32 [3 * (batch_size + 1)]: per-graph node offsets, path | link | node
