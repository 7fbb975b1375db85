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

import ctypes
import weakref

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
        ids = np.asarray(ids, dtype=np.int64)
        if ids.size == 0:
            raise ValueError("collate: empty batch")
        if ids.min() < 0 or ids.max() >= self.num_graphs:
            raise IndexError("collate: graph id out of range")
        if len(ids) > out.batch_size:
            raise ValueError(f"collate_into: {len(ids)} graphs > batch capacity {out.batch_size}")
        # the table's output-side constants are computed once per padded batch (_DescPlan) and the table is written
        # straight into the device-readable ring slot: the per-batch host work is what bounds this step at cfg1
        # sizes (tools/sb_host.py)
        plan = out.__dict__.get("_hgin_desc_plan")
        if plan is None or plan.store is not self:
            plan = out._hgin_desc_plan = _DescPlan(self, out)
        slot = self._desc_slot(plan.max_bytes)
        n, max_count = plan.fill(ids, slot[3])
        stream = torch.cuda.current_stream(self.device)
        _lib.call("hgin_batched_copy", ctypes.c_void_p(slot[0]), n, max_count, ctypes.c_void_p(stream.cuda_stream))
        slot[2].record(stream)
        return out

    def _template(self):
        """Per-graph copy-descriptor tables (built once per store): for every graph and descriptor group (one group
        per buffer and relation) the source pointer, the count and the store-side part of the index shift, plus per
        group how its destination and shift follow the batch offsets.  A batch then costs a handful of numpy ops
        on a (graphs x groups) table instead of a Python loop per graph and buffer.  The store's tensors are fixed
        at construction, so the table is built on first use and kept."""
        tpl = getattr(self, "_tpl", None)
        if tpl is not None:
            return tpl
        col = {t: i for i, t in enumerate(self.types)}
        col.update({r: len(self.types) + i for i, r in enumerate(self.relations)})
        G = self.num_graphs
        cnt_tab = np.zeros((G, len(col)), dtype=np.int64)
        for t in self.types:
            cnt_tab[:, col[t]] = np.diff(self.node_off[t])
        for r in self.relations:
            cnt_tab[:, col[r]] = np.diff(self.edge_off[r])
        no = {t: self.node_off[t][:-1] for t in self.types}
        eo = {r: self.edge_off[r][:-1] for r in self.relations}
        zero = np.zeros(G, dtype=np.int64)

        def P(t: Tensor, off):
            return np.int64(t.data_ptr()) + off * t.element_size()

        # (src pointer [G], count [G], shift [G], dst selector, dst column, dst rows -> elements, dst constant
        #  selector, shift column or -1, shift += j, kind)
        spec = []
        for t in self.types:
            F = self.x[t].shape[1]
            spec.append((P(self.x[t], no[t] * F), cnt_tab[:, col[t]] * F, zero, ("x", t), col[t], F, None, -1, 0,
                         _COPY_KIND[self.x[t].element_size()]))
            spec.append((zero, cnt_tab[:, col[t]], zero, ("batch", t), col[t], 1, None, -1, 1, FILL_I64))
        spec.append((P(self.y, no["path"]), cnt_tab[:, col["path"]], zero, ("y", None), col["path"], 1, None, -1, 0,
                     COPY_F32))
        for r in self.relations:
            s_, _, d = r
            se, sc, ss = self.edge_index[r], self.csr[r], self.csc[r]
            E_store = se.shape[1]
            m, cr_ = cnt_tab[:, col[r]], col[r]
            spec += [
                (P(se, eo[r]), m, -no[s_], ("ei", r), cr_, 1, None, col[s_], 0, COPY_I64_ADD),          # src row
                (P(se, E_store + eo[r]), m, -no[d], ("ei", r), cr_, 1, "e_cap", col[d], 0, COPY_I64_ADD),  # dst
                (P(sc.col, eo[r]), m, -no[s_], ("csr.col", r), cr_, 1, None, col[s_], 0, COPY_I32_ADD),
                (P(sc.perm, eo[r]), m, -eo[r], ("csr.perm", r), cr_, 1, None, cr_, 0, COPY_I32_ADD),
                (P(ss.col, eo[r]), m, -no[d], ("csc.col", r), cr_, 1, None, col[d], 0, COPY_I32_ADD),
                (P(ss.perm, eo[r]), m, -eo[r], ("csc.perm", r), cr_, 1, None, cr_, 0, COPY_I32_ADD),
                (P(sc.rowptr, no[d]), cnt_tab[:, col[d]], -eo[r], ("csr.rowptr", r), col[d], 1, None, cr_, 0,
                 COPY_I32_ADD),
                (P(ss.rowptr, no[s_]), cnt_tab[:, col[s_]], -eo[r], ("csc.rowptr", r), col[s_], 1, None, cr_, 0,
                 COPY_I32_ADD),
            ]
        tab = {
            "col": col, "cnt": cnt_tab,
            "src": np.stack([q[0] for q in spec], 1), "count": np.stack([q[1] for q in spec], 1),
            "shift": np.stack([q[2] for q in spec], 1),
            "dsel": [q[3] for q in spec], "dcol": np.array([q[4] for q in spec]),
            "dmul": np.array([q[5] for q in spec], dtype=np.int64), "csel": [q[6] for q in spec],
            "acol": np.array([max(q[7], 0) for q in spec]), "amask": np.array([int(q[7] >= 0) for q in spec]),
            "jadd": np.array([q[8] for q in spec], dtype=np.int64), "kind": np.array([q[9] for q in spec]),
        }
        self._tpl = tab
        return tab

    def _launch(self, ids, nodes, edges, b_node, b_edge, x_out, batch_out, y_out, ei_out, csr_out, csc_out,
                m_valid, goff=None, cap_graphs: int = 0) -> None:
        """One batched-copy launch filling the output buffers with the graphs ``ids``."""
        arr = self._descriptors(ids, x_out, batch_out, y_out, ei_out, csr_out, csc_out, m_valid, goff, cap_graphs)
        max_count = int(arr["count"].max()) if len(arr) else 0
        stream = torch.cuda.current_stream(self.device)
        slot = self._desc_slot(arr.nbytes)
        ctypes.memmove(slot[0], arr.ctypes.data, arr.nbytes)
        # the copy kernel reads the table in place from device-visible host memory: no host -> device copy (a blit
        # kernel and a launch boundary per batch, ~5 us of the small-batch step) ahead of it
        _lib.call("hgin_batched_copy", ctypes.c_void_p(slot[0]), len(arr), max_count,
                  ctypes.c_void_p(stream.cuda_stream))
        slot[2].record(stream)

    _DESC_SLOTS = 4

    def _desc_slot(self, nbytes: int) -> list:
        """A slot [pointer, capacity, event, structured view] of the ring of descriptor tables in coherent host
        memory (hgin_host_alloc): refilled only once the copy launch that last read it has finished (its event;
        an event that was never recorded counts as finished)."""
        ring = self.__dict__.get("_desc_ring")
        if ring is None:
            ring = self._desc_ring = [[None, 0, torch.cuda.Event(), None] for _ in range(self._DESC_SLOTS)]
            self._desc_next = 0
            weakref.finalize(self, _free_desc_ring, ring)
        slot = ring[self._desc_next]
        self._desc_next = (self._desc_next + 1) % self._DESC_SLOTS
        slot[2].synchronize()
        if slot[1] < nbytes:
            _free_desc_ring([slot])
            cap = max(int(nbytes), 64 << 10) // DESC_DTYPE.itemsize * DESC_DTYPE.itemsize
            p = ctypes.c_void_p()
            _lib.call("hgin_host_alloc", cap, ctypes.byref(p))
            slot[0], slot[1] = p.value, cap
            slot[3] = np.frombuffer((ctypes.c_char * cap).from_address(p.value), dtype=DESC_DTYPE)
        return slot

    def _descriptors(self, ids, x_out, batch_out, y_out, ei_out, csr_out, csc_out, m_valid, goff=None,
                     cap_graphs: int = 0) -> np.ndarray:
        """The copy descriptors of a batch: the per-graph descriptor groups of ``_template`` shifted by the batch
        offsets, then the tail fills (padding rows' rowptr, m_valid, the per-graph offsets)."""
        tab = self._template()
        ids = np.asarray(ids, dtype=np.int64)
        J = len(ids)
        C = tab["cnt"][ids]
        B = np.cumsum(C, 0) - C                      # batch offset of graph j, per node type / relation
        tot = C.sum(0)
        col = tab["col"]
        outs = {"x": x_out, "batch": batch_out, "y": {None: y_out}, "ei": ei_out,
                "csr.col": {r: c.col for r, c in csr_out.items()}, "csr.perm": {r: c.perm for r, c in csr_out.items()},
                "csr.rowptr": {r: c.rowptr for r, c in csr_out.items()},
                "csc.col": {r: c.col for r, c in csc_out.items()}, "csc.perm": {r: c.perm for r, c in csc_out.items()},
                "csc.rowptr": {r: c.rowptr for r, c in csc_out.items()}}
        dts = [outs[a][b] for a, b in tab["dsel"]]
        dbase = np.array([t.data_ptr() for t in dts], dtype=np.int64)
        des = np.array([t.element_size() for t in dts], dtype=np.int64)
        dconst = np.array([dts[k].shape[1] if c == "e_cap" else 0 for k, c in enumerate(tab["csel"])],
                          dtype=np.int64)
        main = np.zeros((J, len(dts)), dtype=DESC_DTYPE)
        main["src"] = tab["src"][ids]
        main["count"] = tab["count"][ids]
        main["dst"] = dbase + (B[:, tab["dcol"]] * tab["dmul"] + dconst) * des
        main["add"] = tab["shift"][ids] + B[:, tab["acol"]] * tab["amask"] + np.arange(J)[:, None] * tab["jadd"]
        main["kind"] = tab["kind"]
        tail = []
        for r in self.relations:
            s_, _, d = r
            E, n_s, n_d = int(tot[col[r]]), int(tot[col[s_]]), int(tot[col[d]])
            cr, cc = csr_out[r].rowptr, csc_out[r].rowptr
            # rowptr[n .. capacity] = E: the last row's end, and empty rows for padding vertices
            tail.append((0, cr.data_ptr() + 4 * n_d, cr.numel() - n_d, E, FILL_I32))
            tail.append((0, cc.data_ptr() + 4 * n_s, cc.numel() - n_s, E, FILL_I32))
        if m_valid is not None:
            tail.append((0, m_valid.data_ptr(), 1, int(tot[col["path"]]), FILL_I32))
        if goff is not None:   # graph j's rows of type t: [goff[t][j], goff[t][j + 1]); graphs past the batch: empty
            for ti, t in enumerate(("path", "link", "node")):
                if t in col:
                    offs = np.concatenate([[0], np.cumsum(C[:, col[t]])])
                    for j in range(cap_graphs + 1):
                        tail.append((0, goff.data_ptr() + 4 * (ti * (cap_graphs + 1) + j), 1,
                                     int(offs[min(j, J)]), FILL_I32))
            # the padding path rows' graph id: cap_graphs, past every real graph, so a pooled segment (GLOBAL_FEATS,
            # models.py:347-352) never mixes them into a real graph and the batch vector stays sorted
            bp = batch_out["path"]
            n_p = int(tot[col["path"]])
            tail.append((0, bp.data_ptr() + 8 * n_p, bp.numel() - n_p, cap_graphs, FILL_I64))
        ta = np.zeros(len(tail), dtype=DESC_DTYPE)
        if tail:
            for k, name in enumerate(("src", "dst", "count", "add", "kind")):
                ta[name] = [q[k] for q in tail]
        return np.concatenate([main.reshape(-1), ta])



def _free_desc_ring(ring) -> None:
    for slot in ring:
        if slot[0]:
            slot[2].synchronize()
            slot[3] = None
            _lib.lib().hgin_host_free(ctypes.c_void_p(slot[0]))
            slot[0], slot[1] = None, 0


class _DescPlan:
    """collate_into's descriptor table for one padded batch, with what depends only on its buffers precomputed: the
    per-group destination pointers, the tails' destinations (the CSR / CSC rowptr past the batch, m_valid, the
    per-graph offsets).  ``fill`` then writes a batch's table into a structured view in a few numpy operations —
    the same table, entry for entry, as GraphStore._descriptors (tests/test_store_host.py)."""

    def __init__(self, store: "GraphStore", out: "PaddedBatch"):
        self.store = store
        tab = self.tab = store._template()
        col = tab["col"]
        outs = {"x": out.x, "batch": out.batch, "y": {None: out.y}, "ei": out.edge_index,
                "csr.col": {r: c.col for r, c in out.csr.items()}, "csr.perm": {r: c.perm for r, c in out.csr.items()},
                "csr.rowptr": {r: c.rowptr for r, c in out.csr.items()},
                "csc.col": {r: c.col for r, c in out.csc.items()}, "csc.perm": {r: c.perm for r, c in out.csc.items()},
                "csc.rowptr": {r: c.rowptr for r, c in out.csc.items()}}
        dts = [outs[a][b] for a, b in tab["dsel"]]
        des = np.array([t.element_size() for t in dts], dtype=np.int64)
        dconst = np.array([dts[k].shape[1] if c == "e_cap" else 0 for k, c in enumerate(tab["csel"])], dtype=np.int64)
        self.dbase = np.array([t.data_ptr() for t in dts], dtype=np.int64) + dconst * des
        self.dscale = tab["dmul"] * des
        self.gd = len(dts)
        rp_ptr, rp_numel, rp_ncol, rp_ecol = [], [], [], []
        for r in store.relations:
            s_, _, d = r
            cr, cc = out.csr[r].rowptr, out.csc[r].rowptr
            rp_ptr += [cr.data_ptr(), cc.data_ptr()]
            rp_numel += [cr.numel(), cc.numel()]
            rp_ncol += [col[d], col[s_]]
            rp_ecol += [col[r], col[r]]
        self.rp_ptr, self.rp_numel = np.array(rp_ptr, dtype=np.int64), np.array(rp_numel, dtype=np.int64)
        self.rp_ncol, self.rp_ecol = np.array(rp_ncol), np.array(rp_ecol)
        self.mv_ptr, self.mv_col = out.m_valid.data_ptr(), col["path"]
        cap = self.cap = out.batch_size
        gt = [(ti, col[t]) for ti, t in enumerate(("path", "link", "node")) if t in col]
        self.g_cols = np.array([c for _, c in gt], dtype=np.int64)
        self.g_ptr = np.array([[out.goff.data_ptr() + 4 * (ti * (cap + 1) + j) for j in range(cap + 1)]
                               for ti, _ in gt], dtype=np.int64).reshape(-1)
        self.bp_ptr, self.bp_numel = out.batch["path"].data_ptr(), out.batch["path"].numel()
        self.n_tail = len(rp_ptr) + 1 + len(gt) * (cap + 1) + 1
        self.max_bytes = (cap * self.gd + self.n_tail) * DESC_DTYPE.itemsize

    def fill(self, ids: np.ndarray, view: np.ndarray):
        """Write the table of the graphs ``ids`` into ``view``; returns (entries, largest count)."""
        tab = self.tab
        J = len(ids)
        C = tab["cnt"][ids]
        B = np.cumsum(C, 0) - C
        tot = C.sum(0)
        nm = J * self.gd
        main = view[:nm].reshape(J, self.gd)
        main["src"] = tab["src"][ids]
        cnt = tab["count"][ids]
        main["count"] = cnt
        main["dst"] = self.dbase + B[:, tab["dcol"]] * self.dscale
        main["add"] = tab["shift"][ids] + B[:, tab["acol"]] * tab["amask"] + np.arange(J)[:, None] * tab["jadd"]
        main["kind"] = tab["kind"]
        main["reserved"] = 0
        t = view[nm:nm + self.n_tail]
        k = len(self.rp_ptr)
        n = tot[self.rp_ncol]
        t["src"] = 0
        t["kind"] = FILL_I32
        t["reserved"] = 0
        t["dst"][:k] = self.rp_ptr + 4 * n
        t["count"][:k] = self.rp_numel - n
        t["add"][:k] = tot[self.rp_ecol]
        t["dst"][k] = self.mv_ptr
        t["count"][k:] = 1
        t["add"][k] = tot[self.mv_col]
        offs = np.zeros((J + 1, len(self.g_cols)), dtype=np.int64)
        np.cumsum(C[:, self.g_cols], 0, out=offs[1:])
        ng = len(self.g_ptr)
        t["dst"][k + 1:k + 1 + ng] = self.g_ptr
        t["add"][k + 1:k + 1 + ng] = offs[np.minimum(np.arange(self.cap + 1), J)].T.reshape(-1)
        n_p = int(tot[self.mv_col])   # the padding path rows' graph id (GraphStore._descriptors)
        t["dst"][-1] = self.bp_ptr + 8 * n_p
        t["count"][-1] = self.bp_numel - n_p
        t["add"][-1] = self.cap
        t["kind"][-1] = FILL_I64
        max_count = max(int(cnt.max()) if cnt.size else 0, int(t["count"].max()))
        return nm + self.n_tail, max_count

@dataclass
class PaddedBatch(HeteroGraph):
    """Static-capacity batch buffers (GraphStore.padded_batch): rows past the current batch are isolated
    padding vertices; ``m_valid`` (device int32) holds the current batch's path count for the fused loss."""
    m_valid: Tensor = None
    csr: Dict[EdgeType, ops.Csr] = None
    csc: Dict[EdgeType, ops.Csr] = None
    batch_size: int = 0
    goff: Tensor = None   # int32 [3 * (batch_size + 1)]: per-graph node offsets, path | link | node
