"""Connected-graph variant of the multi-GPU path: a 1D destination-range partition.

The headline multi-GPU split (``hgin/dist.py``) gives every rank whole graph components, which is the
reference's real unit (a batch is a disjoint union of network samples, ``dataset.py:26, :242``).  One large
*connected* graph has no such cut; this module trains it across ranks with the layout §8.E prescribes
(reported, not the headline):

* rank r of W owns rows [r·c_t, min(N_t, (r+1)·c_t)) of every node type t, c_t = ceil(N_t / W): its slice
  of the features, the path labels and the path readout;
* every relation keeps, on each rank, exactly the edges whose destination the rank owns (relative edge
  order preserved, destination ids made local, source ids global) — the CSR rows the rank aggregates;
* per layer, the source-side node embeddings are **all-gathered** (``AllGatherRows``: N_t·F·s bytes
  received per type), the layer runs unchanged on (gathered sources, owned destinations) through the
  same HIP GINConv kernels, and in the backward the gradient of the gathered table is
  **reduce-scattered** back to its owners (the autograd adjoint of the all-gather);
* parameter gradients and the loss sums are combined by ``GradAllReducer.sync_sqrt_mean`` (one RCCL
  all-reduce), so the ranks train as the single device holding the whole graph (hgin/dist.py semantics).

Forward aggregates are bit-identical to the single-device ones (every destination row sums the same edges
in the same order); the backward's source-gradient sums and the weight-gradient reductions are split over
ranks, so gradients agree within fp32 summation-order tolerance (tests/test_partition_gloo.py,
tests/test_gpu_dist.py).

Overlap (device tensors): a layer's all-gathers are all issued at the layer's start on a communication stream
(``DstRangePartition.prefetch``) and the compute stream waits for each table only just before its first
relation, so the link / node gathers run under the first relations' kernels.  Because the gather's autograd
node runs on that stream, PyTorch runs its backward — the reduce-scatter — there too and makes only the
gradient's consumer wait (the autograd engine's cross-stream hand-off), so each table's reduce-scatter starts
as soon as its gradient is complete and overlaps the remaining relations' backward.  (Bucketing the three
reduce-scatters into one collective would need two strided repacks of GB-sized tables at cfg3 for a saving of
two collective latencies; per-table collectives, overlapped, are the better trade at these sizes.)  The
arithmetic is unchanged, so the results are bitwise those of the serial schedule (``overlap=False``).

Not supported here (they pool or normalise across the whole graph): ``global_feats``, BatchNorm in the
readout, dropout > 0.  ``HGIN_DIST_BACKEND=gloo`` rehearsals stage CUDA tensors through the host (gloo's
collectives are CPU ones); RCCL runs them on the device.
"""
from __future__ import annotations

from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

from .data import HeteroGraph
from .dist import GradAllReducer


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _rank(group) -> int:
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


def _staged(t: torch.Tensor, group) -> bool:
    return t.is_cuda and dist.get_backend(group) == "gloo"


def _all_gather_into(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    if _staged(inp, group):
        o = out.cpu()
        dist.all_gather_into_tensor(o, inp.cpu(), group=group)
        out.copy_(o)
    else:
        dist.all_gather_into_tensor(out, inp, group=group)


def _reduce_scatter_into(out: torch.Tensor, inp: torch.Tensor, group) -> None:
    if _staged(inp, group):
        o = out.cpu()
        dist.reduce_scatter_tensor(o, inp.cpu(), op=dist.ReduceOp.SUM, group=group)
        out.copy_(o)
    else:
        dist.reduce_scatter_tensor(out, inp, op=dist.ReduceOp.SUM, group=group)


class _AllGatherRows(torch.autograd.Function):
    """Forward: the [N, F] table from every rank's [n_r, F] row block (blocks of c rows, the last one may be
    short: padded to c on the wire).  Backward: the reduce-scatter of the [N, F] gradient (sum over ranks)."""

    @staticmethod
    def forward(ctx, x_local: torch.Tensor, n_total: int, chunk: int, group):
        world = _world(group)
        ctx.meta = (x_local.shape[0], n_total, chunk, group)
        src = x_local.contiguous()
        if src.shape[0] != chunk:
            pad = src.new_zeros((chunk,) + tuple(src.shape[1:]))
            pad[: src.shape[0]] = src
            src = pad
        buf = src.new_empty((world * chunk,) + tuple(src.shape[1:]))
        _all_gather_into(buf, src, group)
        return buf[:n_total] if world * chunk != n_total else buf

    @staticmethod
    def backward(ctx, g_full: torch.Tensor):
        n_local, n_total, chunk, group = ctx.meta
        world = _world(group)
        g = g_full.contiguous()
        if world * chunk != n_total:
            pad = g.new_zeros((world * chunk,) + tuple(g.shape[1:]))
            pad[:n_total] = g
            g = pad
        out = g.new_empty((chunk,) + tuple(g.shape[1:]))
        _reduce_scatter_into(out, g, group)
        return (out if n_local == chunk else out[:n_local]), None, None, None


def _collectives() -> bool:
    return dist.is_available() and dist.is_initialized()


class DstRangePartition:
    """1D destination-range partition of a hetero graph's node types over the ranks of ``group``.

    ``overlap`` (default on): issue each layer's all-gathers together on a communication stream (device tensors
    only; see the module docstring); off: one blocking gather per table at its first use."""

    def __init__(self, n_nodes: Dict[str, int], rank: Optional[int] = None, world: Optional[int] = None,
                 group=None, overlap: bool = True):
        self.group = group
        self.overlap = overlap
        self._comm = {}
        self.world = int(world if world is not None else _world(group))
        self.rank = int(rank if rank is not None else _rank(group))
        if not 0 <= self.rank < self.world:
            raise ValueError(f"rank {self.rank} outside world {self.world}")
        self.n_nodes = {t: int(n) for t, n in n_nodes.items()}
        self.chunk = {t: -(-n // self.world) if n else 0 for t, n in self.n_nodes.items()}

    def rows(self, t: str) -> Tuple[int, int]:
        c, n = self.chunk[t], self.n_nodes[t]
        return min(n, self.rank * c), min(n, (self.rank + 1) * c)

    def local_graph(self, graph: HeteroGraph) -> HeteroGraph:
        """This rank's share: owned rows of every node type; per relation the edges whose destination is owned
        (order kept, destination ids local, source ids global); owned path labels and batch entries."""
        for t, n in self.n_nodes.items():
            if graph.num_nodes(t) != n:
                raise ValueError(f"partition built for {n} {t!r} nodes, graph has {graph.num_nodes(t)}")
        x = {t: v[slice(*self.rows(t))] for t, v in graph.x.items()}
        ei = {}
        for rel, e in graph.edge_index.items():
            lo, hi = self.rows(rel[2])
            keep = (e[1] >= lo) & (e[1] < hi)
            el = e[:, keep]
            el[1] -= lo
            ei[rel] = el.contiguous()
        plo, phi = self.rows("path")
        batch = {t: v[slice(*self.rows(t))] for t, v in graph.batch.items()}
        return HeteroGraph(x, ei, graph.y[plo:phi], batch)

    def gather(self, x_local: torch.Tensor, t: str) -> torch.Tensor:
        """The full [N_t, F] table of type t (differentiable: the backward reduce-scatters to the owners).  With
        a process group the collective runs at every world size (at 1 it is the backend's copy)."""
        lo, hi = self.rows(t)
        if x_local.shape[0] != hi - lo:
            raise ValueError(f"{t!r}: rank {self.rank} owns {hi - lo} rows, got {x_local.shape[0]}")
        if self.world == 1 and not _collectives():
            return x_local
        return _AllGatherRows.apply(x_local, self.n_nodes[t], self.chunk[t], self.group)

    def _comm_stream(self, device) -> torch.cuda.Stream:
        s = self._comm.get(device)
        if s is None:
            s = self._comm[device] = torch.cuda.Stream(device=device)
        return s

    def prefetch(self, tables: Dict[str, torch.Tensor]) -> Dict[str, "_Pending"]:
        """Issue the gathers of ``tables`` (type -> owned rows) now: on the communication stream when overlapping
        device tensors, else lazily (each one blocking at its first use)."""
        out = {}
        for t, x in tables.items():
            if self.overlap and x.is_cuda and (self.world > 1 or _collectives()):
                cur = torch.cuda.current_stream(x.device)
                comm = self._comm_stream(x.device)
                comm.wait_stream(cur)                    # x_local is produced on the compute stream
                x.record_stream(comm)
                with torch.cuda.stream(comm):
                    full = self.gather(x, t)
                out[t] = _Pending(full, comm)
            else:
                out[t] = _Pending(None, None, lambda x=x, t=t: self.gather(x, t))
        return out

    def exchange_bytes(self, widths: Dict[str, int], elem: int) -> int:
        """Bytes one rank receives per all-gather round of the given per-type widths (the backward's
        reduce-scatter moves the same amount)."""
        return sum((self.world - 1) * self.chunk[t] * w * elem for t, w in widths.items())


class _Pending:
    """A gathered table that may still be in flight on the communication stream."""

    def __init__(self, full, stream, thunk=None):
        self.full, self.stream, self.thunk = full, stream, thunk

    def get(self) -> torch.Tensor:
        if self.full is None:
            self.full = self.thunk()
        elif self.stream is not None:
            cur = torch.cuda.current_stream(self.full.device)
            cur.wait_stream(self.stream)                 # the table has landed
            self.full.record_stream(cur)                 # allocated on the comm stream, read on this one
            self.stream = None
        return self.full


def _check_supported(model) -> None:
    if getattr(model, "global_feats", False):
        raise NotImplementedError("dst-range partition: global_feats pools over the whole graph")
    if getattr(model, "dropout", 0.0) > 0.0 and model.training:
        raise NotImplementedError("dst-range partition: dropout > 0")
    for m in model.readout.modules():
        if isinstance(m, torch.nn.modules.batchnorm._BatchNorm):
            raise NotImplementedError("dst-range partition: BatchNorm statistics span every rank's paths")


def _select_features(model, x_dict) -> None:
    sel = getattr(model, "_select_features", None)
    if sel is not None:
        sel(x_dict)
    elif not (model.divided_features and model.bl_features):
        raise NotImplementedError("dst-range partition: feature slicing needs the model's _select_features")


def _layer(part: DstRangePartition, hetero_conv, x_local: Dict[str, torch.Tensor], edge_index_dict):
    """One HeteroConv layer on (gathered sources, owned destinations); the per-destination relation sum as
    hgin.conv.HeteroConv's relation loop does it (running sum in the GEMM epilogue where the conv offers it)."""
    outs: Dict[str, list] = {}
    skip = getattr(hetero_conv, "skip", ())
    live = [(rel, ei) for rel, ei in edge_index_dict.items()
            if "__".join(rel) in hetero_conv.convs and "__".join(rel) not in skip]
    srcs = []
    for rel, _ in live:
        if rel[0] == rel[2]:
            raise NotImplementedError("dst-range partition: same-type relations")
        if rel[0] not in srcs:
            srcs.append(rel[0])
    pending = part.prefetch({t: x_local[t] for t in srcs})     # every gather of the layer, in first-use order
    full: Dict[str, torch.Tensor] = {}
    for rel, ei in live:
        src, _, dst = rel
        key = "__".join(rel)
        if src not in full:
            full[src] = pending[src].get()
        conv = hetero_conv.convs[key]
        lst = outs.setdefault(dst, [])
        if getattr(conv, "supports_accum", False) and len(lst) == 1:
            lst[0] = conv((full[src], x_local[dst]), ei, accum=lst[0])
        else:
            lst.append(conv((full[src], x_local[dst]), ei))
    return {t: (v[0] if len(v) == 1 else torch.stack(v, 0).sum(0)) for t, v in outs.items()}


def forward_loss(model, part: DstRangePartition, local: HeteroGraph):
    """(out rows of the owned paths, S_r = Σ over the owned paths of 100·|(out − y) / y|) — the rank's path sum
    of train.py's MAPE (train.py:12-13, :38-40), linear in its paths (hgin/dist.py)."""
    _check_supported(model)
    x = local.x_dict()
    _select_features(model, x)
    origin_path = x["path"]
    for i in range(model.num_layers):   # models.py:355-359
        x = _layer(part, model.convs[i], x, local.edge_index_dict())
    m = int(local.y.numel())
    readout = getattr(model, "_readout", None)
    if m == 0:
        # No owned paths.  The readout still runs (on the empty row block) so every readout parameter gets a
        # (zero) gradient as on the other ranks — GradAllReducer's layout and Adam's state stay rank-independent
        # — and the zero loss sum still reaches every gathered table (the backward's collectives).
        if readout is not None:
            out = readout(x["path"], origin_path, None, None, None)
        else:
            out = torch.cat((x["path"], origin_path), 1) if model.concat_path else x["path"]
            for seq in model.readout:
                out = seq(out)
        return out, out.sum() * 0.0 + x["path"].sum() * 0.0
    if readout is not None:
        out, lv = readout(x["path"], origin_path, None, local.y, None)
    else:   # a plain module stack (the CPU oracle in tests): cat + Sequential readout + train.py's mape
        from .train import mape
        h = torch.cat((x["path"], origin_path), 1) if model.concat_path else x["path"]
        for seq in model.readout:
            h = seq(h)
        out, lv = h, mape(h, local.y.reshape(-1, 1))
    return out, lv * float(m)


def train_step(model, opt, part: DstRangePartition, local: HeteroGraph,
               reducer: Optional[GradAllReducer] = None) -> torch.Tensor:
    """One train.py:31-44 iteration of the whole connected graph across the ranks; returns the graph's loss
    value (MAPE over every path, identical on every rank)."""
    opt.zero_grad()
    _, s_local = forward_loss(model, part, local)
    s_local.backward()
    reducer = reducer or GradAllReducer(model.parameters(), group=part.group)
    m_local = torch.full((), float(local.y.numel()), dtype=torch.float32, device=s_local.device)
    loss_value = reducer.sync_sqrt_mean(s_local, m_local)
    opt.step()
    return loss_value.detach()


__all__ = ["DstRangePartition", "forward_loss", "train_step"]
