"""PyG-compatible message-passing surface backed by libhgin.so.

Mirrors, name for name and argument for argument, what the reference's ``models.py`` uses:

* ``MessagePassing``  — the PyG 2.0.x base class as used by GINConv (``models.py:180``): ``propagate(
  edge_index, x=..., size=None)`` with flow ``source_to_target``, ``aggr='add'``, identity ``message``;
  the same input checks (``edge_index`` must be a 2-D ``torch.long`` tensor with 2 rows -> AssertionError).
* ``GINConv``         — ``models.py:180-228`` (eps Parameter/buffer, ``reset_parameters`` through ``reset``,
  concat / add self term, ``nn(out)``).
* ``GINLayer``        — ``models.py:231-245`` (mlp = Sequential(Linear, PReLU); conv shares it, so the
  state_dict exposes the same tensors under ``mlp.*`` and ``conv.nn.*``).
* ``HeteroConv``      — PyG 2.0.x ``HeteroConv(convs, aggr='sum')`` as built at ``models.py:286-298``:
  ModuleDict keyed ``'__'.join(edge_type)``; relations iterated in ``edge_index_dict`` order, those without
  a conv skipped; outputs summed per destination type.

When ``nn`` is ``Sequential(Linear, PReLU)`` (every GINLayer), GINConv runs the fused HIP path:
aggregate + self term -> MFMA GEMM + bias + PReLU, and HeteroConv hands the previous relation's output for
the same destination type to the epilogue (``accum``), replacing ``torch.stack(outs).sum(0)`` (for two
relations ``a + b``, bit-identical).  Everything runs on the device; CPU tensors raise.
"""
from __future__ import annotations

from typing import Any, Callable, Dict, Optional, Tuple, Union

import torch
from torch import Tensor

from . import ops

EdgeType = Tuple[str, str, str]

# HeteroConv layers of GINLayers run as one autograd node (ops.hetero_gin_layer); setting this to False keeps one
# autograd node per relation, whose shared-node-type gradients autograd adds itself (the equivalence test's reference).
LAYER_FN = True


def reset(value: Any) -> None:
    """models.py:162-167 (re-initialises every child exposing reset_parameters)."""
    if hasattr(value, "reset_parameters"):
        value.reset_parameters()
    else:
        for child in value.children() if hasattr(value, "children") else []:
            reset(child)


class MessagePassing(torch.nn.Module):
    """PyG 2.0.x MessagePassing for Tensor edge_index, aggr='add', identity message (HIP aggregate)."""

    def __init__(self, aggr: Optional[str] = "add", flow: str = "source_to_target", node_dim: int = -2, **kwargs):
        super().__init__()
        if aggr not in ("add", "sum"):
            raise NotImplementedError(f"hgin MessagePassing: aggr={aggr!r} (only 'add' is on the HIP path)")
        if flow != "source_to_target":
            raise NotImplementedError("hgin MessagePassing: only flow='source_to_target'")
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim

    def _graph(self, edge_index: Tensor, x_src: Tensor, x_dst: Optional[Tensor], size) -> ops.RelationGraph:
        if not isinstance(edge_index, Tensor):
            raise NotImplementedError("hgin: SparseTensor adjacency is not supported (models.py:222-225 is "
                                      "unreachable with [2, E] edge_index)")
        ops.check_edge_index(edge_index)
        n_src = x_src.size(0) if size is None or size[0] is None else int(size[0])
        if x_dst is not None:
            n_dst = x_dst.size(0)
        elif size is not None and size[1] is not None:
            n_dst = int(size[1])
        else:
            n_dst = int(edge_index[1].max()) + 1 if edge_index.numel() else 0
        return ops.relation_graph(edge_index, n_src, n_dst)

    def propagate(self, edge_index: Tensor, size=None, **kwargs) -> Tensor:
        x = kwargs["x"]
        if isinstance(x, Tensor):
            x = (x, x)
        if type(self).message is not MessagePassing.message:
            raise NotImplementedError("hgin: only the identity message runs on the HIP aggregate")
        graph = self._graph(edge_index, x[0], x[1], size)
        return ops.aggregate(x[0], None, None, graph, ops.COMBINE_NONE)

    def message(self, x_j: Tensor) -> Tensor:
        return x_j


def _fusable_mlp(nn: torch.nn.Module) -> bool:
    return (isinstance(nn, torch.nn.Sequential) and len(nn) == 2 and isinstance(nn[0], torch.nn.Linear)
            and nn[0].bias is not None and isinstance(nn[1], torch.nn.PReLU) and nn[1].weight.numel() == 1)


class GINConv(MessagePassing):
    """GINConv of models.py:180-228 (PyG 2.0.2 GINConv + the concat option)."""

    supports_accum = True

    def __init__(self, nn: Callable, eps: float = 0.0, train_eps: bool = False, concat: bool = False, **kwargs):
        kwargs.setdefault("aggr", "add")
        super().__init__(**kwargs)
        self.nn = nn
        self.initial_eps = eps
        self.concat = concat
        if train_eps:
            self.eps = torch.nn.Parameter(torch.Tensor([eps]))
        else:
            self.register_buffer("eps", torch.Tensor([eps]))
        self.reset_parameters()

    def reset_parameters(self):
        reset(self.nn)
        self.eps.data.fill_(self.initial_eps)

    def forward(self, x: Union[Tensor, Tuple[Tensor, Optional[Tensor]]], edge_index: Tensor, size=None,
                accum: Optional[Tensor] = None) -> Tensor:
        if isinstance(x, Tensor):
            x = (x, x)
        x_src, x_r = x
        graph = self._graph(edge_index, x_src, x_r, size)
        mode = ops.COMBINE_NONE if x_r is None else (ops.COMBINE_CONCAT if self.concat else ops.COMBINE_ADD)
        if x_r is not None and _fusable_mlp(self.nn):
            lin, act = self.nn[0], self.nn[1]
            return ops.gin_conv(x_src, x_r, self.eps, lin.weight, lin.bias, act.weight, graph, mode, accum)
        out = ops.aggregate(x_src, x_r, self.eps if x_r is not None else None, graph, mode)
        out = self.nn(out)
        return out if accum is None else accum + out

    def __repr__(self):
        return "{}(nn={})".format(self.__class__.__name__, self.nn)


class GINLayer(torch.nn.Module):
    """models.py:231-245."""

    supports_accum = True

    def __init__(self, in_channels: int, out_channels: int, concat: bool = False) -> None:
        super().__init__()
        self.mlp = torch.nn.Sequential(torch.nn.Linear(in_channels, out_channels), torch.nn.PReLU())
        self.conv = GINConv(self.mlp, eps=0, train_eps=True, concat=concat)

    def forward(self, x, edge_index, accum: Optional[Tensor] = None):
        return self.conv(x, edge_index, accum=accum)


class HeteroConv(torch.nn.Module):
    """PyG 2.0.x HeteroConv(convs, aggr) with the per-destination sum fused into the conv epilogue."""

    def __init__(self, convs: Dict[EdgeType, torch.nn.Module], aggr: Optional[str] = "sum"):
        super().__init__()
        self.convs = torch.nn.ModuleDict({"__".join(k): v for k, v in convs.items()})
        self.aggr = aggr
        self.skip: set = set()   # relation keys whose outputs are dead (see models.HetroGIN.prune_dead)

    def reset_parameters(self):
        for conv in self.convs.values():
            conv.reset_parameters()

    def _layer_specs(self, x_dict, edge_index_dict):
        """The relations of this call for the one-node layer path (ops.hetero_gin_layer), or None when it does not
        apply: every live relation a GINLayer-style GINConv (Linear + PReLU, trainable-or-buffer eps) between two
        different node types, device inputs, aggr='sum'."""
        if self.aggr != "sum" or not LAYER_FN:
            return None
        types, specs, params = [], [], []
        for edge_type, edge_index in edge_index_dict.items():
            src, _, dst = edge_type
            key = "__".join(edge_type)
            if key not in self.convs or key in self.skip:
                continue
            conv = self.convs[key]
            conv = getattr(conv, "conv", conv)
            if not isinstance(conv, GINConv) or not _fusable_mlp(conv.nn) or src == dst:
                return None
            for t in (src, dst):
                if t not in types:
                    types.append(t)
            x_src, x_dst = x_dict[src], x_dict[dst]
            if not (x_src.is_cuda and x_dst.is_cuda):
                return None
            graph = conv._graph(edge_index, x_src, x_dst, None)
            mode = ops.COMBINE_CONCAT if conv.concat else ops.COMBINE_ADD
            specs.append(ops.RelSpec(types.index(src), types.index(dst), graph, mode))
            lin, act = conv.nn[0], conv.nn[1]
            params.append((conv.eps, lin.weight, lin.bias, act.weight))
        if not specs:
            return None
        return types, specs, params

    def forward(self, x_dict: Dict[str, Tensor], edge_index_dict: Dict[EdgeType, Tensor]) -> Dict[str, Tensor]:
        plan = self._layer_specs(x_dict, edge_index_dict)
        if plan is not None:
            # one autograd node for the layer: the gradient sums over relations sharing a node type happen inside
            # the backward kernels (ops._HeteroGINLayerFn); same forward arithmetic as the loop below
            types, specs, params = plan
            ys = ops.hetero_gin_layer([x_dict[t] for t in types], specs, params)
            dst_order = []
            for sp in specs:
                if types[sp.dst] not in dst_order:
                    dst_order.append(types[sp.dst])
            return dict(zip(dst_order, ys))
        outs: Dict[str, list] = {}
        for edge_type, edge_index in edge_index_dict.items():
            src, _, dst = edge_type
            key = "__".join(edge_type)
            if key not in self.convs or key in self.skip:
                continue
            conv = self.convs[key]
            xin = x_dict[src] if src == dst else (x_dict[src], x_dict[dst])
            lst = outs.setdefault(dst, [])
            if self.aggr == "sum" and getattr(conv, "supports_accum", False) and len(lst) == 1:
                lst[0] = conv(xin, edge_index, accum=lst[0])     # running sum in the GEMM epilogue
                continue
            lst.append(conv(xin, edge_index))
        res: Dict[str, Tensor] = {}
        for k, v in outs.items():
            if len(v) == 1:
                res[k] = v[0]
            elif self.aggr is None:
                res[k] = torch.stack(v, dim=1)
            else:
                out = getattr(torch, self.aggr)(torch.stack(v, dim=0), dim=0)
                res[k] = out[0] if isinstance(out, tuple) else out
        return res
