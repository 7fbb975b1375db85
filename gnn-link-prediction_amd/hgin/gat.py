"""HetroGAT's graph attention on the MI355X path (F4 widening; reference ``models.py:380-506``, PyG 2.0.2 ``GATConv``).

``GATConv(in_channels, out_channels, heads=1, concat=True, negative_slope=0.2, dropout=0.0, add_self_loops=True,
bias=True)`` keeps PyG 2.0.2's surface and state_dict (``att_src``, ``att_dst``, ``bias``, ``lin_src.weight``,
``lin_dst.weight``), its lazy ``(-1, -1)`` input projections (``Linear``: an UninitializedParameter until the first
forward, then glorot-initialised on the parameter's device in forward call order, lin_src before lin_dst — the RNG
order of the reference) and its edge handling: self-loops removed and (i, i) added for i < min(N_src, N_dst), for
bipartite relations too.  The projections run on the split-mode MFMA GEMMs (``ops.gemm_nt`` / ``ops.gemm_tn``); the
per-edge logits, the per-destination softmax, the weighted aggregate and their backward are the HIP kernels of
``csrc/hgin_gat.hip`` on the self-loop-adjusted relation's CSR (forward, backward destination side) and CSC (backward
source side).  fp32; dropout on the attention must be 0 (the reference's configuration), as on the GIN path.
"""
from __future__ import annotations

import ctypes
import math
from dataclasses import dataclass
from typing import Optional, Tuple, Union

import torch
from torch import Tensor

from . import _lib, ops
from .ops import _p, _stream, _workspace


def glorot(t: Optional[Tensor]) -> None:
    """torch_geometric.nn.inits.glorot: U(-a, a) with a = sqrt(6 / (size(-2) + size(-1)))."""
    if t is not None:
        a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
        t.data.uniform_(-a, a)


class Linear(torch.nn.Module):
    """PyG 2.0.2 ``torch_geometric.nn.dense.linear.Linear`` as GATConv builds it (no bias, glorot weight), lazy when
    ``in_channels`` is -1: materialised [out, in] at the first call (a forward pre-hook) or from a loaded state_dict."""

    def __init__(self, in_channels: int, out_channels: int, bias: bool = False, weight_initializer: str = "glorot"):
        super().__init__()
        if bias or weight_initializer != "glorot":
            raise NotImplementedError("hgin.gat.Linear: GATConv's bias-free glorot projection only")
        self.in_channels, self.out_channels = in_channels, out_channels
        if in_channels > 0:
            self.weight = torch.nn.Parameter(torch.Tensor(out_channels, in_channels))
        else:
            self.weight = torch.nn.parameter.UninitializedParameter()
            self._hook = self.register_forward_pre_hook(self._initialize)
        self.register_parameter("bias", None)
        self._register_load_state_dict_pre_hook(self._lazy_load_hook)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        if self.in_channels > 0:
            glorot(self.weight)

    @torch.no_grad()
    def _initialize(self, module, inputs) -> None:
        if isinstance(self.weight, torch.nn.parameter.UninitializedParameter):
            self.in_channels = inputs[0].size(-1)
            self.weight.materialize((self.out_channels, self.in_channels))
            self.reset_parameters()
        self._hook.remove()
        delattr(self, "_hook")

    def _lazy_load_hook(self, state_dict, prefix, *args) -> None:
        w = state_dict.get(prefix + "weight")
        if w is not None and isinstance(self.weight, torch.nn.parameter.UninitializedParameter):
            self.in_channels = w.size(-1)
            self.weight.materialize(w.shape)
            if hasattr(self, "_hook"):
                self._hook.remove()
                delattr(self, "_hook")

    def _save_to_state_dict(self, destination, prefix, keep_vars):
        # as PyG's Linear: an uninitialised weight is saved as the UninitializedParameter itself
        if isinstance(self.weight, torch.nn.parameter.UninitializedParameter):
            destination[prefix + "weight"] = self.weight
        else:
            destination[prefix + "weight"] = self.weight if keep_vars else self.weight.detach()

    def forward(self, x: Tensor) -> Tensor:
        return _project(x, self.weight)


class _ProjectFn(torch.autograd.Function):
    """y = x W^T (bias-free) on the NT GEMM; backward: g_W = g_y^T x (TN GEMM), g_x = g_y W (NT GEMM)."""

    @staticmethod
    def forward(ctx, x, w):
        ctx.save_for_backward(x, w)
        return ops.gemm_nt(x, w)

    @staticmethod
    def backward(ctx, g):
        x, w = ctx.saved_tensors
        g = g.contiguous()
        gx = ops.gemm_nt(g, w.t().contiguous()) if ctx.needs_input_grad[0] else None
        gw = ops.gemm_tn(g, x) if ctx.needs_input_grad[1] else None
        return gx, gw


def _project(x: Tensor, w: Tensor) -> Tensor:
    ops.require_device(x, w, what="hgin.gat.Linear")
    if x.dtype != torch.float32 or w.dtype != torch.float32:
        raise NotImplementedError("hgin GATConv: fp32 only")
    if x.size(-1) != w.size(1):
        # the reference's F.linear raises on this too (models.py:425 GATConv(H, H) fed H * heads columns)
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({x.size(0)}x{x.size(-1)} and "
                           f"{w.size(1)}x{w.size(0)})")
    return _ProjectFn.apply(x, w)


@dataclass
class GatGraph:
    csr: ops.Csr          # self-loop-adjusted relation by destination
    csc: ops.Csr          # ... by source
    cpos: Tensor          # int32 [E]: CSR position of each CSC entry
    n_edges: int


def gat_graph(edge_index: Tensor, n_src: int, n_dst: int, add_self_loops: bool) -> GatGraph:
    """The relation's edge list as GATConv sees it (PyG 2.0.2 remove_self_loops + add_self_loops(num_nodes =
    min(N_src, N_dst)) on a Tensor edge_index), as CSR + CSC + the CSC -> CSR position map; cached on the
    edge_index tensor (invalidated by in-place edits, like ops.relation_graph)."""
    ops.check_edge_index(edge_index)
    key = (int(n_src), int(n_dst), bool(add_self_loops))
    cache = getattr(edge_index, "_hgin_gat", None)
    if cache is not None and cache[0] == edge_index._version and key in cache[1]:
        return cache[1][key]
    ei = edge_index
    if add_self_loops:
        n = min(int(n_src), int(n_dst))
        loop = torch.arange(n, dtype=torch.long, device=ei.device)
        ei = torch.cat([ei[:, ei[0] != ei[1]], torch.stack([loop, loop], 0)], dim=1).contiguous()
    csr = ops.build_csr(ei, 1, int(n_dst), int(n_src))
    csc = ops.build_csr(ei, 0, int(n_src), int(n_dst), validate=False)
    E = int(ei.size(1))
    inv = torch.empty(E, dtype=torch.int32, device=ei.device)
    inv[csr.perm.long()] = torch.arange(E, dtype=torch.int32, device=ei.device)
    g = GatGraph(csr, csc, inv[csc.perm.long()].contiguous(), E)
    if cache is None or cache[0] != edge_index._version:
        cache = (edge_index._version, {})
        try:
            edge_index._hgin_gat = cache
        except (AttributeError, RuntimeError):
            return g
    cache[1][key] = g
    return g


def _wsum(x: Tensor, w: Optional[Tensor], H: int, C: int) -> Tensor:
    """[H * C] = sum_n w[n, h] x[n, h * C + c] (w None: plain column sums), fixed-order (hgin_gat_wsum_f32)."""
    n = x.size(0)
    out = torch.empty(H * C, dtype=torch.float32, device=x.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_gat_wsum_workspace_size(n, H, C, ctypes.byref(nbytes)), "gat_wsum_workspace_size")
    ws = _workspace(nbytes.value, x.device)
    _lib.call("hgin_gat_wsum_f32", _p(x), x.stride(0), n, H, C, _p(w), _p(out), _p(ws), nbytes.value, _stream(x))
    return out


def _attn_one_pass(H: int, C: int) -> bool:
    """hgin_gat_attn_fwd_f32 takes the shape (the wave-group form: C a multiple of 4 with C / 4 a power of two,
    H * C <= 256; HGIN_GAT_WAVE=0 turns it off); the tensors are contiguous and 16-B aligned by construction."""
    return bool(_lib.lib().hgin_gat_attn_supported(int(H), int(C)))


def _logits(x: Tensor, att: Tensor, H: int, C: int) -> Tensor:
    a = torch.empty(x.size(0), H, dtype=torch.float32, device=x.device)
    _lib.call("hgin_gat_logits_f32", _p(x), x.stride(0), x.size(0), H, C, _p(att), _p(a), _stream(x))
    return a


class _GatAttentionFn(torch.autograd.Function):
    """out = sum_k softmax_k(leaky_relu(a_s[j_k] + a_d[i])) x_s[j_k] + bias [+ accum] per destination and head, with
    a_s = (x_s . att_src).sum(-1), a_d = (x_d . att_dst).sum(-1) (x_d None: no destination term)."""

    @staticmethod
    def forward(ctx, xs, xd, att_src, att_dst, bias, accum, graph: GatGraph, H: int, C: int, slope: float):
        att_s = att_src.reshape(-1).contiguous()
        att_d = att_dst.reshape(-1).contiguous()
        a_d = _logits(xd, att_d, H, C) if xd is not None else None
        n_dst = graph.csr.n_rows
        alpha = torch.empty(graph.n_edges, H, dtype=torch.float32, device=xs.device)
        out = torch.empty(n_dst, H * C, dtype=torch.float32, device=xs.device)
        acc_ld = accum.stride(0) if accum is not None else 0
        al16 = lambda t: t is None or (t.data_ptr() % 16 == 0 and (t.dim() < 2 or t.stride(0) % 4 == 0))  # noqa: E731
        if _attn_one_pass(H, C) and al16(xs) and al16(accum) and al16(bias) and al16(att_s):
            # one pass: a_s from the gathered x_s rows (hgin_gat_attn_fwd_f32); the backward forms a_s itself
            a_s = None
            _lib.call("hgin_gat_attn_fwd_f32", _p(graph.csr.rowptr), _p(graph.csr.col), n_dst, H, C, _p(xs),
                      xs.stride(0), _p(att_s), _p(a_d), ctypes.c_float(slope), _p(bias), _p(accum), acc_ld, _p(alpha),
                      _p(out), out.stride(0), _stream(xs))
        else:
            a_s = _logits(xs, att_s, H, C)
            _lib.call("hgin_gat_fwd_f32", _p(graph.csr.rowptr), _p(graph.csr.col), n_dst, H, C, _p(xs), xs.stride(0),
                      _p(a_s), _p(a_d), ctypes.c_float(slope), _p(bias), _p(accum), acc_ld, _p(alpha), _p(out),
                      out.stride(0), _stream(xs))
        ctx.save_for_backward(xs, xd, att_s, att_d, a_s, a_d, alpha)
        ctx.graph, ctx.H, ctx.C, ctx.slope = graph, H, C, slope
        ctx.has_bias, ctx.has_accum = bias is not None, accum is not None
        ctx.att_shapes = (att_src.shape, att_dst.shape)
        return out

    @staticmethod
    def backward(ctx, g_out):
        xs, xd, att_s, att_d, a_s, a_d, alpha = ctx.saved_tensors
        graph, H, C, slope = ctx.graph, ctx.H, ctx.C, ctx.slope
        if a_s is None:   # the one-pass forward formed a_s on the fly (same arithmetic as hgin_gat_logits_f32)
            a_s = _logits(xs, att_s, H, C)
        g_out = g_out.contiguous()
        dev = g_out.device
        n_dst, n_src = graph.csr.n_rows, graph.csc.n_rows
        g_pre = torch.empty(graph.n_edges, H, dtype=torch.float32, device=dev)
        g_ad = torch.empty(n_dst, H, dtype=torch.float32, device=dev) if xd is not None else None
        g_xd = torch.empty(n_dst, H * C, dtype=torch.float32, device=dev) if xd is not None else None
        _lib.call("hgin_gat_bwd_dst_f32", _p(graph.csr.rowptr), _p(graph.csr.col), n_dst, H, C, _p(xs), xs.stride(0),
                  _p(g_out), g_out.stride(0), _p(alpha), _p(a_s), _p(a_d), ctypes.c_float(slope), _p(att_d), _p(g_pre),
                  _p(g_ad), _p(g_xd), g_xd.stride(0) if g_xd is not None else 0, _stream(g_out))
        g_as = torch.empty(n_src, H, dtype=torch.float32, device=dev)
        g_xs = torch.empty(n_src, H * C, dtype=torch.float32, device=dev)
        _lib.call("hgin_gat_bwd_src_f32", _p(graph.csc.rowptr), _p(graph.csc.col), _p(graph.cpos), n_src, H, C,
                  _p(g_out), g_out.stride(0), _p(alpha), _p(g_pre), _p(att_s), _p(g_as), _p(g_xs), g_xs.stride(0),
                  _stream(g_out))
        g_att_src = _wsum(xs, g_as, H, C).reshape(ctx.att_shapes[0]) if ctx.needs_input_grad[2] else None
        g_att_dst = None
        if xd is not None and ctx.needs_input_grad[3]:
            g_att_dst = _wsum(xd, g_ad, H, C).reshape(ctx.att_shapes[1])
        elif ctx.needs_input_grad[3]:
            g_att_dst = torch.zeros(ctx.att_shapes[1], dtype=torch.float32, device=dev)
        g_bias = _wsum(g_out, None, 1, H * C) if (ctx.has_bias and ctx.needs_input_grad[4]) else None
        g_acc = g_out if ctx.has_accum else None
        return g_xs, g_xd, g_att_src, g_att_dst, g_bias, g_acc, None, None, None, None


class GATConv(torch.nn.Module):
    """PyG 2.0.2 GATConv (see the module docstring) with HeteroConv's running sum fused into the output (accum)."""

    supports_accum = True

    def __init__(self, in_channels: Union[int, Tuple[int, int]], out_channels: int, heads: int = 1,
                 concat: bool = True, negative_slope: float = 0.2, dropout: float = 0.0, add_self_loops: bool = True,
                 bias: bool = True, **kwargs):
        super().__init__()
        if kwargs.get("aggr", "add") not in ("add", "sum"):
            raise NotImplementedError("hgin GATConv: aggr='add' only (PyG's default)")
        self.in_channels, self.out_channels = in_channels, out_channels
        self.heads, self.concat, self.negative_slope = heads, concat, negative_slope
        self.dropout, self.add_self_loops = dropout, add_self_loops
        if isinstance(in_channels, int):
            self.lin_src = Linear(in_channels, heads * out_channels, bias=False, weight_initializer="glorot")
            self.lin_dst = self.lin_src
        else:
            self.lin_src = Linear(in_channels[0], heads * out_channels, False, weight_initializer="glorot")
            self.lin_dst = Linear(in_channels[1], heads * out_channels, False, weight_initializer="glorot")
        self.att_src = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        self.att_dst = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        if bias and concat:
            self.bias = torch.nn.Parameter(torch.Tensor(heads * out_channels))
        elif bias:
            self.bias = torch.nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self) -> None:
        self.lin_src.reset_parameters()
        self.lin_dst.reset_parameters()
        glorot(self.att_src)
        glorot(self.att_dst)
        if self.bias is not None:
            self.bias.data.fill_(0)

    def forward(self, x, edge_index: Tensor, size=None, accum: Optional[Tensor] = None) -> Tensor:
        if not isinstance(edge_index, Tensor):
            raise NotImplementedError("hgin GATConv: SparseTensor adjacency is not supported")
        if self.dropout > 0.0 and self.training:
            raise NotImplementedError("hgin GATConv: attention dropout > 0 (the reference runs it at 0)")
        H, C = self.heads, self.out_channels
        if isinstance(x, Tensor):
            x_src = x_dst = self.lin_src(x)
        else:
            x_src, x_dst = x
            x_src = self.lin_src(x_src)
            if x_dst is not None:
                x_dst = self.lin_dst(x_dst)
        n_src = x_src.size(0)
        if x_dst is not None:
            n_dst = x_dst.size(0)
        elif size is not None:
            n_dst = int(size[1])
        else:
            n_dst = n_src
        if size is not None and self.add_self_loops:
            raise NotImplementedError("hgin GATConv: an explicit size with add_self_loops")
        graph = gat_graph(edge_index, n_src, n_dst, self.add_self_loops)
        if not self.concat:
            raise NotImplementedError("hgin GATConv: concat=False (mean over heads) is not used by HetroGAT")
        bias = self.bias
        if accum is not None and accum.shape != (n_dst, H * C):
            raise ValueError("hgin GATConv: accum shape")
        return _GatAttentionFn.apply(x_src.contiguous(), x_dst.contiguous() if x_dst is not None else None,
                                     self.att_src, self.att_dst, bias, accum, graph, H, C, float(self.negative_slope))
