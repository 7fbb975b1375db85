"""Autograd ops over libhgin.so (device tensors only — there is no CPU fallback).

Reference call path being replaced:
  GINConv.forward (models.py:201-217) -> MessagePassing.propagate (models.py:208: index_select +
  torch_scatter.scatter sum) -> cat / add of (1 + eps) * x_r (models.py:210-215) -> self.nn(out) =
  Linear + PReLU (models.py:236-239) ; HeteroConv's stack().sum(0) over relations into one node type.

Ops:
  * ``relation_graph(edge_index, n_src, n_dst)`` — validated stable CSR (by dst) + lazily a CSC (by src),
    cached on the edge_index tensor (invalidated by in-place edits through ``_version``).
  * ``aggregate(...)``      — A3/A4 fused aggregate + self term; autograd (backward: CSC aggregate +
                              deterministic combine backward).
  * ``gin_conv(...)``       — A3-A5 fused for the GINLayer case nn = Sequential(Linear, PReLU): aggregate
                              + combine -> MFMA GEMM with bias / PReLU / relation-sum epilogue; backward
                              PReLU+bias (deterministic), dW / dX GEMMs, CSC aggregate, eps grad.
"""
from __future__ import annotations

import ctypes
import os
from dataclasses import dataclass
from typing import Optional

import torch
from torch import Tensor

from . import _lib, profiling

COMBINE_NONE, COMBINE_ADD, COMBINE_CONCAT = 0, 1, 2
STATUS_ROW_OOR, STATUS_COL_OOR, STATUS_UNSORTED = 1, 2, 4


def _p(t: Optional[Tensor]):
    return None if t is None else ctypes.c_void_p(t.data_ptr())


def _stream(t: Tensor):
    return ctypes.c_void_p(torch.cuda.current_stream(t.device).cuda_stream)


def require_device(*tensors, what: str = "hgin") -> None:
    for t in tensors:
        if t is not None and not t.is_cuda:
            raise RuntimeError(f"{what}: expected HIP device tensors; the MI355X path has no CPU fallback "
                               f"(got a tensor on {t.device})")


def _f32(t: Tensor, what: str) -> Tensor:
    """Storage dtype check: float32, or bfloat16 for the cfg5 path (bf16 storage, fp32 arithmetic)."""
    if t.dtype not in (torch.float32, torch.bfloat16):
        raise TypeError(f"{what}: expected float32 or bfloat16, got {t.dtype}")
    return t


def _sfx(t: Tensor) -> str:
    """Entry-point suffix for a storage dtype (hgin_*_f32 / hgin_*_bf16)."""
    return "bf16" if t.dtype == torch.bfloat16 else "f32"


def _same_dtype(what: str, *ts) -> None:
    dts = {t.dtype for t in ts if t is not None}
    if len(dts) > 1:
        raise TypeError(f"{what}: mixed feature dtypes {sorted(map(str, dts))}")


def _as(t: Optional[Tensor], dtype) -> Optional[Tensor]:
    """A GEMM operand copy of an fp32 master parameter in the storage dtype (bf16 path)."""
    return t if (t is None or t.dtype == dtype) else t.to(dtype)


def _workspace(nbytes: int, device) -> Tensor:
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------------------------------
# A12: CSR / CSC
# ---------------------------------------------------------------------------------------------------
# Degree skew (SURVEY.md §8.D Zipf variant): rows with more than LONG_ROW_MIN edges leave the row-per-lane-group
# walk (serial in a row's edges) for the chunked long-row kernels (hgin_aggregate_long_*, LONG_CHUNK edges per
# wave, chunk sums added in a fixed order: deterministic, re-associated).  Uniform GIN graphs (max in-degree
# ~40 at cfg3) never reach it, so their aggregates stay bit-exact.  HGIN_LONG_ROW=0 keeps every row sequential.
LONG_ROW_MIN = int(os.environ.get("HGIN_LONG_ROW", "2048"))
# fp32 split mode: the 128 x 128 NT tile copies its B stages from pre-split planes by LDS-DMA (k_gemm_nt kBdma);
# HGIN_NT_BDMA=0 keeps the per-tile split
BDMA = os.environ.get("HGIN_NT_BDMA", "1") != "0" and os.environ.get("HGIN_F32_GEMM", "split") != "mfma32"
# libhgin's weight-stationary fp32 forms (try_ws_f32 / try_ws_f32_comb) take K = N = 256 with one A source before
# the tiled kernel is considered; they read W directly, so no split planes are built for them
WS32 = os.environ.get("HGIN_NT_WS32", "1")[:1] != "0" and os.environ.get("HGIN_F32_GEMM", "split") != "mfma32"
LONG_CHUNK = 1024
# the first layer's fp32 K = 512 dW without an input gradient: the weight-stationary PReLU-fused pass over columns
# [0, 256) (storing g_z into a scratch) + a plain pass over [256, 512) (10.85 vs 12.33 ms at M = 6M on the tiled fused
# kernel, profiles/r04/gpu_a/gemm_ab_*.json; the round-4 switch to the tiled form is gone)
DW512_WSD = True


@dataclass
class LongRows:
    rowptr_short: Tensor   # int32 [n_rows + 1]: the CSR with the long rows emptied
    col_short: Tensor      # int32 [E - long edges]
    long_rows: Tensor      # int32 [n_long]
    item_ptr: Tensor       # int32 [n_long + 1]
    items: Tensor          # int32 [2 * n_items]: (begin, end) edge ranges into the full col, per row in edge order
    n_items: int


@dataclass
class Csr:
    rowptr: Tensor   # int32 [n_rows + 1]
    col: Tensor      # int32 [E]   other endpoint, in stable sorted order
    perm: Tensor     # int32 [E]   original edge id of each sorted position
    n_rows: int
    n_cols: int
    long: Optional[LongRows] = None

    @property
    def n_edges(self) -> int:
        return int(self.col.numel())


def split_long_rows(csr: Csr, min_deg: int = None, chunk: int = None) -> Csr:
    """Attach the long-row split of ``csr`` (rows with more than ``min_deg`` edges), if it has any."""
    min_deg = LONG_ROW_MIN if min_deg is None else int(min_deg)
    chunk = LONG_CHUNK if chunk is None else int(chunk)
    csr.long = None
    if min_deg <= 0 or csr.n_edges == 0 or csr.n_rows == 0:
        return csr
    rp = csr.rowptr.long()
    deg = rp[1:] - rp[:-1]
    if int(deg.max()) <= min_deg:          # one host sync per CSR build (cached with the graph)
        return csr
    is_long = deg > min_deg
    long_rows = torch.nonzero(is_long).flatten()
    d = deg[long_rows]
    nch = (d + chunk - 1) // chunk
    item_ptr = torch.cat([torch.zeros(1, dtype=torch.long, device=d.device), torch.cumsum(nch, 0)])
    n_items = int(item_ptr[-1])
    row_of_item = torch.repeat_interleave(torch.arange(long_rows.numel(), device=d.device), nch)
    local = torch.arange(n_items, device=d.device) - item_ptr[row_of_item]
    beg = rp[long_rows][row_of_item] + local * chunk
    end = torch.minimum(beg + chunk, rp[long_rows + 1][row_of_item])
    deg_short = torch.where(is_long, torch.zeros_like(deg), deg)
    rowptr_short = torch.cat([torch.zeros(1, dtype=torch.long, device=d.device), torch.cumsum(deg_short, 0)])
    keep = torch.repeat_interleave(~is_long, deg)
    csr.long = LongRows(rowptr_short.to(torch.int32), csr.col[keep].contiguous(), long_rows.to(torch.int32),
                        item_ptr.to(torch.int32), torch.stack([beg, end], 1).to(torch.int32).reshape(-1).contiguous(),
                        n_items)
    return csr


def build_csr(edge_index: Tensor, key_row: int, n_rows: int, n_cols: int, validate: bool = True) -> Csr:
    """Stable COO->CSR of a [2, E] int64 edge_index on the device (key_row 1: by dst, 0: by src)."""
    require_device(edge_index, what="build_csr")
    check_edge_index(edge_index)
    ei = edge_index.contiguous()
    E = int(ei.size(1))
    dev = ei.device
    rowptr = torch.empty(n_rows + 1, dtype=torch.int32, device=dev)
    col = torch.empty(E, dtype=torch.int32, device=dev)
    perm = torch.empty(E, dtype=torch.int32, device=dev)
    status = torch.zeros(1, dtype=torch.int32, device=dev)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_csr_workspace_size(E, n_rows, ctypes.byref(nbytes)), "hgin_csr_workspace_size")
    ws = _workspace(nbytes.value, dev)
    _lib.call("hgin_csr_build", _p(ei), E, key_row, n_rows, n_cols, _p(rowptr), _p(col), _p(perm), _p(status),
              _p(ws), nbytes.value, _stream(ei))
    if validate:
        st = int(status.item())
        if st:
            which = []
            if st & STATUS_ROW_OOR:
                which.append(f"{'dst' if key_row == 1 else 'src'} index out of range [0, {n_rows})")
            if st & STATUS_COL_OOR:
                which.append(f"{'src' if key_row == 1 else 'dst'} index out of range [0, {n_cols})")
            raise IndexError("edge_index: " + "; ".join(which))
    return split_long_rows(Csr(rowptr, col, perm, n_rows, n_cols))


def check_edge_index(edge_index: Tensor) -> None:
    """PyG 2.0.x MessagePassing.__check_input__ for Tensor adjacency (AssertionError on violation)."""
    assert edge_index.dtype == torch.long, "edge_index must be torch.long"
    assert edge_index.dim() == 2, "edge_index must be 2-dimensional"
    assert edge_index.size(0) == 2, "edge_index must have shape [2, num_edges]"


class RelationGraph:
    """CSR (by dst) for the forward aggregate + CSC (by src) for the backward, built once per edge_index."""

    def __init__(self, edge_index: Tensor, n_src: int, n_dst: int):
        self.edge_index = edge_index
        self.n_src = int(n_src)
        self.n_dst = int(n_dst)
        self._csr: Optional[Csr] = None
        self._csc: Optional[Csr] = None

    @property
    def n_edges(self) -> int:
        return int(self.edge_index.size(1))

    @property
    def csr(self) -> Csr:
        if self._csr is None:
            self._csr = build_csr(self.edge_index, 1, self.n_dst, self.n_src)
        return self._csr

    @property
    def csc(self) -> Csr:
        if self._csc is None:
            # the CSR build already validated both endpoint ranges
            self._csc = build_csr(self.edge_index, 0, self.n_src, self.n_dst, validate=self._csr is None)
        return self._csc


def attach_relation_graph(edge_index: Tensor, n_src: int, n_dst: int, csr: Csr, csc: Optional[Csr]) -> RelationGraph:
    """Register prebuilt CSR / CSC for this edge_index (F1 device collation builds them without a sort)."""
    g = RelationGraph(edge_index, n_src, n_dst)
    g._csr, g._csc = csr, csc
    edge_index._hgin_graphs = (edge_index._version, {(int(n_src), int(n_dst)): g})
    return g


def relation_graph(edge_index: Tensor, n_src: int, n_dst: int) -> RelationGraph:
    """Cached RelationGraph for this edge_index tensor (cache lives on the tensor, keyed by sizes)."""
    key = (int(n_src), int(n_dst))
    cache = getattr(edge_index, "_hgin_graphs", None)
    ver = edge_index._version
    if cache is None or cache[0] != ver:
        cache = (ver, {})
        try:
            edge_index._hgin_graphs = cache
        except (AttributeError, RuntimeError):
            return RelationGraph(edge_index, n_src, n_dst)
    g = cache[1].get(key)
    if g is None:
        g = RelationGraph(edge_index, n_src, n_dst)
        g.csr  # build + validate eagerly (errors surface at the call site, like PyG's)
        cache[1][key] = g
    return g


# ---------------------------------------------------------------------------------------------------
# raw launches
# ---------------------------------------------------------------------------------------------------
def _long_ok(lr: Optional[LongRows], x_src: Tensor, x_dst: Optional[Tensor], out: Tensor, mode: int) -> bool:
    """Whether the long-row kernels take these operands (4-wide rows; otherwise every row walks serially)."""
    if lr is None:
        return False
    f = int(x_src.size(1))
    ok = f % 4 == 0 and x_src.stride(0) % 4 == 0 and out.stride(0) % 4 == 0
    ok = ok and x_src.data_ptr() % (4 * x_src.element_size()) == 0 and out.data_ptr() % (4 * out.element_size()) == 0
    if mode == COMBINE_ADD:
        ok = ok and x_dst.stride(0) % 4 == 0 and x_dst.data_ptr() % (4 * x_dst.element_size()) == 0
    return ok


def aggregate_into(csr: Csr, x_src: Tensor, x_dst: Optional[Tensor], eps: Optional[Tensor], mode: int,
                   out: Tensor) -> Tensor:
    f_src = int(x_src.size(1))
    f_dst = int(x_dst.size(1)) if x_dst is not None else 0
    lr = csr.long if _long_ok(csr.long, x_src, x_dst, out, mode) else None

    def launch():
        rowptr, col = (lr.rowptr_short, lr.col_short) if lr is not None else (csr.rowptr, csr.col)
        _lib.call(f"hgin_aggregate_{_sfx(x_src)}", _p(rowptr), _p(col), csr.n_rows, _p(x_src),
                  x_src.stride(0), f_src, _p(x_dst), x_dst.stride(0) if x_dst is not None else 0, f_dst, _p(eps),
                  mode, _p(out), out.stride(0), _stream(out))
        if lr is not None:
            part = torch.empty(lr.n_items * f_src, dtype=torch.float32, device=out.device)
            _lib.call(f"hgin_aggregate_long_{_sfx(x_src)}", _p(csr.col), _p(lr.items), lr.n_items, _p(lr.long_rows),
                      _p(lr.item_ptr), lr.long_rows.numel(), _p(x_src), x_src.stride(0), f_src, _p(x_dst),
                      x_dst.stride(0) if x_dst is not None else 0, f_dst, _p(eps), mode, _p(out), out.stride(0),
                      _p(part), part.numel() * 4, _stream(out))

    probe = profiling.active()
    if probe is None:
        launch()
    else:
        probe.around("aggregate", profiling.aggregate_bytes(csr.n_edges, csr.n_rows, f_src, f_dst, mode,
                                                            x_src.element_size()), launch)
    return out


def _rowmajor(t: Tensor) -> Tensor:
    return t if (t.dim() == 2 and t.stride(1) == 1) else t.contiguous()


def prelu_bwd(g_y: Tensor, z: Tensor, prelu: Tensor):
    M, N = z.shape
    g_z = torch.empty_like(z)
    g_a = torch.empty(1, dtype=torch.float32, device=z.device)
    g_b = torch.empty(N, dtype=torch.float32, device=z.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_prelu_bwd_workspace_size(M, N, ctypes.byref(nbytes)), "prelu_bwd_workspace_size")
    ws = _workspace(nbytes.value, z.device)
    _same_dtype("prelu_bwd", g_y, z)
    _lib.call(f"hgin_prelu_bwd_{_sfx(z)}", _p(g_y), g_y.stride(0), _p(z), M, N, _p(prelu), _p(g_z), _p(g_a), _p(g_b),
              _p(ws), nbytes.value, _stream(z))
    return g_z, g_a, g_b


def combine_bwd(g: Tensor, x_dst: Tensor, eps: Tensor, want_gx: bool):
    n, f = x_dst.shape
    gx = torch.empty_like(x_dst) if want_gx else None
    g_eps = torch.empty(1, dtype=torch.float32, device=x_dst.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_combine_bwd_workspace_size(n, ctypes.byref(nbytes)), "combine_bwd_workspace_size")
    ws = _workspace(nbytes.value, x_dst.device)
    _same_dtype("combine_bwd", g, x_dst)
    _lib.call(f"hgin_combine_bwd_{_sfx(x_dst)}", _p(g), g.stride(0), _p(x_dst), x_dst.stride(0), n, f, _p(eps),
              _p(gx), gx.stride(0) if gx is not None else 0, _p(g_eps), _p(ws), nbytes.value, _stream(x_dst))
    return gx, g_eps


def nt_planes(b: Tensor, M: int = 1 << 20, ws_form: bool = False) -> Optional[Tensor]:
    """The fp32 B operand [N, K] of an NT GEMM pre-converted into its three bf16 split planes (hgin_nt_planes_f32,
    N * K * 6 bytes), which the split-mode 128 x 128 tile copies into LDS by DMA instead of splitting B per tile
    (bit-identical), or None where that kernel does not take the shape: ``ws_form`` = the call qualifies for
    libhgin's weight-stationary form (which reads W itself), and M = 0 launches nothing."""
    if not (BDMA and b.dtype == torch.float32) or M == 0:
        return None
    N, K = b.shape
    if ws_form and WS32 and N == 256 and K in (128, 256, 512):
        return None
    if N == 0 or K == 0 or K % 32 or b.stride(1) != 1:
        return None
    if N % 128 or b.data_ptr() % 16 or b.stride(0) % 4:
        return None
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_nt_planes_size(N, K, b.element_size(), ctypes.byref(nbytes)), "hgin_nt_planes_size")
    out = torch.empty(nbytes.value, dtype=torch.uint8, device=b.device)
    _lib.call(f"hgin_nt_planes_{_sfx(b)}", _p(b), b.stride(0), N, K, _p(out), _stream(b))
    return out


def gemm_nt(a: Tensor, b: Tensor) -> Tensor:
    """c = a @ b^T on the matrix cores (a [M,K], b [N,K], both K-contiguous; c in the operands' dtype)."""
    a, b = _rowmajor(a), _rowmajor(b)
    _same_dtype("gemm_nt", a, b)
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty(M, N, dtype=a.dtype, device=a.device)
    planes = nt_planes(b, M, ws_form=N == 256 and K in (128, 256))   # (k_wss_f32 EPI 5 reads W itself)
    _probed("gemm_dx", 2.0 * M * N * K, a.element_size() * (M * K + N * K + M * N),
            lambda: _lib.call(f"hgin_gemm_nt_{_sfx(a)}", _p(a), a.stride(0), _p(b), b.stride(0), _p(c), c.stride(0),
                              M, N, K, _p(planes), _stream(a)))
    return c


def _probed(kind: str, flops: float, nbytes: float, launch) -> None:
    """Run ``launch``; inside a profiling window, timed with HIP events as ``kind`` (work = FLOPs, plus its
    algorithmic HBM bytes)."""
    probe = profiling.active()
    if probe is None:
        launch()
    else:
        probe.around(kind, flops, launch, nbytes)


def gemm_nt_combine(a: Tensor, b: Tensor, x_dst: Tensor, eps: Tensor, cs: int, want_gx: bool,
                    g_prev: Optional[Tensor] = None):
    """(c, g_x_dst, g_eps): c = a @ b^T, g_x_dst = (1 + eps) c[:, cs:] [+ g_prev, in place], g_eps =
    sum(c[:, cs:] * x_dst) in one GEMM launch + a final sum (hgin_gemm_nt_combine_*): the dX GEMM of a GINConv
    backward with the self term's backward in its epilogue."""
    a, b = _rowmajor(a), _rowmajor(b)
    _same_dtype("gemm_nt_combine", a, b, x_dst, g_prev)
    M, K = a.shape
    N = b.shape[0]
    c = torch.empty(M, N, dtype=a.dtype, device=a.device)
    if g_prev is not None:
        assert want_gx and g_prev.shape == (M, N - cs) and g_prev.stride(1) == 1
        gx = g_prev                      # accumulated in place
    else:
        gx = torch.empty(M, N - cs, dtype=a.dtype, device=a.device) if want_gx else None
    g_eps = torch.empty(1, dtype=torch.float32, device=a.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_gemm_nt_combine_workspace_size(M, N, ctypes.byref(nbytes)), "nt_combine_workspace")
    ws = _workspace(nbytes.value, a.device)
    s = a.element_size()
    nb = s * (M * K + N * K + M * N + M * (N - cs) * (1 + int(gx is not None) + int(g_prev is not None)))
    planes = nt_planes(b, M, ws_form=cs == 0 and b.stride(0) == K)
    _probed("gemm_dx", 2.0 * M * N * K, nb,
            lambda: _lib.call(f"hgin_gemm_nt_combine_{_sfx(a)}", _p(a), a.stride(0), _p(b), b.stride(0), _p(c),
                              c.stride(0), M, N, K, _p(x_dst), x_dst.stride(0), _p(gx),
                              gx.stride(0) if gx is not None else 0, _p(g_prev),
                              g_prev.stride(0) if g_prev is not None else 0, cs, _p(eps), _p(g_eps),
                              _p(ws), nbytes.value, _p(planes), _stream(a)))
    return c, gx, g_eps


def gemm_tn(a: Tensor, b1: Tensor, b2: Optional[Tensor] = None) -> Tensor:
    """out[N, K] (fp32) = a[M, N]^T @ [b1 | b2] (weight gradients), split-M MFMA + deterministic slab reduce."""
    a, b1 = _rowmajor(a), _rowmajor(b1)
    if b2 is not None:
        b2 = _rowmajor(b2)
    _same_dtype("gemm_tn", a, b1, b2)
    M, N = a.shape
    k1 = b1.shape[1]
    K = k1 + (b2.shape[1] if b2 is not None else 0)
    out = torch.empty(N, K, dtype=torch.float32, device=a.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_gemm_tn_workspace_size(M, N, K, ctypes.byref(nbytes)), "gemm_tn_workspace_size")
    ws = _workspace(nbytes.value, a.device)
    _probed("gemm_dw", 2.0 * M * N * K, a.element_size() * M * (N + K) + 4 * N * K,
            lambda: _lib.call(f"hgin_gemm_tn_{_sfx(a)}", _p(a), a.stride(0), _p(b1), b1.stride(0), k1, _p(b2),
                              b2.stride(0) if b2 is not None else 0, M, N, K, _p(out), out.stride(0), _p(ws),
                              nbytes.value, _stream(a)))
    return out


def mlp_bwd_fused(z: Tensor, n: int, k: int) -> bool:
    """True where libhgin runs the PReLU backward inside the dW GEMM (fp32, N and K >= 16)."""
    return z.dtype == torch.float32 and n >= 16 and k >= 16


def mlp_bwd_w(g_y: Tensor, z: Tensor, prelu: Tensor, b1: Tensor, b2: Optional[Tensor] = None,
              want_gz: bool = False, y_alt: Optional[Tensor] = None):
    """Backward of prelu([b1 | b2] @ W^T + b) up to the weights: (g_w [N, K] fp32, g_a [1], g_b [N], g_z).

    g_z = z > 0 ? g_y : a * g_y is formed inside the weight-gradient GEMM where fused (mlp_bwd_fused) and
    then returned as None unless ``want_gz``; otherwise (bf16, narrow layers) it is materialised — by the
    weight-stationary dW itself where it takes the shape (k_wsd_*<..., prelu_bwd_fused>: g_z formed in its LDS
    staging and stored, no separate PReLU-backward pass), else by hgin_prelu_bwd_* ahead of the TN GEMM.
    ``y_alt``: the forward's y when it ran with zy (gin_mlp_fwd): read in place of z when the slope is > 0
    (hgin_gin_mlp_bwd_w_zy_bf16)."""
    g_y, b1 = _rowmajor(g_y), _rowmajor(b1)
    if b2 is not None:
        b2 = _rowmajor(b2)
    _same_dtype("mlp_bwd_w", g_y, z, b1, b2)
    M, N = z.shape
    k1 = b1.shape[1]
    K = k1 + (b2.shape[1] if b2 is not None else 0)
    dev = z.device
    fused = mlp_bwd_fused(z, N, K)
    # the first layer's fp32 K = 512 dW (no input gradient, so g_z is not wanted): through the weight-stationary
    # two-pass form (PReLU-fused pass over columns [0, 256) storing g_z into a scratch, plain pass over [256, 512) on
    # it) instead of the tiled fused kernel
    scratch_gz = fused and not want_gz and z.dtype == torch.float32 and N == 256 and K == 512 and DW512_WSD
    g_z = torch.empty_like(z) if (want_gz or not fused or scratch_gz) else None
    g_w = torch.empty(N, K, dtype=torch.float32, device=dev)
    g_a = torch.empty(1, dtype=torch.float32, device=dev)
    g_b = torch.empty(N, dtype=torch.float32, device=dev)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_gin_mlp_bwd_w_workspace_size(M, N, K, z.element_size(), int(g_z is not None),
                                                            ctypes.byref(nbytes)), "gin_mlp_bwd_w_workspace_size")
    ws = _workspace(nbytes.value, dev)
    s = z.element_size()
    # algorithmic: g_y, z and B read once, g_z written when it is returned (the weight-stationary kernels form it in
    # their staging and store it; elsewhere a separate PReLU-backward pass writes it and the TN GEMM reads it back)
    nb = s * M * (2 * N + K + (N if g_z is not None else 0)) + 4 * N * K
    if y_alt is not None:
        if not (z.dtype == torch.bfloat16 and g_z is not None and z.is_contiguous() and y_alt.shape == z.shape
                and y_alt.dtype == z.dtype and y_alt.is_contiguous()):
            raise RuntimeError("mlp_bwd_w: y_alt needs the bf16 z-from-y layout (dense [M, N] z and y)")
        _probed("gemm_dw", 2.0 * M * N * K, nb,
                lambda: _lib.call("hgin_gin_mlp_bwd_w_zy_bf16", _p(g_y), g_y.stride(0), _p(z), _p(y_alt), _p(prelu),
                                  _p(b1), b1.stride(0), k1, _p(b2), b2.stride(0) if b2 is not None else 0, M, N, K,
                                  _p(g_w), g_w.stride(0), _p(g_a), _p(g_b), _p(g_z), N, _p(ws), nbytes.value,
                                  _stream(z)))
        return g_w, g_a, g_b, g_z
    _probed("gemm_dw", 2.0 * M * N * K, nb,
            lambda: _lib.call(f"hgin_gin_mlp_bwd_w_{_sfx(z)}", _p(g_y), g_y.stride(0), _p(z), z.stride(0), _p(prelu),
                              _p(b1), b1.stride(0), k1, _p(b2), b2.stride(0) if b2 is not None else 0, M, N, K,
                              _p(g_w), g_w.stride(0), _p(g_a), _p(g_b), _p(g_z), N, _p(ws), nbytes.value, _stream(z)))
    return g_w, g_a, g_b, (None if scratch_gz else g_z)


def self_wgrad(G: Tensor, weight: Tensor, f: int, concat: bool, eps: Tensor):
    """(g_w, g_eps) of a first-layer GINConv from G = g_z^T [aggregate | x_dst] (hgin_self_wgrad_f32):
    g_w = [G[:, :f] | (1 + eps) G[:, f:]] (concat) or G[:, :f] (add); g_eps = sum(W_self * G[:, f:])."""
    N, KG = G.shape
    w = weight if weight.dtype == torch.float32 else weight.float()   # bf16 path: the GEMM's operand copy
    g_w = torch.empty(N, KG if concat else f, dtype=torch.float32, device=G.device)
    g_eps = torch.empty(1, dtype=torch.float32, device=G.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_self_wgrad_workspace_size(N, KG, ctypes.byref(nbytes)), "self_wgrad_workspace_size")
    ws = _workspace(nbytes.value, G.device)
    _lib.call("hgin_self_wgrad_f32", _p(G), G.stride(0), _p(w), w.stride(0), N, KG, f, int(concat), _p(eps), _p(g_w),
              g_w.stride(0), _p(g_eps), _p(ws), nbytes.value, _stream(G))
    return g_w, g_eps


def zy_form(N: int, K: int) -> bool:
    """Shapes whose bf16 forward is the weight-stationary k_ws_bf16 (N in {128, 256}, K in {128, 256, 512}), the
    only kernel that skips z under zy.  Elsewhere the forward writes z anyway, and a y_alt backward would only add a
    restore pass (k_zy_restore) over it — the readout's Linear(128, 32): 0.34 ms per cfg5 step."""
    return N in (128, 256) and K in (128, 256, 512)


def gin_mlp_fwd(comb: Tensor, weight: Tensor, bias: Tensor, prelu: Optional[Tensor], accum: Optional[Tensor],
                save_z: bool = True, comb2: Optional[Tensor] = None, eps2: Optional[Tensor] = None,
                zy: bool = False):
    """y = prelu([comb | s * comb2] @ W^T + b) [+ accum]  (prelu None: plain Linear, y = z, nothing saved);
    s = 1 + eps2[0] when ``eps2`` is given (the concat GINConv's self term formed in the GEMM's loads), else 1.

    fp32 storage: everything fp32.  bf16 storage (cfg5): comb / comb2 / weight / accum / z / y bf16, bias and
    prelu fp32; the plain Linear (the readout head) returns fp32.

    ``zy`` (bf16, no accum, z kept): hgin_gin_mlp_fwd_zy_bf16 — with a positive slope the kernel may leave z unwritten
    (y = prelu(z) determines it); its backward must then be mlp_bwd_w(..., y_alt=y)."""
    M, k1 = comb.shape
    K = k1 + (comb2.shape[1] if comb2 is not None else 0)
    N = weight.shape[0]
    _same_dtype("gin_mlp_fwd", comb, comb2, weight, accum)
    sfx = _sfx(comb)
    dt = comb.dtype
    z = torch.empty(M, N, dtype=dt, device=comb.device) if (save_z and prelu is not None) else None
    y = torch.empty(M, N, dtype=dt if prelu is not None else torch.float32, device=comb.device)
    ld2 = comb2.stride(0) if comb2 is not None else 0
    # ws_form: libhgin's weight-stationary kernels take the call and read W themselves — K = N = 256 with one source,
    # or the first layer's [aggregate | (1 + eps) x_dst] at 256 + 256 without accum (two k_wss_f32 passes)
    ws_form = prelu is not None and ((comb2 is None and K == 256) or
                                     (eps2 is not None and accum is None and k1 == 256 and K == 512))
    planes = nt_planes(weight, M, ws_form=ws_form) if weight.stride(1) == 1 else None
    zy = zy and dt == torch.bfloat16 and prelu is not None and accum is None and z is not None

    def launch():
        if prelu is None:
            _lib.call(f"hgin_linear_fwd_{sfx}", _p(comb), comb.stride(0), k1, _p(comb2), ld2, _p(weight), _p(bias),
                      _p(y), M, N, K, _p(planes), _stream(comb))
        elif zy:
            _lib.call("hgin_gin_mlp_fwd_zy_bf16", _p(comb), comb.stride(0), k1, _p(comb2), ld2, _p(eps2), _p(weight),
                      _p(bias), _p(prelu), _p(z), _p(y), M, N, K, _stream(comb))
        else:
            _lib.call(f"hgin_gin_mlp_fwd_{sfx}", _p(comb), comb.stride(0), k1, _p(comb2), ld2, _p(eps2), _p(weight),
                      _p(bias), _p(prelu), _p(accum), _p(z), _p(y), M, N, K, _p(planes), _stream(comb))

    probe = profiling.active()
    if probe is None:
        launch()
    else:
        # (the untimed probe pass may sync: with zy the weight-stationary kernel writes no z when the slope is > 0)
        z_written = z is not None and not (zy and zy_form(N, K) and float(prelu) > 0)
        probe.around("gin_mlp" if prelu is not None else "linear", 2.0 * M * N * K, launch,
                     profiling.gemm_bytes(M, N, K, comb.element_size(), z_written, accum is not None))
    return z, y


# ---------------------------------------------------------------------------------------------------
# autograd
# ---------------------------------------------------------------------------------------------------
_ZERO = {}


def _zero(device) -> Tensor:
    t = _ZERO.get(device)
    if t is None:
        t = _ZERO[device] = torch.zeros(1, dtype=torch.float32, device=device)
    return t


LAZY_SELF = True     # tests compare the lazy self-term gradient with the materialised one (bit-identical)


class _LazySelf:
    """A node type's running gradient that is still only (1 + eps) C: the first self-term contribution of an ADD-mode
    GINConv (C = its g_comb), kept unmaterialised when the next use is a CSC aggregate's running gradient, which then
    applies it as its own self term — the dX GEMM skips its g_x_dst stream (N_dst x F stores) and the aggregate reads C
    instead of g_x_dst: the same sum, fl(fl(1 + eps) C) added after the edge sum in both."""
    __slots__ = ("c", "eps")

    def __init__(self, c: Tensor, eps: Tensor):
        self.c, self.eps = c, eps


def _backward_aggregate(graph: RelationGraph, g_agg: Tensor, prev=None) -> Tensor:
    """d x_src = index_add over the reversed relation = the A3 kernel on the CSC (edge order kept).  ``prev``:
    a running gradient of the source type, added in the same pass (ADD self term with eps 0: prev + sum) into a
    fresh buffer — the same HBM bytes as accumulating in place (prev read once, the sum written once), without
    aliasing the kernels' restrict-qualified x_dst / out (include/hgin.h: out must not overlap any input)."""
    csc = graph.csc
    if isinstance(prev, _LazySelf):
        out = torch.empty_like(prev.c)
        return aggregate_into(csc, g_agg, prev.c, prev.eps, COMBINE_ADD, out)
    if prev is not None:
        out = torch.empty_like(prev)
        return aggregate_into(csc, g_agg, prev, _zero(g_agg.device), COMBINE_ADD, out)
    g = torch.empty(graph.n_src, g_agg.size(1), dtype=g_agg.dtype, device=g_agg.device)
    return aggregate_into(csc, g_agg, None, None, COMBINE_NONE, g)


class _AggregateFn(torch.autograd.Function):
    """propagate + self term (generic path: any nn applied by the caller)."""

    @staticmethod
    def forward(ctx, x_src, x_dst, eps, graph: RelationGraph, mode: int):
        f_src = x_src.size(1)
        width = f_src + (x_dst.size(1) if mode == COMBINE_CONCAT else 0)
        out = torch.empty(graph.n_dst, width, dtype=x_src.dtype, device=x_src.device)
        aggregate_into(graph.csr, x_src, x_dst, eps, mode, out)
        ctx.graph, ctx.mode, ctx.f_src = graph, mode, f_src
        ctx.save_for_backward(x_dst, eps)
        return out

    @staticmethod
    def backward(ctx, g_out):
        x_dst, eps = ctx.saved_tensors
        g_out = _rowmajor(g_out)
        need_src, need_dst, need_eps = ctx.needs_input_grad[:3]
        g_src = g_dst = g_eps = None
        if need_src:
            g_src = _backward_aggregate(ctx.graph, g_out[:, :ctx.f_src])
        if ctx.mode != COMBINE_NONE and (need_dst or need_eps):
            gs = g_out[:, ctx.f_src:] if ctx.mode == COMBINE_CONCAT else g_out
            g_dst, g_eps = combine_bwd(gs, x_dst, eps, need_dst)
        return g_src, g_dst, (g_eps.view_as(eps) if need_eps and g_eps is not None else None), None, None


def _gin_forward(x_src, x_dst, eps, weight, bias, prelu, accum, graph: RelationGraph, mode: int, data_inputs: bool,
                 zy: bool = False):
    """One GINConv + GINLayer MLP forward: y = prelu(comb @ W^T + b) [+ accum], comb = aggregate + self term.
    Returns (y, w_op, comb, z) — what the backward needs besides x_dst / eps / prelu.  ``zy``: gin_mlp_fwd's z-from-y
    mode (bf16 without accum); the backward then takes y_alt = y."""
    f_src = x_src.size(1)
    w_op = _as(weight, x_src.dtype)          # bf16 path: the GEMM reads a bf16 copy of the fp32 master
    if mode == COMBINE_CONCAT and data_inputs:
        # inputs are data (the first layer): the backward never needs the concat, so the self half
        # (1 + eps) x_dst is formed in the GEMM's tile loads instead of being written by the aggregate and
        # read back (2 * N_dst * F_dst * s bytes less per relation); comb holds the aggregate only
        comb = torch.empty(graph.n_dst, f_src, dtype=x_src.dtype, device=x_src.device)
        aggregate_into(graph.csr, x_src, None, None, COMBINE_NONE, comb)
        if x_src.dtype == torch.bfloat16 and eps is not None and weight.dtype == torch.float32:
            # bf16 storage: (1 + eps) is folded into the self half of the weight operand, [W_agg | (1 + eps) W_self]
            # rounded to bf16 once from the fp32 master, instead of bf16((1 + eps) x_dst) on every row — the same
            # product with one bf16 rounding fewer and no eps-scaling pass in the GEMM (k_ws_bf16 K = 512: 3.31 ->
            # 2.78 ms at M = 6M, profiles/r03/s17).  The backward keeps the unfolded operand (dW, eps gradient).
            w_f = torch.cat((weight[:, :f_src], weight[:, f_src:] * (1.0 + eps)), 1).to(torch.bfloat16)
            z, y = gin_mlp_fwd(comb, w_f, bias, prelu, accum, comb2=x_dst, zy=zy)
        else:
            z, y = gin_mlp_fwd(comb, w_op, bias, prelu, accum, comb2=x_dst, eps2=eps, zy=zy)
    else:
        width = f_src + (x_dst.size(1) if mode == COMBINE_CONCAT else 0)
        comb = torch.empty(graph.n_dst, width, dtype=x_src.dtype, device=x_src.device)
        aggregate_into(graph.csr, x_src, x_dst, eps, mode, comb)
        z, y = gin_mlp_fwd(comb, w_op, bias, prelu, accum, zy=zy)
    return y, w_op, comb, z


def _gin_backward(g_y, x_dst, eps, weight, prelu, comb, z, graph: RelationGraph, mode: int, f_src: int,
                  need_src: bool, need_dst: bool, need_eps: bool, need_w: bool,
                  g_src_prev=None, g_dst_prev: Optional[Tensor] = None,
                  y_alt: Optional[Tensor] = None, lazy_dst: bool = False):
    """Backward of _gin_forward: (g_src, g_dst, g_eps, g_w, g_b, g_a).  ``g_src_prev`` / ``g_dst_prev``: running
    gradients of the source / destination node type from other relations, which g_src / g_dst accumulate onto
    in place inside the CSC aggregate (ADD mode, eps 0) and the dX GEMM's epilogue — autograd's sum over the
    relations sharing a node type without separate add kernels (the returned tensors are then those buffers).
    ``lazy_dst`` (ADD mode, no g_dst_prev): g_dst is returned as a _LazySelf for the caller's next CSC aggregate of the
    same node type, and the dX GEMM writes no g_x_dst; ``g_src_prev`` may be such a _LazySelf."""
    g_y = _rowmajor(g_y)
    g_w = g_src = g_dst = g_eps = None
    if need_src or need_dst:
        # (a side stream overlapping dW with the dX GEMM + CSC aggregate measured 1 % slower on cfg2 / cfg2bf:
        # each of these kernels already fills the 256 CUs)
        g_w, g_a, g_b, g_z = mlp_bwd_w(g_y, z, prelu, comb, want_gz=True, y_alt=y_alt)
        cs = f_src if mode == COMBINE_CONCAT else 0
        if mode != COMBINE_NONE and cs % 4 == 0 and x_dst.stride(1) == 1:
            # dX = g_z W [N_dst, K] with the self term's backward in the GEMM epilogue
            lazy = lazy_dst and need_dst and mode == COMBINE_ADD and g_dst_prev is None
            g_comb, g_dst, g_eps = gemm_nt_combine(g_z, weight.t().contiguous(), x_dst, eps, cs, need_dst and not lazy,
                                                   g_prev=g_dst_prev if need_dst else None)
            if lazy:
                g_dst = _LazySelf(g_comb, eps)
        else:
            g_comb = gemm_nt(g_z, weight.t().contiguous())      # dX = g_z W   [N_dst, K]
            if mode != COMBINE_NONE:
                g_dst, g_eps = combine_bwd(g_comb[:, cs:], x_dst, eps, need_dst)
                if g_dst is not None and g_dst_prev is not None:
                    g_dst = g_dst_prev.add_(g_dst)
        if need_src:
            g_src = _backward_aggregate(graph, g_comb[:, :f_src], g_src_prev)
    elif need_eps and mode != COMBINE_NONE:
        # Only parameters need gradients (the first layer, whose inputs are data):
        # sum(g_comb[:, self] * x_dst) = sum(W_self * (g_z^T x_dst)), so one TN pass over
        # [aggregate | x_dst] yields dW and the eps gradient and the [N_dst, K] dX GEMM is skipped.
        if mode == COMBINE_CONCAT:
            G, g_a, g_b, _ = mlp_bwd_w(g_y, z, prelu, comb[:, :f_src], x_dst, y_alt=y_alt)
        else:
            G, g_a, g_b, _ = mlp_bwd_w(g_y, z, prelu, comb, x_dst, y_alt=y_alt)
        g_w, g_eps = self_wgrad(G, weight, f_src, mode == COMBINE_CONCAT, eps)
        g_w = g_w if need_w else None
    elif mode == COMBINE_CONCAT and comb.size(1) == f_src:
        # the forward kept only the aggregate (inputs are data): dW of the self block = (1 + eps) g_z^T x_dst
        G, g_a, g_b, _ = mlp_bwd_w(g_y, z, prelu, comb, x_dst, y_alt=y_alt)
        g_w = self_wgrad(G, weight, f_src, True, eps)[0] if need_w else None
    else:
        g_w, g_a, g_b, _ = mlp_bwd_w(g_y, z, prelu, comb, y_alt=y_alt)
    return g_src, g_dst, g_eps, g_w, g_b, g_a


class _GINConvFn(torch.autograd.Function):
    """Fused GINConv + GINLayer MLP: y = prelu(comb @ W^T + b) [+ accum], comb = aggregate + self term."""

    @staticmethod
    def forward(ctx, x_src, x_dst, eps, weight, bias, prelu, accum, graph: RelationGraph, mode: int):
        data_inputs = not (ctx.needs_input_grad[0] or ctx.needs_input_grad[1])
        y, w_op, comb, z = _gin_forward(x_src, x_dst, eps, weight, bias, prelu, accum, graph, mode, data_inputs)
        ctx.graph, ctx.mode, ctx.f_src = graph, mode, x_src.size(1)
        ctx.save_for_backward(x_dst, eps, w_op, prelu, comb, z)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x_dst, eps, weight, prelu, comb, z = ctx.saved_tensors   # weight: the operand copy the forward used
        need_src, need_dst, need_eps, need_w, need_b, need_a, need_acc = ctx.needs_input_grad[:7]
        g_src, g_dst, g_eps, g_w, g_b, g_a = _gin_backward(g_y, x_dst, eps, weight, prelu, comb, z, ctx.graph,
                                                           ctx.mode, ctx.f_src, need_src, need_dst, need_eps, need_w)
        g_acc = g_y if need_acc else None
        return (g_src, g_dst, (g_eps.view_as(eps) if (need_eps and g_eps is not None) else None),
                g_w if need_w else None, g_b if need_b else None, (g_a.view_as(prelu) if need_a else None), g_acc,
                None, None)


@dataclass
class RelSpec:
    """One relation of a HeteroConv layer for the layer-level path: node-type indices, graph, combine mode."""
    src: int
    dst: int
    graph: RelationGraph
    mode: int


class _HeteroGINLayerFn(torch.autograd.Function):
    """A whole HeteroConv(aggr='sum') layer of GINLayers (models.py:286-298) as ONE autograd node, so the
    backward controls how the gradients of a node type consumed by several relations are summed (autograd would
    add them with separate elementwise kernels: 3.1 ms / step at cfg5, 6.2 ms at cfg3): every contribution after
    the first accumulates in place inside the kernel that produces it (the CSC aggregate's ADD self term with
    eps 0, the dX GEMM's combine epilogue).  Relations run in forward order (the second relation into a type adds
    the first's output in its epilogue, as conv.HeteroConv does); the backward visits them in reverse (autograd's
    order) and skips relations whose output gradient is None (dead relations).

    Inputs: (specs, n_types, *tensors) with tensors = node features per type, then (eps, weight, bias, prelu) per
    relation.  Outputs: one tensor per destination type, in order of first appearance."""

    @staticmethod
    def forward(ctx, specs, n_types, *tensors):
        xs = tensors[:n_types]
        need = ctx.needs_input_grad[2:]
        outs = {}
        saved = []
        for i, sp in enumerate(specs):
            eps, w, b, a = tensors[n_types + 4 * i: n_types + 4 * i + 4]
            data_inputs = not (need[sp.src] or need[sp.dst])
            # bf16: the first relation into a type has no accum, so its y determines z (gin_mlp_fwd zy)
            zy = xs[sp.src].dtype == torch.bfloat16 and sp.dst not in outs and zy_form(w.size(0), w.size(1))
            y, w_op, comb, z = _gin_forward(xs[sp.src], xs[sp.dst], eps, w, b, a, outs.get(sp.dst), sp.graph,
                                            sp.mode, data_inputs, zy=zy)
            outs[sp.dst] = y
            saved += [w_op, comb, z, y if zy else None]
        ctx.specs, ctx.n_types = specs, n_types
        ctx.out_types = list(outs)
        ctx.f_src = [xs[sp.src].size(1) for sp in specs]
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(*tensors, *saved)
        return tuple(outs[t] for t in ctx.out_types)

    @staticmethod
    def backward(ctx, *g_outs):
        specs, nt = ctx.specs, ctx.n_types
        st = ctx.saved_tensors
        xs = st[:nt]
        npar = 4 * len(specs)
        params = st[nt:nt + npar]
        saved = st[nt + npar:]
        need = ctx.needs_input_grad[2:]
        g_of = dict(zip(ctx.out_types, g_outs))
        gx = [None] * nt
        gp = [None] * npar

        def next_use_is_aggregate(i, t):
            # the first relation after i in backward order that touches type t's running gradient reads it as a CSC
            # aggregate's running gradient (t its source, ADD mode) — not as a dX epilogue's g_prev, not returned
            for j in reversed(range(i)):
                sj = specs[j]
                if g_of.get(sj.dst) is None:
                    continue
                if sj.dst == t and need[t]:
                    return False
                if sj.src == t and need[t]:
                    return sj.mode == COMBINE_ADD
            return False

        for i in reversed(range(len(specs))):
            sp = specs[i]
            g_y = g_of.get(sp.dst)
            if g_y is None:
                continue
            eps, _, _, prelu = params[4 * i: 4 * i + 4]
            w_op, comb, z, y_alt = saved[4 * i: 4 * i + 4]
            pn = need[nt + 4 * i: nt + 4 * i + 4]
            g_src, g_dst, g_eps, g_w, g_b, g_a = _gin_backward(
                g_y, xs[sp.dst], eps, w_op, prelu, comb, z, sp.graph, sp.mode, ctx.f_src[i], need[sp.src],
                need[sp.dst], pn[0], pn[1], g_src_prev=gx[sp.src], g_dst_prev=gx[sp.dst], y_alt=y_alt,
                lazy_dst=LAZY_SELF and sp.mode == COMBINE_ADD and gx[sp.dst] is None and sp.src != sp.dst
                and next_use_is_aggregate(i, sp.dst))
            if need[sp.src]:
                gx[sp.src] = g_src
            if need[sp.dst]:
                gx[sp.dst] = g_dst
            gp[4 * i] = g_eps.view_as(eps) if (pn[0] and g_eps is not None) else None
            gp[4 * i + 1] = g_w if pn[1] else None
            gp[4 * i + 2] = g_b if pn[2] else None
            gp[4 * i + 3] = g_a.view_as(prelu) if (pn[3] and g_a is not None) else None
        return (None, None, *gx, *gp)


def hetero_gin_layer(xs, specs, params):
    """Outputs (one per destination type, in order of first appearance) of a HeteroConv layer of GINLayers run as
    one autograd node (_HeteroGINLayerFn).  ``xs``: node features per type index; ``params``: (eps, weight,
    bias, prelu) per relation."""
    require_device(*xs, what="hgin.hetero_gin_layer")
    xs = [_rowmajor(_f32(x, "x")) for x in xs]
    _same_dtype("hgin.hetero_gin_layer", *xs)
    flat = []
    for sp, (eps, w, b, a) in zip(specs, params):
        f_src = xs[sp.src].size(1)
        width = f_src + (xs[sp.dst].size(1) if sp.mode == COMBINE_CONCAT else 0)
        if sp.mode == COMBINE_ADD and xs[sp.dst].size(1) != f_src:
            raise RuntimeError(f"GINConv add: feature sizes differ ({f_src} vs {xs[sp.dst].size(1)})")
        if w.size(1) != width:
            raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({sp.graph.n_dst}x{width} and "
                               f"{w.size(1)}x{w.size(0)})")
        flat += [eps, _rowmajor(w), b.contiguous(), a]
    return _HeteroGINLayerFn.apply(specs, len(xs), *xs, *flat)


_ONE = {}


def _one(device) -> Tensor:
    t = _ONE.get(device)
    if t is None:
        t = _ONE[device] = torch.ones(1, dtype=torch.float32, device=device)
    return t


class _LinearPReLUFn(torch.autograd.Function):
    """Linear [+ PReLU] of the readout (models.py:300-330, :373-374) on the MFMA kernels.  The input is the
    column concatenation [x1 | x2] (cat((x_path, raw path features)), models.py:362-371) read from its two
    sources directly; ``prelu`` None is a plain Linear (the head)."""

    @staticmethod
    def forward(ctx, x1, x2, weight, bias, prelu):
        w_op = _as(weight, x1.dtype)
        # (no accum: y determines z, gin_mlp_fwd zy)
        zy = x1.dtype == torch.bfloat16 and prelu is not None and zy_form(weight.size(0), weight.size(1))
        z, y = gin_mlp_fwd(x1, w_op, bias, prelu, None, comb2=x2, zy=zy)
        ctx.save_for_backward(x1, x2, w_op, prelu, z, y if zy else None)
        return y

    @staticmethod
    def backward(ctx, g_y):
        x1, x2, weight, prelu, z, y_alt = ctx.saved_tensors
        need_x1, need_x2, need_w, need_b, need_a = ctx.needs_input_grad
        g_y = _rowmajor(g_y)
        k1 = x1.size(1)
        if prelu is None:   # g_z = g_y; the PReLU-backward kernel with slope 1 yields the bias column sums
            g_z, _, g_b = prelu_bwd(g_y, g_y, _one(g_y.device))
            g_a = None
            g_z = g_z.to(x1.dtype)     # bf16 path: the head's output (and g_y) are fp32, its operands bf16
            g_w = gemm_tn(g_z, x1, x2) if need_w else None
            g_x1 = gemm_nt(g_z, weight[:, :k1].t().contiguous()) if need_x1 else None
            g_x2 = gemm_nt(g_z, weight[:, k1:].t().contiguous()) if (need_x2 and x2 is not None) else None
        else:
            g_w, g_a, g_b, g_z = mlp_bwd_w(g_y, z, prelu, x1, x2, want_gz=need_x1 or (need_x2 and x2 is not None),
                                           y_alt=y_alt)
            g_x1 = gemm_nt(g_z, weight[:, :k1].t().contiguous()) if need_x1 else None
            g_x2 = gemm_nt(g_z, weight[:, k1:].t().contiguous()) if (need_x2 and x2 is not None) else None
        return (g_x1, g_x2, g_w if need_w else None, (g_b if need_b else None),
                (g_a.view_as(prelu) if (need_a and g_a is not None) else None))


def linear_prelu(x1: Tensor, weight: Tensor, bias: Tensor, prelu: Optional[Tensor],
                 x2: Optional[Tensor] = None) -> Tensor:
    """prelu([x1 | x2] @ W^T + b) (prelu None: plain Linear), forward and backward on libhgin.so."""
    require_device(x1, x2, weight, bias, prelu, what="hgin.linear_prelu")
    x1 = _rowmajor(_f32(x1, "x"))
    if x2 is not None:
        x2 = _rowmajor(_f32(x2, "x2"))
        if x2.size(0) != x1.size(0):
            raise RuntimeError("linear_prelu: x1 / x2 row counts differ")
    _same_dtype("hgin.linear_prelu", x1, x2)
    width = x1.size(1) + (x2.size(1) if x2 is not None else 0)
    if weight.size(1) != width:
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({x1.size(0)}x{width} and "
                           f"{weight.size(1)}x{weight.size(0)})")
    return _LinearPReLUFn.apply(x1, x2, _rowmajor(weight), bias.contiguous(), prelu)


def aggregate(x_src: Tensor, x_dst: Optional[Tensor], eps: Optional[Tensor], graph: RelationGraph,
              mode: int) -> Tensor:
    require_device(x_src, x_dst, eps, what="hgin.aggregate")
    x_src = _rowmajor(_f32(x_src, "x_src"))
    if x_dst is not None:
        x_dst = _rowmajor(_f32(x_dst, "x_dst"))
    _same_dtype("hgin.aggregate", x_src, x_dst)
    if mode == COMBINE_ADD and x_dst.size(1) != x_src.size(1):
        raise RuntimeError(f"GINConv add: feature sizes differ ({x_src.size(1)} vs {x_dst.size(1)})")
    if mode != COMBINE_NONE and x_dst.size(0) != graph.n_dst:
        raise RuntimeError("x_dst rows != number of destination nodes")
    return _AggregateFn.apply(x_src, x_dst, eps, graph, mode)


def gin_conv(x_src: Tensor, x_dst: Tensor, eps: Tensor, weight: Tensor, bias: Tensor, prelu: Tensor,
             graph: RelationGraph, mode: int, accum: Optional[Tensor] = None) -> Tensor:
    require_device(x_src, x_dst, eps, weight, bias, prelu, accum, what="hgin.gin_conv")
    x_src = _rowmajor(_f32(x_src, "x_src"))
    x_dst = _rowmajor(_f32(x_dst, "x_dst"))
    width = x_src.size(1) + (x_dst.size(1) if mode == COMBINE_CONCAT else 0)
    if mode == COMBINE_ADD and x_dst.size(1) != x_src.size(1):
        raise RuntimeError(f"GINConv add: feature sizes differ ({x_src.size(1)} vs {x_dst.size(1)})")
    if weight.size(1) != width:
        raise RuntimeError(f"mat1 and mat2 shapes cannot be multiplied ({graph.n_dst}x{width} and "
                           f"{weight.size(1)}x{weight.size(0)})")
    _same_dtype("hgin.gin_conv", x_src, x_dst, accum)
    if accum is not None:
        accum = accum.contiguous()      # the epilogue reads accum with row stride N
    return _GINConvFn.apply(x_src, x_dst, eps, _rowmajor(weight), bias.contiguous(), prelu, accum, graph, mode)


_last_pool_status: Optional[Tensor] = None


def global_pool(x: Tensor, batch: Tensor, check: bool = False) -> Tensor:
    """[N, 2F] = [global_mean_pool | global_max_pool](x, batch) gathered back to the rows (models.py:347-352), on
    hgin_global_pool_*: deterministic, no host sync.  ``batch`` must be non-decreasing (PyG collation); the kernel
    flags a descending pair in a device status word (HGIN_STATUS_UNSORTED), read by ``check_pool_order()`` (one host
    sync) or at once with ``check=True``.  The pooled inputs are data (raw path features): no gradient flows through
    the pooling."""
    global _last_pool_status
    require_device(x, batch, what="hgin.global_pool")
    x = _rowmajor(_f32(x, "x"))
    if torch.is_grad_enabled() and x.requires_grad:
        raise NotImplementedError("hgin.global_pool: no backward (the reference pools the raw input features)")
    if batch.dtype != torch.long or batch.dim() != 1 or batch.numel() != x.size(0):
        raise ValueError("hgin.global_pool: batch must be int64 [N] with one entry per row")
    n, f = x.shape
    out = torch.empty(n, 2 * f, dtype=x.dtype, device=x.device)
    status = torch.zeros(1, dtype=torch.int32, device=x.device)
    nbytes = ctypes.c_size_t(0)
    _lib.check(_lib.lib().hgin_global_pool_workspace_size(n, f, ctypes.byref(nbytes)), "global_pool_workspace_size")
    ws = _workspace(nbytes.value, x.device)
    _lib.call(f"hgin_global_pool_{_sfx(x)}", _p(batch.contiguous()), n, _p(x), x.stride(0), f, _p(out), out.stride(0),
              _p(status), _p(ws), nbytes.value, _stream(x))
    _last_pool_status = status
    if check:
        check_pool_order()
    return out


def check_pool_order() -> None:
    """Raise if the last global_pool call saw a batch vector that is not non-decreasing (one host sync)."""
    st = _last_pool_status
    if st is not None and int(st.item()) & STATUS_UNSORTED:
        raise ValueError("hgin.global_pool: batch must be non-decreasing (PyG collation order)")


# ---------------------------------------------------------------------------------------------------
# F3: fused readout head + MAPE loss
# ---------------------------------------------------------------------------------------------------
class _HeadMapeFn(torch.autograd.Function):
    """out = h @ w^T + b (the head Linear(K, 1), models.py:326-330) and loss_value = mape(out, y)
    (train.py:12-13, :38-42) in one forward pass and one backward pass; ``out`` is returned for metrics
    and carries no gradient (train.py back-propagates through the loss only)."""

    @staticmethod
    def forward(ctx, h, weight, bias, y, m_valid):
        M, K = h.shape
        dev = h.device
        out = torch.empty(M, 1, dtype=torch.float32, device=dev)
        lv = torch.empty((), dtype=torch.float32, device=dev)
        w = weight.reshape(-1).to(torch.float32).contiguous()
        nbytes = ctypes.c_size_t(0)
        _lib.check(_lib.lib().hgin_head_mape_workspace_size(M, K, ctypes.byref(nbytes)), "head_mape_workspace")
        ws = _workspace(nbytes.value, dev)
        _lib.call(f"hgin_head_mape_fwd_{_sfx(h)}", _p(h), h.stride(0), M, K, _p(w), _p(bias), _p(y), _p(m_valid),
                  _p(out), _p(lv), _p(ws), nbytes.value, _stream(h))
        ctx.m_valid = m_valid
        ctx.save_for_backward(h, w, y, out)
        ctx.mark_non_differentiable(out)
        return out, lv

    @staticmethod
    def backward(ctx, g_out_unused, g_lv):
        h, w, y, out = ctx.saved_tensors
        need_h, need_w, need_b = ctx.needs_input_grad[:3]
        M, K = h.shape
        dev = h.device
        g_lv = g_lv.to(torch.float32).reshape(1).contiguous()
        g_h = torch.empty_like(h) if need_h else None
        g_w = torch.empty(1, K, dtype=torch.float32, device=dev)
        g_b = torch.empty(1, dtype=torch.float32, device=dev)
        nbytes = ctypes.c_size_t(0)
        _lib.check(_lib.lib().hgin_head_mape_workspace_size(M, K, ctypes.byref(nbytes)), "head_mape_workspace")
        ws = _workspace(nbytes.value, dev)
        _lib.call(f"hgin_head_mape_bwd_{_sfx(h)}", _p(h), h.stride(0), M, K, _p(w), _p(y), _p(out), _p(g_lv),
                  _p(ctx.m_valid), _p(g_h), g_h.stride(0) if g_h is not None else K, _p(g_w), _p(g_b), _p(ws),
                  nbytes.value, _stream(h))
        return g_h, (g_w if need_w else None), (g_b if need_b else None), None, None


def head_mape(h: Tensor, weight: Tensor, bias: Tensor, y: Tensor, m_valid: Optional[Tensor] = None):
    """(out [M, 1], loss_value) = (h @ W^T + b, 100 * mean(|(out - y) / y|)) on libhgin.so (F3).

    ``m_valid``: optional device int32 [1]; only rows < m_valid are labelled (padded static batches)."""
    require_device(h, weight, bias, y, what="hgin.head_mape")
    h = _rowmajor(_f32(h, "h"))
    if weight.dim() != 2 or weight.size(0) != 1 or weight.size(1) != h.size(1):
        raise RuntimeError(f"head_mape: weight must be [1, {h.size(1)}], got {list(weight.shape)}")
    y = y.reshape(-1)
    if y.numel() != h.size(0):
        raise RuntimeError(f"head_mape: {y.numel()} labels for {h.size(0)} rows")
    if y.dtype != torch.float32:
        raise TypeError(f"head_mape: labels must be float32, got {y.dtype}")
    if m_valid is not None and (m_valid.dtype != torch.int32 or m_valid.numel() != 1):
        raise TypeError("head_mape: m_valid must be a device int32 tensor with one element")
    return _HeadMapeFn.apply(h, weight, bias.reshape(1).to(torch.float32).contiguous(), y.contiguous(), m_valid)
