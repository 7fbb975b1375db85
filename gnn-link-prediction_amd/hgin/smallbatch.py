"""The reference's real training loop in a handful of launches per batch (dataset.py:26, :239-244;
train.py:25-44): ``SmallBatchStep`` runs a HetroGIN train step over a padded batch of small graphs with the fused
kernels of ``csrc/hgin_smallbatch.hip`` (per layer one aggregate + MLP launch over every relation and row of the
batch, the readout + MAPE + readout backward in tiles of 8 rows, per layer one or two backward launches, one
fixed-order gradient reduction that applies the sqrt-MAPE scale and, for Adam, the parameter update: 3 L + 1
launches), captured once into a hipGraph and replayed per batch after one device collation launch.

It takes the model train.py builds from config.json (``HetroGIN`` with GINLayer convs, Linear + shared PReLU
readout, Linear head; and for MODEL == "GAT" ``HetroGAT``'s one GATConv layer — heads a power of two <= 32,
out_channels 4 / 8 / 16, heads x out_channels <= 128 — as k_sb_gat_fwd / k_sb_gat_bwd: 1 + readout + 2 launches) and its
GLOBAL_FEATS (one pooling launch ahead of the step, models.py:347-352) and MLP_BN
(the readout as 2 nhid + 1 launches around the BatchNorm's batch statistics, models.py:303-313) and DROPOUT
(masks hashed per step, models.py:358-359) switches, at small widths: hidden <= 128, first-layer GEMM K <= 128, readout widths <= 256, <= 3 hidden readout
layers, <= 4 layers, fp32.  ``SmallBatchStep.supports(model)``
says whether it applies; ``hgin.graphs.CapturedTrainStep`` (one launch per op, any shape) is the general path.

Parameters' ``.grad`` become views of one flat gradient buffer the reduction kernel writes (replays rewrite them in
place); the step returns the batch's device ``loss_value`` (train.py:40), no host sync.
"""
from __future__ import annotations

import ctypes
from typing import Optional, Sequence

import torch

from . import _lib, ops
from .conv import GINConv, GINLayer
from .models import HetroGIN
from .store import GraphStore

MAX_L, MAX_HID, REL = 4, 3, 4
N_PARTS = 128  # row chunks of the weight-gradient partials (fixed: the reduction order does not depend on the batch)
RO_ROWS = 8    # path rows per readout tile (csrc/hgin_smallbatch.hip kSbRows; the launcher checks the tile count)
TYPES = ("path", "link", "node")
RELS = (("path", "uses", "link"), ("link", "includes", "path"), ("link", "connects", "node"), ("node", "has", "link"))
_P = ctypes.c_void_p
_I64 = ctypes.c_int64
_I32 = ctypes.c_int32


class _SbConv(ctypes.Structure):
    _fields_ = [("w", _P), ("b", _P), ("slope", _P), ("eps", _P), ("goff", _I64)]


class _SbGat(ctypes.Structure):   # csrc/hgin_smallbatch.hip SbGat
    _fields_ = [("ws", _P), ("wd", _P), ("att_s", _P), ("att_d", _P), ("b", _P), ("goff", _I64)]


class _SbArgs(ctypes.Structure):   # field for field csrc/hgin_smallbatch.hip SbArgs
    _fields_ = [("x", _P * 3), ("ldx", _I64 * 3), ("fdim", _I32 * 3), ("cols", (_I32 * 8) * 3),
                ("rowptr", _P * REL), ("col", _P * REL), ("cptr", _P * REL), ("cdst", _P * REL),
                ("goff", _P), ("G", _I32), ("y", _P), ("m_valid", _P),
                ("L", _I32), ("H", _I32), ("conv", (_SbConv * REL) * MAX_L),
                ("concat_path", _I32), ("pool_w", _I32), ("pool_ld", _I32), ("pooled", _P), ("pbatch", _P),
                ("nhid", _I32), ("rw", _I32 * MAX_HID),
                ("row_w", _P * MAX_HID), ("row_b", _P * MAX_HID), ("ro_slope", _P), ("head_w", _P), ("head_b", _P),
                ("ro_goff", _I64 * MAX_HID), ("ro_slope_goff", _I64), ("head_goff", _I64),
                ("p_gin", _I64), ("p_ro", _I64),
                ("act", _P), ("act_off", (_I64 * 3) * MAX_L),
                ("comb", _P), ("comb_off", (_I64 * REL) * MAX_L),
                ("zb", _P), ("zb_off", (_I64 * REL) * MAX_L),
                ("gA", _P), ("gB", _P), ("g_off", _I64 * 3),
                ("gc", _P), ("gc_off", _I64 * REL), ("kmax", _I32),
                ("cap", _I32 * 3), ("part_gin", _P), ("n_parts", _I32), ("part_ro", _P), ("loss_part", _P),
                ("slope_part", _P), ("n_tiles", _I32), ("ro_wlds", _I32),
                ("ro_in", _P * (MAX_HID + 1)), ("ro_gz", _P * (MAX_HID + 1)),
                ("gflat", _P), ("loss_value", _P),
                ("pflat", _P), ("mflat", _P), ("vflat", _P), ("adam_step", _P),
                ("lr", ctypes.c_float), ("beta1", ctypes.c_float), ("beta2", ctypes.c_float),
                ("adam_eps", ctypes.c_float), ("weight_decay", ctypes.c_float),
                ("bn_w", _P * MAX_HID), ("bn_b", _P * MAX_HID), ("bn_rm", _P * MAX_HID), ("bn_rv", _P * MAX_HID),
                ("bn_nbt", _P * MAX_HID), ("bn_goff", _I64 * MAX_HID), ("bn_eps", ctypes.c_float),
                ("bn_mom", ctypes.c_float), ("bn_buf", _P), ("bn_off", (_I64 * 5) * MAX_HID),
                ("drop_ctr", _P), ("drop_seed", ctypes.c_uint64), ("drop_thr", ctypes.c_uint32),
                ("drop_inv", ctypes.c_float), ("eval_only", _I32), ("out_pred", _P), ("loss_acc", _P),
                ("dead_conv", ctypes.c_uint32),
                ("gat", _I32), ("gat_heads", _I32), ("gat_c", _I32), ("gat_slope", ctypes.c_float),
                ("gatc", _SbGat * REL), ("gat_st", _P), ("gat_st_off", _I64 * REL)]


_OFFSET_FIELDS = ("goff", "m_valid", "conv", "rw", "ro_goff", "p_ro", "act_off", "zb_off", "gc_off", "n_tiles",
                  "loss_value", "adam_step", "weight_decay", "bn_off", "drop_inv", "loss_acc",
                  "dead_conv", "gatc", "gat_st_off")


def foldable(opt: torch.optim.Optimizer, params=None) -> bool:
    """Adam with one parameter group, float hyperparameters, amsgrad / maximize / decoupled weight decay off: its update
    can run inside the fused step's final kernel (csrc/hgin_smallbatch.hip adam_update, L2 weight decay through the
    gradient).  With ``params`` (the model's parameters): the group must hold exactly those, all requiring gradients —
    the folded update writes every parameter of the model."""
    if type(opt) is not torch.optim.Adam or len(opt.param_groups) != 1:
        return False
    g = opt.param_groups[0]
    if (g.get("amsgrad", False) or g.get("maximize", False) or g.get("differentiable", False)
            or g.get("decoupled_weight_decay", False) or isinstance(g["lr"], torch.Tensor)
            or any(isinstance(b, torch.Tensor) for b in g["betas"])):
        return False
    if params is not None:
        params = list(params)
        if {id(p) for p in g["params"]} != {id(p) for p in params} or len(g["params"]) != len(params):
            return False
        if not all(p.requires_grad for p in params):
            return False
    return True


def _hyper(opt: torch.optim.Optimizer) -> tuple:
    g = opt.param_groups[0]
    return (float(g["lr"]), float(g["betas"][0]), float(g["betas"][1]), float(g["eps"]), float(g["weight_decay"]))


def dead_convs(L: int) -> set:
    """(layer, relation index) of the convs whose outputs cannot reach the readout: the reference's
    autograd leaves their parameters' .grad None, so torch's Adam skips them (no step, no weight decay)."""
    dead, live_types = set(), {"path"}
    for l in range(L - 1, -1, -1):
        needed = set()
        for ri, (src, _, dst) in enumerate(RELS):
            if dst in live_types:
                needed.update((src, dst))
            else:
                dead.add((l, ri))
        live_types = needed
    return dead


def check_layout() -> None:
    """The ctypes mirror of SbArgs against the library's own sizeof / offsetof (raises on an ABI mismatch)."""
    lib = _lib.lib()
    if ctypes.sizeof(_SbArgs) != int(lib.hgin_sb_args_size()):
        raise RuntimeError(f"SbArgs: {ctypes.sizeof(_SbArgs)} != {lib.hgin_sb_args_size()} bytes")
    offs = (ctypes.c_int64 * len(_OFFSET_FIELDS))()
    _lib.check(lib.hgin_sb_args_offsets(offs, len(_OFFSET_FIELDS)), "hgin_sb_args_offsets")
    for name, o in zip(_OFFSET_FIELDS, offs):
        if getattr(_SbArgs, name).offset != o:
            raise RuntimeError(f"SbArgs.{name}: offset {getattr(_SbArgs, name).offset} != {o}")


def _column_map(model: HetroGIN, raw: dict) -> dict:
    """The raw feature columns models.py:333-342 keeps per type, as index lists (the model's own slicing applied to
    column-index rows)."""
    probe = {t: torch.arange(raw[t], dtype=torch.float32).reshape(1, -1) for t in TYPES}
    model._select_features(probe)
    return {t: [int(v) for v in probe[t].reshape(-1).tolist()] for t in TYPES}


GAT_C = (4, 8, 16)   # GATConv out_channels the fused kernels are instantiated for (csrc/hgin_smallbatch.hip)


def _gat_convs(model):
    """HetroGAT (models.py:380-506): the one layer's GATConv per relation, or a reason string."""
    from .gat import GATConv
    if model.num_layers != 1:
        return "HetroGAT layers (the fused step runs the reference's one-layer HetroGAT)"
    hc = model.convs[0]
    if hc.skip or hc.aggr != "sum" or len(hc.convs) != REL:
        return "pruned relations / aggr / relation set"
    row = []
    for r in RELS:
        key = "__".join(r)
        conv = hc.convs[key] if key in hc.convs else None
        if not isinstance(conv, GATConv):
            return f"relation {key}"
        nh, c = conv.heads, conv.out_channels
        if (not conv.concat or not conv.add_self_loops or conv.dropout != 0.0 or conv.bias is None
                or conv.lin_src is conv.lin_dst or nh & (nh - 1) or nh > 32 or c not in GAT_C or nh * c > 128):
            return f"GATConv {key} (concat, self loops, no attention dropout, bias, heads a power of two <= 32, " \
                   f"out_channels in {GAT_C}, heads x out_channels <= 128)"
        row.append(conv)
    if len({(c.heads, c.out_channels, c.negative_slope) for c in row}) != 1:
        return "GATConv heads / widths / slopes differ between relations"
    return [row]


def _structure(model: torch.nn.Module):
    """(convs, hidden readout Linears, the shared slope, head Linear, H, BatchNorms) or a reason string when the fused
    step does not take the model.  HetroGIN: convs[l][r] = (Linear, PReLU weight, eps); HetroGAT: convs[0][r] = the
    GATConv, H = heads x out_channels."""
    from .models import HetroGAT
    gat = type(model) is HetroGAT
    if type(model) is not HetroGIN and not gat:
        return "not a HetroGIN / HetroGAT"
    if not 0.0 <= model.dropout < 1.0:
        return "dropout probability"
    if not 1 <= model.num_layers <= MAX_L:
        return "layers"
    if gat:
        convs = _gat_convs(model)
        if isinstance(convs, str):
            return convs
        return _readout_structure(model, convs, convs[0][0].heads * convs[0][0].out_channels)
    convs = []
    for l, hc in enumerate(model.convs):
        if hc.skip or hc.aggr != "sum":
            return "pruned relations / aggr"
        row = []
        for r in RELS:
            key = "__".join(r)
            if key not in hc.convs or not isinstance(hc.convs[key], GINLayer):
                return f"relation {key}"
            conv: GINConv = hc.convs[key].conv
            nn = conv.nn
            if not (isinstance(nn, torch.nn.Sequential) and len(nn) == 2 and isinstance(nn[0], torch.nn.Linear)
                    and nn[0].bias is not None and isinstance(nn[1], torch.nn.PReLU) and nn[1].weight.numel() == 1):
                return "GIN MLP"
            if conv.concat != (l == 0) or not isinstance(conv.eps, torch.nn.Parameter):
                return "combine mode / eps"
            row.append((nn[0], nn[1].weight, conv.eps))
        if len(hc.convs) != REL:
            return "relation set"
        convs.append(row)
    return _readout_structure(model, convs, model.convs[0].convs["path__uses__link"].conv.nn[0].out_features)


def _readout_structure(model, convs, H):
    ro = list(model.readout)
    hidden, slope, bns = [], None, []
    for seq in ro[:-1]:
        seq = list(seq)
        bn = None
        if len(seq) == 3 and type(seq[1]) is torch.nn.BatchNorm1d:   # MLP_BN (models.py:303-313)
            bn = seq.pop(1)
            if not (bn.affine and bn.track_running_stats and bn.momentum is not None):
                return "readout BatchNorm (needs affine, running statistics, a momentum)"
        if not (len(seq) == 2 and isinstance(seq[0], torch.nn.Linear) and isinstance(seq[1], torch.nn.PReLU)
                and seq[1].weight.numel() == 1):
            return "readout layer"
        if slope is not None and seq[1].weight is not slope:
            return "readout activation not shared"
        slope = seq[1].weight
        hidden.append(seq[0])
        bns.append(bn)
    if any(b is None for b in bns):
        if any(b is not None for b in bns):
            return "readout BatchNorm on some layers only"
        bns = None
    elif len({(b.eps, b.momentum) for b in bns}) != 1:
        return "readout BatchNorm eps / momentum differ between layers"
    head = ro[-1]
    if not (len(head) == 1 and isinstance(head[0], torch.nn.Linear) and head[0].out_features == 1
            and head[0].bias is not None):
        return "head"
    if not 1 <= len(hidden) <= MAX_HID:
        return "readout depth"
    if H > 128 or any(l.out_features > 256 for l in hidden):
        return "widths"
    if any(p.dtype != torch.float32 for p in model.parameters()
           if not isinstance(p, torch.nn.parameter.UninitializedParameter)):
        return "dtype"
    return convs, hidden, slope, head[0], H, bns


def _materialize(model: torch.nn.Module, store: GraphStore, ids: Sequence[int]) -> None:
    """HetroGAT's lazy (-1, -1) projections (PyG 2.0.2 Linear, models.py:413-418) take their shapes and glorot values
    at the first forward, in forward order (the reference's RNG order): one general-path forward on a warm-up batch, in
    eval mode (no dropout draw, no BatchNorm update), materialises them before the fused step lays out its buffers."""
    b = store.collate(list(ids))
    was = model.training
    model.eval()
    try:
        with torch.no_grad():
            model(b.x_dict(), b.edge_index_dict(), b.batch["path"])
    finally:
        model.train(was)


class SmallBatchStep:
    """Fused HetroGIN / HetroGAT train step over padded small-graph batches (see the module docstring)."""

    @staticmethod
    def supports(model: torch.nn.Module) -> bool:
        return not isinstance(_structure(model), str)

    def __init__(self, model: HetroGIN, opt: torch.optim.Optimizer, store: GraphStore, batch_size: int,
                 warmup_ids: Sequence[Sequence[int]], warmup: int = 2, fold_optimizer: bool = True,
                 readout: str = "auto", _eval: bool = False, n_parts: Optional[int] = None):
        if readout not in ("auto", "scalar"):
            raise ValueError("SmallBatchStep: readout is 'auto' (32-row MFMA tiles where they fit) or 'scalar'")
        if warmup_ids and any(isinstance(p, torch.nn.parameter.UninitializedParameter) for p in model.parameters()):
            _materialize(model, store, warmup_ids[0])
        st = _structure(model)
        if isinstance(st, str):
            raise ValueError(f"SmallBatchStep: model not supported ({st}); use hgin.graphs.CapturedTrainStep")
        self._eval = bool(_eval)
        self.folded = not self._eval and bool(fold_optimizer) and foldable(opt, model.parameters())
        if not self._eval and not self.folded and not all(g.get("capturable", False) for g in opt.param_groups):
            raise ValueError("SmallBatchStep needs Adam (folded into the step) or a capturable optimizer")
        if not warmup_ids:
            raise ValueError("SmallBatchStep needs at least one warm-up batch")
        convs, hidden, slope, head, H, bns = st
        self.model, self.opt, self.store = model, opt, store
        dev = store.device
        pb = store.padded_batch(batch_size)
        self.batch = pb
        if any(store.x[t].dtype != torch.float32 for t in TYPES):
            raise ValueError("SmallBatchStep: fp32 features only")
        raw = {t: int(store.x[t].shape[1]) for t in TYPES}
        cols = _column_map(model, raw)
        fdim = {t: len(cols[t]) for t in TYPES}
        if any(f > 8 for f in fdim.values()):
            raise ValueError("SmallBatchStep: at most 8 input feature columns per type")
        L = model.num_layers
        K0 = [fdim[s] + fdim[d] for (s, _, d) in RELS]
        if max(K0) > 128:
            raise ValueError("SmallBatchStep: first-layer K > 128")
        cap = {t: int(pb.x[t].shape[0]) for t in TYPES}
        a = _SbArgs()
        keep = []   # tensors whose pointers the args hold

        def P(t: torch.Tensor):
            keep.append(t)
            return t.data_ptr()

        for ti, t in enumerate(TYPES):
            a.x[ti] = P(pb.x[t])
            a.ldx[ti] = pb.x[t].stride(0)
            a.fdim[ti] = fdim[t]
            for k, c in enumerate(cols[t]):
                a.cols[ti][k] = c
        for ri, r in enumerate(RELS):
            a.rowptr[ri], a.col[ri] = P(pb.csr[r].rowptr), P(pb.csr[r].col)
            a.cptr[ri], a.cdst[ri] = P(pb.csc[r].rowptr), P(pb.csc[r].col)
        a.goff, a.G, a.y, a.m_valid = P(pb.goff), batch_size, P(pb.y), P(pb.m_valid)
        a.L, a.H = L, H
        self.gat = not isinstance(convs[0][0], tuple)
        self._ptr_refs = []   # (setter, tensor): the argument block's parameter pointers (re-pointed after folding)

        def PP(setter, t: torch.Tensor):
            self._ptr_refs.append((setter, t))
            setter(P(t))

        def field(obj, name):
            return lambda v: setattr(obj, name, v)

        def elem(arr, i):
            def put(v):
                arr[i] = v
            return put
        # flat gradient layout: the convs (GIN: W, b, slope, eps per layer / relation; GAT: att_src, att_dst, bias,
        # lin_src.weight, lin_dst.weight per relation), then the readout
        off = 0
        param_off = {}
        conv_params = {}   # (layer, relation) -> its parameters
        if self.gat:
            g0 = convs[0][0]
            a.gat, a.gat_heads, a.gat_c, a.gat_slope = 1, g0.heads, g0.out_channels, float(g0.negative_slope)
            for ri, r in enumerate(RELS):
                conv = convs[0][ri]
                ks, kd = fdim[r[0]], fdim[r[2]]
                if tuple(conv.lin_src.weight.shape) != (H, ks) or tuple(conv.lin_dst.weight.shape) != (H, kd):
                    raise ValueError(f"SmallBatchStep: {r} projections {tuple(conv.lin_src.weight.shape)}, "
                                     f"{tuple(conv.lin_dst.weight.shape)} != {(H, ks)}, {(H, kd)}")
                gc = a.gatc[ri]
                gc.goff = a.conv[0][ri].goff = off
                prm = (conv.att_src, conv.att_dst, conv.bias, conv.lin_src.weight, conv.lin_dst.weight)
                for name, t in zip(("att_s", "att_d", "b", "ws", "wd"), prm):
                    PP(field(gc, name), t)
                for t in prm:
                    param_off[t] = off
                    off += t.numel()
                conv_params[(0, ri)] = prm
        else:
            for l in range(L):
                for ri, r in enumerate(RELS):
                    lin, pw, eps = convs[l][ri]
                    K = K0[ri] if l == 0 else H
                    if tuple(lin.weight.shape) != (H, K):
                        raise ValueError(f"SmallBatchStep: layer {l} {r} weight {tuple(lin.weight.shape)} != {(H, K)}")
                    c = a.conv[l][ri]
                    c.goff = off
                    for name, t in zip(("w", "b", "slope", "eps"), (lin.weight, lin.bias, pw, eps)):
                        PP(field(c, name), t)
                    param_off[lin.weight] = off
                    param_off[lin.bias] = off + H * K
                    param_off[pw] = off + H * K + H
                    param_off[eps] = off + H * K + H + 1
                    off += H * K + H + 2
                    conv_params[(l, ri)] = (lin.weight, lin.bias, pw, eps)
        p_gin = off
        a.concat_path = int(bool(model.concat_path))
        a.nhid = len(hidden)
        if model.global_feats:   # models.py:347-352: [mean | max] of the raw path rows per graph, pooled per step
            if 2 * fdim["path"] != model.global_feats_size:
                raise ValueError("SmallBatchStep: GLOBAL_FEATS needs 4 path feature columns")
            a.pool_w = a.pool_ld = 2 * fdim["path"]
        w0 = H + (fdim["path"] if model.concat_path else 0) + a.pool_w
        win = w0
        for i, lin in enumerate(hidden):
            if tuple(lin.weight.shape) != (lin.out_features, win):
                raise ValueError("SmallBatchStep: readout widths")
            a.rw[i] = lin.out_features
            PP(elem(a.row_w, i), lin.weight)
            PP(elem(a.row_b, i), lin.bias)
            a.ro_goff[i] = off
            param_off[lin.weight] = off
            param_off[lin.bias] = off + lin.weight.numel()
            off += lin.weight.numel() + lin.out_features
            if bns:   # its BatchNorm's gamma, then beta
                bn = bns[i]
                PP(elem(a.bn_w, i), bn.weight)
                PP(elem(a.bn_b, i), bn.bias)
                a.bn_rm[i], a.bn_rv[i] = P(bn.running_mean), P(bn.running_var)
                a.bn_nbt[i] = P(bn.num_batches_tracked)
                a.bn_goff[i] = off
                param_off[bn.weight], param_off[bn.bias] = off, off + lin.out_features
                off += 2 * lin.out_features
            win = lin.out_features
        PP(field(a, "ro_slope"), slope)
        a.ro_slope_goff = off
        param_off[slope] = off
        off += 1
        PP(field(a, "head_w"), head.weight)
        PP(field(a, "head_b"), head.bias)
        a.head_goff = off
        param_off[head.weight] = off
        param_off[head.bias] = off + head.weight.numel()
        off += head.weight.numel() + 1
        a.p_gin, a.p_ro = p_gin, off - p_gin
        params = list(model.parameters())
        if {id(p) for p in params} != {id(p) for p in param_off}:
            raise ValueError("SmallBatchStep: the model has parameters outside the fused step")
        dead = dead_convs(L)
        self.dead_params = set()   # ids of the parameters that get no gradient (.grad stays None, as in the reference)
        for (l, ri) in dead:
            a.dead_conv |= 1 << (4 * l + ri)
            self.dead_params.update(id(t) for t in conv_params[(l, ri)])
        # scratch
        f32 = dict(dtype=torch.float32, device=dev)

        def blocks(sizes):
            offs, tot = [], 0
            for n in sizes:
                offs.append(tot)
                tot += n
            return offs, torch.zeros(max(tot, 1), **f32)

        act_sizes = [cap[t] * H for _ in range(L) for t in TYPES]
        o, self.act = blocks(act_sizes)
        a.act = P(self.act)
        for l in range(L):
            for ti in range(3):
                a.act_off[l][ti] = o[l * 3 + ti]
        kdim = lambda l, ri: K0[ri] if l == 0 else H   # noqa: E731
        o, self.comb = blocks([cap[RELS[ri][2]] * kdim(l, ri) for l in range(L) for ri in range(REL)])
        a.comb = P(self.comb)
        o2, self.zb = blocks([cap[RELS[ri][2]] * H for l in range(L) for ri in range(REL)])
        a.zb = P(self.zb)
        for l in range(L):
            for ri in range(REL):
                a.comb_off[l][ri] = o[l * REL + ri]
                a.zb_off[l][ri] = o2[l * REL + ri]
        o, self.gA = blocks([cap[t] * H for t in TYPES])
        _, self.gB = blocks([cap[t] * H for t in TYPES])
        a.gA, a.gB = P(self.gA), P(self.gB)
        for ti in range(3):
            a.g_off[ti] = o[ti]
        kmax = max(max(K0), H)
        o2, self.gc = blocks([cap[r[2]] * kmax for r in RELS])
        a.gc, a.kmax = P(self.gc), kmax
        for ri in range(REL):
            a.gc_off[ri] = o2[ri]
        if self.gat:   # per relation [cap_dst][heads][2 + K_src]: the forward's softmax state for the backward
            o2, self.gat_st = blocks([cap[r[2]] * a.gat_heads * (2 + fdim[r[0]]) for r in RELS])
            a.gat_st = P(self.gat_st)
            for ri in range(REL):
                a.gat_st_off[ri] = o2[ri]
        for ti, t in enumerate(TYPES):
            a.cap[ti] = cap[t]
        # row chunks of the weight-gradient partials: fixed per model, so the reduction order does not depend on the
        # batch (n_parts: an override for A/B measurements)
        self.n_parts = n_parts if n_parts is not None else N_PARTS
        if not 1 <= self.n_parts <= 1024:
            raise ValueError("SmallBatchStep: n_parts in [1, 1024]")
        a.n_parts = self.n_parts
        self.part_gin = torch.zeros(self.n_parts * p_gin, **f32)
        a.part_gin = P(self.part_gin)
        self.gflat = torch.zeros(off, **f32)
        self.loss_value = torch.zeros((), **f32)
        a.gflat, a.loss_value = P(self.gflat), P(self.loss_value)
        if not self._eval:
            for p in params:
                o = param_off[p]
                p.grad = None if id(p) in self.dead_params else self.gflat[o:o + p.numel()].view_as(p)
        if self.folded:
            self._fold_adam(a, params, param_off, off, convs, hidden, slope, head, L, keep, bns)
        widths = (ctypes.c_int32 * MAX_HID)(*[a.rw[i] for i in range(MAX_HID)])
        lds = ctypes.c_size_t(0)
        # the readout: 32-row tiles on the matrix cores, their weights in LDS where they fit, else read through the
        # caches (mode 4); the 8-row scalar tiles (with the hidden weights in LDS, 1, else without, 0) where neither fits
        # the LDS, or asked for (readout="scalar")
        # (MLP_BN: the k_sb_bn_* launches, mode 3)
        # (MLP_BN in evaluation: the plain readout with BatchNorm's running-statistics affine map, bn_eval)
        modes = (3,) if bns and not self._eval else ((2, 4, 1, 0) if readout == "auto" else (1, 0))
        for wl in modes:
            _lib.check(_lib.lib().hgin_sb_readout_lds_bytes(H, w0 - H, int(w0 > H), a.nhid, widths, wl,
                                                            ctypes.byref(lds)), "hgin_sb_readout_lds_bytes")
            if lds.value <= 159 * 1024:
                break
        else:
            raise ValueError("SmallBatchStep: readout tile exceeds LDS")
        a.ro_wlds = wl
        n_tiles = (cap["path"] + RO_ROWS - 1) // RO_ROWS
        a.n_tiles = n_tiles
        self.part_ro = torch.zeros(self.n_parts * a.p_ro, **f32)
        self.loss_part = torch.zeros(n_tiles, **f32)
        self.slope_part = torch.zeros(n_tiles, **f32)
        a.part_ro, a.loss_part, a.slope_part = P(self.part_ro), P(self.loss_part), P(self.slope_part)
        # per readout layer (the head last): input rows and pre-activation gradient rows
        ro_w = [w0] + [a.rw[i] for i in range(a.nhid)]
        self.ro_in = [torch.zeros(cap["path"] * ro_w[i], **f32) for i in range(a.nhid + 1)]
        self.ro_gz = [torch.zeros(cap["path"] * (ro_w[i + 1] if i < a.nhid else 1), **f32)
                      for i in range(a.nhid + 1)]
        for i in range(a.nhid + 1):
            a.ro_in[i], a.ro_gz[i] = P(self.ro_in[i]), P(self.ro_gz[i])
        if bns and self._eval:
            a.bn_eps = float(bns[0].eps)
        elif bns:   # per hidden layer: z, g_y [cap_path][N], forward / backward tile partials [tiles][2][N], statistics
            nt32 = (cap["path"] + 31) // 32
            sizes = []
            for i in range(a.nhid):
                N = a.rw[i]
                sizes += [cap["path"] * N, cap["path"] * N, nt32 * 2 * N, nt32 * 2 * N, 2 * N]
            o, self.bn_buf = blocks(sizes)
            a.bn_buf = P(self.bn_buf)
            for i in range(a.nhid):
                for k in range(5):
                    a.bn_off[i][k] = o[5 * i + k]
            a.bn_eps, a.bn_mom = float(bns[0].eps), float(bns[0].momentum)
        if self._eval:   # forward + loss only, the running sums on the device
            a.eval_only = 1
            self.out_pred = torch.zeros(cap["path"], **f32)
            self.loss_acc = torch.zeros(2, **f32)
            a.out_pred, a.loss_acc = P(self.out_pred), P(self.loss_acc)
        elif model.dropout > 0.0:   # models.py:358-359: masks hashed from a seed drawn here and a device step counter
            self.drop_ctr = torch.zeros(1, dtype=torch.int64, device=dev)
            a.drop_ctr = P(self.drop_ctr)
            a.drop_seed = int(torch.randint(0, 2 ** 62, (1,)).item())
            a.drop_thr = min(int(round(float(model.dropout) * 2 ** 32)), 2 ** 32 - 1)
            a.drop_inv = 1.0 / (1.0 - float(model.dropout))
        if a.pool_w:   # per graph [mean | max], formed by the first layer's launch
            self.pooled = torch.zeros(batch_size, a.pool_ld, **f32)
            a.pooled, a.pbatch = P(self.pooled), P(pb.batch["path"])
        check_layout()
        self.args, self._keep, self.lds = a, keep, lds.value
        # warm-up on a side stream (optimizer state, allocator pools), then capture the step (+ torch's optimizer
        # when it is not folded) once
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(max(1, warmup)):
                store.collate_into(warmup_ids[i % len(warmup_ids)], pb)
                self._launch()
                if not self.folded and not self._eval:
                    opt.step()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph):
            self._launch()
            if not self.folded and not self._eval:
                opt.step()
        self._ptrs = [p.data_ptr() for p in params]
        self._first, self._last = params[0], params[-1]
        if self._eval:
            self.loss_acc.zero_()

    def _fold_adam(self, a, params, param_off, total, convs, hidden, slope, head, L, keep, bns) -> None:
        """The parameters become views of one flat buffer in the gradient layout, Adam's moments two more and its
        step count one device scalar; the optimizer's state entries are re-pointed at them (its existing state, if
        any, copied in), so opt.state_dict() stays meaningful.  The step then owns the optimizer: calling
        opt.step() as well would update twice.  The parameters of dead convs (no gradient in the reference) keep no
        state, as in torch's Adam, which never steps them."""
        f32 = dict(dtype=torch.float32, device=self.gflat.device)
        self.pflat = torch.empty(total, **f32)
        self.mflat = torch.zeros(total, **f32)
        self.vflat = torch.zeros(total, **f32)
        self.adam_step = torch.zeros((), **f32)
        steps = set()
        with torch.no_grad():
            for p in params:
                o, n = param_off[p], p.numel()
                self.pflat[o:o + n].copy_(p.detach().reshape(-1))
                state = self.opt.state.get(p)
                if state and id(p) not in self.dead_params:
                    self.mflat[o:o + n].copy_(state["exp_avg"].reshape(-1))
                    self.vflat[o:o + n].copy_(state["exp_avg_sq"].reshape(-1))
                    steps.add(float(state["step"]))
        if len(steps) > 1:
            raise ValueError("SmallBatchStep: the optimizer's parameters are at different step counts")
        self.adam_step.fill_(steps.pop() if steps else 0.0)
        for p in params:
            o, n = param_off[p], p.numel()
            p.data = self.pflat[o:o + n].view_as(p)
            if id(p) in self.dead_params:
                self.opt.state.pop(p, None)
                continue
            self.opt.state[p] = {"step": self.adam_step, "exp_avg": self.mflat[o:o + n].view_as(p),
                                 "exp_avg_sq": self.vflat[o:o + n].view_as(p)}
        # the kernels' parameter pointers: the views' (the struct was filled from the old storage)
        for setter, t in self._ptr_refs:
            setter(t.data_ptr())
        keep += [self.pflat, self.mflat, self.vflat, self.adam_step]
        a.pflat, a.mflat, a.vflat = self.pflat.data_ptr(), self.mflat.data_ptr(), self.vflat.data_ptr()
        a.adam_step = self.adam_step.data_ptr()
        self._set_hyper(a)
        self._params, self._param_off = params, param_off
        self._live = [p for p in params if id(p) not in self.dead_params]
        self._state_first = self.opt.state[self._live[0]]["exp_avg"]

    def _set_hyper(self, a) -> None:
        self._hyp = _hyper(self.opt)
        a.lr, a.beta1, a.beta2, a.adam_eps, a.weight_decay = self._hyp

    def _sync_optimizer(self) -> None:
        """The folded Adam's hyperparameters and state live in the captured launch and the flat buffers: follow the
        optimizer when it has changed since — a new lr / betas / eps / weight_decay in its param group (an LR scheduler,
        a manual edit) re-captures the step with them; a replaced state (opt.load_state_dict) is copied into the flat
        moments and step count and re-pointed at them.  A changed parameter set raises."""
        g = self.opt.param_groups
        if len(g) != 1 or len(g[0]["params"]) != len(self._params) or any(
                p is not q for p, q in zip(g[0]["params"], self._params)):
            raise RuntimeError("SmallBatchStep: the folded optimizer's parameter groups changed; build a new step")
        st = self.opt.state.get(self._live[0])
        if st is None or st.get("exp_avg") is not self._state_first:
            steps = set()
            with torch.no_grad():
                for p in self._live:
                    o, n = self._param_off[p], p.numel()
                    s = self.opt.state.get(p)
                    if not s:
                        raise RuntimeError("SmallBatchStep: the optimizer's new state misses a parameter")
                    self.mflat[o:o + n].copy_(s["exp_avg"].reshape(-1))
                    self.vflat[o:o + n].copy_(s["exp_avg_sq"].reshape(-1))
                    steps.add(float(s["step"]))
            if len(steps) != 1:
                raise RuntimeError("SmallBatchStep: the optimizer's new state has parameters at different steps")
            self.adam_step.fill_(steps.pop())
            for p in self._params:
                if id(p) in self.dead_params:
                    self.opt.state.pop(p, None)
                    continue
                o, n = self._param_off[p], p.numel()
                self.opt.state[p] = {"step": self.adam_step, "exp_avg": self.mflat[o:o + n].view_as(p),
                                     "exp_avg_sq": self.vflat[o:o + n].view_as(p)}
            self._state_first = self.opt.state[self._live[0]]["exp_avg"]
        if _hyper(self.opt) != self._hyp:
            self._set_hyper(self.args)
            torch.cuda.synchronize()
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph):
                self._launch()

    def _launch(self) -> None:
        _lib.call("hgin_sb_step", ctypes.addressof(self.args), ctypes.sizeof(self.args), self.lds,
                  ops._stream(self.gflat))

    def step(self, ids: Sequence[int]) -> torch.Tensor:
        """One training step on the graphs ``ids``; returns the device loss_value (no host sync)."""
        if self.folded:
            self._sync_optimizer()
        self.store.collate_into(ids, self.batch)
        self.graph.replay()
        return self.loss_value


class SmallBatchEval(SmallBatchStep):
    """train.py's evaluation loops — ``test()`` (train.py:70-113, after ``model.eval()``) and ``evaluate()``
    (:322-348) — on the fused small-batch kernels: per batch one device collation + one hipGraph replay of the L
    forward launches, the readout up to its MAPE numerator (the head's outputs kept in ``out_pred``) and a one-block
    loss launch that also adds the batch's loss_value and its path-weighted form into device accumulators (the
    reference's ``running_loss += loss_value.item()`` and ``running_loss_mape += mape * n_paths``): a whole pass syncs
    the host once, in ``result()``.  Same interface as ``hgin.graphs.CapturedEvalStep``; the model must be in eval
    mode (dropout off; MLP_BN's BatchNorm reads its running statistics: an affine map in the readout's epilogue).

    The replay reads the parameters in place: if they have been re-allocated since (a SmallBatchStep constructed
    afterwards folds them into its flat buffer), ``step`` re-captures first."""

    def __init__(self, model: HetroGIN, store: GraphStore, batch_size: int, warmup_ids: Sequence[Sequence[int]],
                 warmup: int = 2):
        if model.training:
            raise ValueError("SmallBatchEval: call model.eval() first (train.py:192, :329)")
        self._ctor = (store, batch_size, list(warmup_ids), warmup)
        super().__init__(model, None, store, batch_size, warmup_ids, warmup, _eval=True)
        self.batches = 0

    @staticmethod
    def supports(model: torch.nn.Module) -> bool:
        return not isinstance(_structure(model), str)

    def step(self, ids: Sequence[int]) -> torch.Tensor:
        """Evaluate the graphs ``ids``; returns the batch's device loss_value (overwritten by the next step).  The
        predictions are ``self.out_pred[:n_paths]`` until then."""
        # (a re-allocation — a folding SmallBatchStep, model.to() — moves every parameter: the first and the last
        # are checked, cheaply, per batch)
        if self._first.data_ptr() != self._ptrs[0] or self._last.data_ptr() != self._ptrs[-1]:
            acc, n = self.loss_acc.clone(), self.batches
            store, bs, wids, w = self._ctor
            SmallBatchStep.__init__(self, self.model, None, store, bs, wids, w, _eval=True)
            self.loss_acc.copy_(acc)
            self.batches = n
        self.store.collate_into(ids, self.batch)
        self.graph.replay()
        self.batches += 1
        return self.loss_value

    def reset(self) -> None:
        self.loss_acc.zero_()
        self.batches = 0

    def result(self, n_paths: int) -> tuple:
        """(average loss over the batches, path-weighted MAPE) = test()'s (average_loss, mape_loss) for a loss_func
        of MAPE; ``n_paths`` = the paths evaluated.  One host sync."""
        s, w = (float(v) for v in self.loss_acc.cpu())
        return s / max(self.batches, 1), w / max(n_paths, 1)
