"""QTBaseline on libhgin.so — drop-in for ``models.py:42-158``.

Same constructor keywords and the same ``forward(data) -> (delay[n_paths], feats[n_links, 3])`` contract
(``data`` carries ``edge_index``, ``edge_type``, ``type``, ``P``, ``L`` as produced by
``generateFiles.py:183-231`` / ``dataset.py:66-85``).  The reference forces the CPU
(``models.py:72-73, :89, :153``) and runs a Python loop of gathers / scatters per path position; here the
sample is prepared once on the device (path<->link edge runs, a stable CSR by destination ordered by
(position, edge) built with ``hgin_csr_build``) and every iteration is three kernel launches
(``csrc/hgin_qt.hip``).  Outputs are returned on the input's device, like the reference's CPU tensors
when the input is on the CPU.  Sums run in the reference's order (bit-identical traffic sums); the
``rho**B`` powers use the device ``powf`` (tolerance, see tests/test_gpu_qt.py).
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Tuple

import torch

from . import _lib, ops
from .ops import _p, _stream


@dataclass
class QtPlan:
    """Per-sample preparation: edge runs and the (position, edge)-ordered CSR by destination."""
    n: int
    src: torch.Tensor        # int32 [E0] path<->link edge sources (original order)
    dst: torch.Tensor        # int32 [E0]
    pos: torch.Tensor        # int32 [E0] position inside the source run
    run_ptr: torch.Tensor    # int32 [n_runs + 1]
    run_src: torch.Tensor    # int32 [n_runs]
    csr: ops.Csr             # rows = destination vertex, col = edge id, ordered by (pos, edge id)
    link_ids: torch.Tensor   # int32 [n_links]
    path_mask: torch.Tensor  # bool [n]


def plan(edge_index: torch.Tensor, edge_type: torch.Tensor, vtype: torch.Tensor, device) -> QtPlan:
    ei = edge_index.to(device).long()
    et = edge_type.to(device)
    vt = vtype.to(device)
    n = int(vt.numel())
    sel = et == 0
    src, dst = ei[0, sel], ei[1, sel]
    e0 = int(src.numel())
    start = torch.ones(e0, dtype=torch.bool, device=device)
    if e0 > 1:
        start[1:] = src[1:] != src[:-1]
    first = torch.nonzero(start).view(-1)                      # models.py:17-29: runs of equal sources
    run = torch.cumsum(start.to(torch.int32), 0) - 1
    pos = torch.arange(e0, device=device) - first[run.long()] if e0 else torch.zeros(0, dtype=torch.long,
                                                                                     device=device)
    n_pos = int(pos.max()) + 1 if e0 else 0
    eid = torch.arange(e0, device=device)
    by_pos = ops.build_csr(torch.stack([eid, pos]), 1, n_pos, max(e0, 1))            # stable: (pos, edge id)
    order = by_pos.perm.long()
    csr = ops.build_csr(torch.stack([order, dst[order]]), 1, n, max(e0, 1))          # by dst, order kept
    run_ptr = torch.cat([first, torch.tensor([e0], device=device)]).to(torch.int32)
    link_ids = torch.nonzero(vt == 1).view(-1).to(torch.int32)
    return QtPlan(n, src.to(torch.int32), dst.to(torch.int32), pos.to(torch.int32), run_ptr,
                  src[first].to(torch.int32), csr, link_ids, vt == 0)


class QTBaseline(torch.nn.Module):
    """models.py:42-158 (no parameters)."""

    def __init__(self, num_iterations=3, G_dim=4, P_dim=3, L_dim=1, device=None, **kwargs):
        super().__init__(**kwargs)
        self.num_iterations = num_iterations
        self.G_dim, self.P_dim, self.L_dim = G_dim, P_dim, L_dim
        self.H = self.H_p = self.H_l = self.H_n = 2
        self.buffer = 32
        self.device = torch.device(device) if device is not None else torch.device("cuda")

    def forward(self, data) -> Tuple[torch.Tensor, torch.Tensor]:
        dev = self.device
        if dev.type != "cuda":
            raise RuntimeError("hgin QTBaseline runs on the HIP device (no CPU fallback)")
        out_dev = data.type.device
        pl = plan(data.edge_index, data.edge_type, data.type, dev)
        n, n_runs, n_links = pl.n, int(pl.run_src.numel()), int(pl.link_ids.numel())
        P = data.P.to(dev, torch.float32)
        Lraw = data.L.to(dev, torch.float32).reshape(-1)
        a = torch.zeros(n, device=dev)
        a[pl.path_mask] = P[:, self.P_dim - 2]                  # X[:, path_og.stop - 2] (models.py:92)
        cap = (Lraw / 1000).contiguous()                        # X[is_l, link_og.start] (models.py:77, :88)
        bp = torch.full((n,), 0.5, device=dev)
        val = torch.empty(max(int(pl.src.numel()), 1), device=dev)
        t_sum = torch.empty(n, device=dev)
        rho = torch.empty(n_links, device=dev)
        pi0 = torch.empty(n_links, device=dev)
        occ = torch.empty(n_links, device=dev)
        x = torch.zeros(n, device=dev)
        s = _stream(a)
        for _ in range(self.num_iterations):
            _lib.call("hgin_qt_traffic", _p(pl.run_ptr), n_runs, _p(pl.run_src), _p(pl.dst), _p(a), _p(bp), _p(val),
                      s)
            _lib.call("hgin_qt_link_sum", _p(pl.csr.rowptr), _p(pl.csr.col), _p(pl.pos), _p(val), n, _p(t_sum), s)
            bp.zero_()
            _lib.call("hgin_qt_links", _p(pl.link_ids), n_links, _p(t_sum), _p(cap), _p(Lraw), self.buffer, _p(bp),
                      _p(rho), _p(pi0), _p(occ), _p(x), s)
        out = torch.zeros(n, device=dev)
        _lib.call("hgin_qt_delay", _p(pl.run_ptr), n_runs, _p(pl.run_src), _p(pl.dst), _p(x), _p(out), s)
        delay = out[pl.path_mask]
        feats = torch.stack([occ, rho, pi0], 1)
        return delay.to(out_dev), feats.to(out_dev)
