"""CPU restatement of the reference's queueing-theory baseline (``models.py:15-158``) — TEST INFRASTRUCTURE.

Only tests/, ``__graft_entry__.smoke()`` and bench.py's cpu_baseline may import this module; the product
(``hgin.qt.QTBaseline``) runs on libhgin.so.  Pinned bit-for-bit to fixtures produced by executing the
reference's own ``QTBaseline`` (``tests/golden/make_golden_qt.py`` → ``tests/golden/qt_*.pt``).

The model, per sample (one homogeneous graph of path / link / node vertices):

* ``separate_edge_timesteps`` (``models.py:15-39``): of the path<->link edges (``edge_type == 0``, both
  directions), each edge's *position* is its index within the run of consecutive edges with the same
  source; ``pl_at_time[k]`` = the edges at position k, in original order.
* ``update_traffic`` (``models.py:103-121``): ``traffic = A`` (each path's PktsGen, 0 elsewhere); for
  k >= 1 the sources of position k-1 edges are thinned, ``traffic[src] *= 1 - bp[dst]``; for every k,
  ``T += scatter_sum(traffic[src_k] -> dst_k)``.
* ``update_blocking_probs`` (``models.py:125-132``): M/M/1/B with B = 32 on ``rho = T / (capacity/1000)``.
* three iterations (``models.py:134-145``), then the mean queue occupancy ``res`` per link from the
  truncated geometric series, and the per-path delay = sum over its links of ``res * 32000 / capacity``
  (``models.py:149-158``).
"""
from __future__ import annotations

from typing import List, Tuple

import torch

BUFFER = 32


def edge_positions(src: torch.Tensor) -> torch.Tensor:
    """Index of each edge inside its run of equal consecutive sources (models.py:17-29)."""
    n = src.numel()
    if n == 0:
        return torch.zeros(0, dtype=torch.long)
    start = torch.ones(n, dtype=torch.bool)
    start[1:] = src[1:] != src[:-1]
    first = torch.nonzero(start).view(-1)
    run = torch.cumsum(start.long(), 0) - 1
    return torch.arange(n) - first[run]


def position_groups(pos: torch.Tensor) -> List[torch.Tensor]:
    """pl_at_time: edge ids per position, original order inside a position (models.py:31-37)."""
    k_max = int(pos.max()) + 1 if pos.numel() else 0
    return [torch.nonzero(pos == k).view(-1) for k in range(k_max)]


def traffic_sum(src, dst, groups, a, bp) -> torch.Tensor:
    """update_traffic (models.py:103-121): per-position thinning and scatter sums, in the reference's order."""
    n = a.numel()
    t_sum = torch.zeros(n)
    traffic = None
    for k, idx in enumerate(groups):
        if k == 0:
            traffic = a.clone()
        else:
            prev = groups[k - 1]
            traffic[src[prev]] *= (1.0 - torch.gather(bp, 0, dst[prev]))
        t_sum += torch.zeros(n).scatter_add_(0, dst[idx], torch.gather(traffic, 0, src[idx]))
    return t_sum


def qt_baseline(edge_index, edge_type, vtype, P, L, num_iterations: int = 3) -> Tuple[torch.Tensor, torch.Tensor]:
    """(per-path delay [n_paths], per-link [occupancy, rho, pi_0] [n_links, 3]) as models.py:54-158."""
    ei = edge_index.long()
    n = vtype.numel()
    is_p, is_l = vtype == 0, vtype == 1
    sel = edge_type == 0
    src, dst = ei[0, sel], ei[1, sel]
    groups = position_groups(edge_positions(src))

    a = torch.zeros(n)
    a[is_p] = (P * torch.ones(int(is_p.sum()), 1))[:, 1]            # X[:, path_og.stop - 2]
    cap = (L * torch.ones(int(is_l.sum()), 1)) / 1000                 # X[is_l, link_og.start]
    cap = cap.view(-1)
    bp = 0.5 * torch.ones(n)

    for _ in range(num_iterations):
        t_sum = traffic_sum(src, dst, groups, a, bp)
        rho_all = 0.0 * bp
        rho_all[is_l] = t_sum[is_l] / cap
        bp = ((1.0 - rho_all) * torch.pow(rho_all, BUFFER)) / ((1.0 - torch.pow(rho_all, BUFFER + 1)) + 1e-08)
        rhos = t_sum[is_l] / cap
        pi_0 = (1 - rhos) / (1 - torch.pow(rhos, BUFFER + 1))
        occ = 1 * pi_0
        for j in range(32):
            pi_0 = pi_0 * rhos
            occ += (j + 1) * pi_0
        occ = occ / 32

    x = torch.zeros(n)
    x[is_l] = occ * 32000.0 / (L.squeeze(-1) * torch.ones(int(is_l.sum())))
    delay = torch.zeros(n).scatter_add_(0, src, torch.gather(x, 0, dst))[is_p]
    return delay, torch.cat([occ.view(-1, 1), rhos.view(-1, 1), pi_0.view(-1, 1)], 1)
