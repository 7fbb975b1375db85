"""Data-parallel training over one 8-GPU node: one process per GPU, RCCL over xGMI.

The reference is single-device (train.py:28,177).  Its unit of data parallelism is the graph batch: a
PyG mini-batch is a disjoint union of independent network samples (dataset.py:26, :242), so partitioning
by component gives every rank whole graphs — forward and backward aggregates stay local and the only
exchange is the parameter-gradient all-reduce (the north star's "embedding-gradient all-reduce").

``GradAllReducer`` flattens every gradient into ONE contiguous fp32 buffer (1.1 MB at cfg2, 5.5 MB at
cfg3 — one ring all-reduce, latency- not bandwidth-bound on xGMI), all-reduces it (sum) and scales by
1 / world_size, which equals the gradient of the mean loss over all ranks' paths when ranks hold equal path
counts.  Parameters whose gradient is None on this rank (dead relations, SURVEY.md §0.7 — the same set on
every rank, since every rank runs the same model on the same schema) are left None, so Adam skips them
exactly as it does single-device.
"""
from __future__ import annotations

from typing import Iterable, List

import torch
import torch.distributed as dist


def world() -> int:
    return dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1


def rank() -> int:
    return dist.get_rank() if dist.is_available() and dist.is_initialized() else 0


class GradAllReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        seen, ps = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        self.params: List[torch.nn.Parameter] = ps
        self.group = group

    def sync(self) -> None:
        n = world()
        if n == 1:
            return
        live = [p for p in self.params if p.grad is not None]
        if not live:
            return
        # pack / unpack as single multi-tensor launches (one cat, one foreach copy): a per-parameter copy
        # loop would add ~2 x 60 tiny kernels to every step on every rank
        grads = [p.grad for p in live]
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        flat.mul_(1.0 / n)
        parts = flat.split([g.numel() for g in grads])
        torch._foreach_copy_(grads, [v.view_as(g) for v, g in zip(parts, grads)])
