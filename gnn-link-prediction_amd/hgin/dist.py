"""Data-parallel training over one 8-GPU node: one process per GPU, RCCL over xGMI.

The reference is single-device (train.py:28,177).  Its unit of data parallelism is the graph batch: a
PyG mini-batch is a disjoint union of independent network samples (dataset.py:26, :242), so partitioning
by component gives every rank whole graphs — forward and backward aggregates stay local and the only
exchange is the parameter-gradient all-reduce (the north star's "embedding-gradient all-reduce").

Semantics: N ranks holding the components of ONE batch train exactly as one device holding the whole
batch (train.py:40-44: ``loss = sqrt(mape(out, label))`` over every path of the batch).  With S_r the
rank's sum of 100·|(out − y) / y| over its m_r paths, the batch loss is L = ΣS_r / Σm_r and

    ∇ sqrt(L) = Σ_r ∇S_r / (2 · M · sqrt(L)),   M = Σ m_r.

So every rank back-propagates its own S_r (linear in its paths, no collective inside the step), and
``GradAllReducer.sync_sqrt_mean`` all-reduces ONE contiguous fp32 buffer [every gradient | S_r | m_r]
(1.4 MB at cfg3 — one ring all-reduce, latency-bound on xGMI), then scales the gradients by
1 / (2 M sqrt(L)) on the device (no host sync).  The result equals the single-device gradient of the
union up to fp32 summation order, for any split of the paths over the ranks (tests/test_dist_gloo.py,
tests/test_gpu_dist.py).  Parameters whose gradient is None (dead relations, SURVEY.md §0.7 — the same
set on every rank, since every rank runs the same model on the same schema) stay None, so Adam skips them
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

    def _live(self):
        return [p for p in self.params if p.grad is not None]

    def sync_sqrt_mean(self, s_local: torch.Tensor, m_local: torch.Tensor) -> torch.Tensor:
        """After ``S_r.backward()`` on every rank: all-reduce [grads | S_r | m_r] once, scale the gradients to
        ∇ sqrt(ΣS / Σm) and return the batch loss value L = ΣS / Σm (a device scalar, no host sync)."""
        grads = [p.grad for p in self._live()]
        dev = s_local.device
        tail = torch.stack([s_local.detach().reshape(()).to(torch.float32),
                            m_local.detach().reshape(()).to(device=dev, dtype=torch.float32)])
        # pack / unpack as single multi-tensor launches (one cat, one foreach copy): a per-parameter copy
        # loop would add ~2 x 60 tiny kernels to every step on every rank
        flat = torch.cat([g.reshape(-1) for g in grads] + [tail])
        if world() > 1:
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        s_tot, m_tot = flat[-2], flat[-1]
        loss_value = s_tot / m_tot
        if grads:
            scale = 0.5 / (m_tot * torch.sqrt(loss_value))
            body = flat[:-2].mul_(scale)
            parts = body.split([g.numel() for g in grads])
            torch._foreach_copy_(grads, [v.view_as(g) for v, g in zip(parts, grads)])
        return loss_value
