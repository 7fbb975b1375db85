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
tests/test_gpu_dist.py).

The packed layout is rank-independent: every parameter has its slot, a locally-missing (None) gradient is sent
as zeros, and one presence count per parameter rides in the same buffer.  A parameter whose gradient is None on
every rank (dead relations, SURVEY.md §0.7 — the same set everywhere, since every rank runs the same model on
the same schema) stays None, so Adam skips it exactly as it does single-device.  A parameter live on some ranks
but not others would be a layout bug in the caller (hgin/partition.py runs the readout even on a rank that owns
no paths so this cannot happen); it is detected on the device without a host sync (``inconsistent``) and
``check()`` raises on it.
"""
from __future__ import annotations

from typing import Iterable, List

import torch
import torch.distributed as dist


def world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def rank(group=None) -> int:
    return dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0


class GradAllReducer:
    def __init__(self, params: Iterable[torch.nn.Parameter], group=None):
        seen, ps = set(), []
        for p in params:
            if p.requires_grad and id(p) not in seen:
                seen.add(id(p))
                ps.append(p)
        self.params: List[torch.nn.Parameter] = ps
        self.group = group
        self.inconsistent = None    # device bool: some parameter had a gradient on some ranks only
        self._flat = None
        self._pres = {}             # live-parameter set -> its device presence vector (built once per set)

    def sync_sqrt_mean(self, s_local: torch.Tensor, m_local: torch.Tensor) -> torch.Tensor:
        """After ``S_r.backward()`` on every rank: all-reduce [grads | presence | S_r | m_r] once, scale the
        gradients to ∇ sqrt(ΣS / Σm) and return the batch loss value L = ΣS / Σm (a device scalar, no host
        sync).  Every rank sends every parameter's slot (zeros where its gradient is None)."""
        dev = s_local.device
        sizes = [p.numel() for p in self.params]
        n_body, n_par = sum(sizes), len(self.params)
        if self._flat is None or self._flat.device != dev or self._flat.numel() != n_body + n_par + 2:
            self._flat = torch.empty(n_body + n_par + 2, dtype=torch.float32, device=dev)
        flat = self._flat
        live = [i for i, p in enumerate(self.params) if p.grad is not None]
        # pack as a few multi-tensor launches (one zero fill, one foreach copy): a per-parameter copy loop
        # would add ~2 x 60 tiny kernels to every step on every rank
        flat.zero_()
        body = flat[:n_body].split(sizes)
        if live:
            torch._foreach_copy_([body[i].view_as(self.params[i].grad) for i in live],
                                 [self.params[i].grad for i in live])
        pres = flat[n_body:n_body + n_par]
        key = (dev, tuple(live))
        if key not in self._pres:
            v = torch.zeros(n_par, dtype=torch.float32)
            v[live] = 1.0
            self._pres[key] = v.to(dev)
        pres.copy_(self._pres[key])
        flat[-2] = s_local.detach().reshape(()).to(torch.float32)
        flat[-1] = m_local.detach().reshape(()).to(device=dev, dtype=torch.float32)
        if dist.is_available() and dist.is_initialized():
            # (also at world size 1: the collective path itself then runs on the backend)
            dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=self.group)
        w = float(world(self.group))
        bad = ((pres > 0) & (pres < w)).any()
        self.inconsistent = bad if self.inconsistent is None else (self.inconsistent | bad)
        s_tot, m_tot = flat[-2], flat[-1]
        loss_value = s_tot / m_tot
        if live:
            scale = 0.5 / (m_tot * torch.sqrt(loss_value))
            flat[:n_body].mul_(scale)
            torch._foreach_copy_([self.params[i].grad for i in live],
                                 [body[i].view_as(self.params[i].grad) for i in live])
        return loss_value

    def check(self) -> None:
        """Raise if any step so far saw a parameter with a gradient on some ranks but not on others (one host
        sync; tests and the bench call it after the timed region)."""
        if self.inconsistent is not None and bool(self.inconsistent):
            raise RuntimeError("GradAllReducer: a parameter had a gradient on some ranks only (rank-dependent "
                               "dead parameters: the ranks' updates diverge)")
