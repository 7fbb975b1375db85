"""hipGraph-captured training step for shuffled mini-batches of small graphs.

The reference's real workload is batches of 8 small network graphs (dataset.py:239-244, train.py:25-44):
a few thousand vertices per step, so every kernel is tiny and the step is bound by the host issuing ~300
launches (Python, autograd, ctypes).  HIP graphs remove that: the step runs on static-capacity buffers
(``GraphStore.padded_batch``: capacity = batch size x the largest graph; padding vertices isolated, the
fused loss limited to the batch's paths through a device-side count), is captured once after a short
warm-up, and each iteration is one batched-copy launch (``GraphStore.collate_into``) + one graph replay.

Numerically the padded step is the unpadded step: padding rows have no edges, so they never feed a real
row; their loss rows are masked, so their gradients are exactly zero and add nothing to any parameter
gradient.  The optimizer must be capturable (``torch.optim.Adam(..., capturable=True)``).
"""
from __future__ import annotations

from typing import Sequence

import torch

from .store import GraphStore, PaddedBatch
from .train import train_step


class CapturedTrainStep:
    def __init__(self, model: torch.nn.Module, opt: torch.optim.Optimizer, store: GraphStore, batch_size: int,
                 warmup_ids: Sequence[Sequence[int]], warmup: int = 3):
        if not all(g.get("capturable", False) for g in opt.param_groups):
            raise ValueError("CapturedTrainStep needs a capturable optimizer (e.g. Adam(..., capturable=True))")
        if not warmup_ids:
            raise ValueError("CapturedTrainStep needs at least one warm-up batch")
        self.model, self.opt, self.store = model, opt, store
        self.batch: PaddedBatch = store.padded_batch(batch_size)
        # warm-up on a side stream (allocator pools, lazily created constants, the optimizer state)
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for i in range(warmup):
                store.collate_into(warmup_ids[i % len(warmup_ids)], self.batch)
                train_step(model, opt, self.batch)
        torch.cuda.current_stream().wait_stream(side)
        self.graph = torch.cuda.CUDAGraph()
        opt.zero_grad(set_to_none=True)
        with torch.cuda.graph(self.graph):
            self.loss = train_step(model, opt, self.batch)

    def step(self, ids: Sequence[int]) -> torch.Tensor:
        """One training step on the graphs ``ids``; returns the device loss_value (no host sync)."""
        self.store.collate_into(ids, self.batch)
        self.graph.replay()
        return self.loss
