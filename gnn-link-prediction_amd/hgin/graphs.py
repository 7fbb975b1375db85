"""hipGraph-captured training and evaluation steps for shuffled mini-batches of small graphs.

The reference's real workload is batches of 8 small network graphs (dataset.py:239-244, train.py:25-44):
a few thousand vertices per step, so every kernel is tiny and the step is bound by the host issuing ~300
launches (Python, autograd, ctypes).  HIP graphs remove that: the step runs on static-capacity buffers
(``GraphStore.padded_batch``: capacity = batch size x the largest graph; padding vertices isolated, the
fused loss limited to the batch's paths through a device-side count), is captured once after a short
warm-up, and each iteration is one batched-copy launch (``GraphStore.collate_into``) + one graph replay.

Numerically the padded step is the unpadded step (MLP_BN's batch statistics taken over the batch's rows only;
dropout draws its masks per replay, so a step with dropout equals an eager step in distribution, not bitwise):
padding rows have no edges, so they never feed a real row; their loss rows
are masked, so their gradients are exactly zero and add nothing to any parameter gradient.  GLOBAL_FEATS' pooling
(models.py:347-352) sees the padding path rows as one more graph (collate_into gives them the id batch_size, past
every real graph), so the real graphs' pooled features are the exact batch's.  The optimizer must be capturable (``torch.optim.Adam(..., capturable=True)``).
"""
from __future__ import annotations

from typing import Optional, Sequence

import torch

from .store import GraphStore, PaddedBatch
from .train import mape, train_step


def _check_row_independent(model: torch.nn.Module) -> None:
    """A padded batch equals the exact batch only when nothing mixes rows across the batch outside the
    graph's edges: padding path rows carry stale data and still pass through the readout.  MLP_BN's BatchNorm1d
    takes its statistics over the first m_valid rows only (models._masked_batch_norm); global pooling pools the
    padding rows as a graph of their own; dropout is row-wise and draws fresh masks on every replay — the captured
    RNG offset advances — as an eager step would.  Other BatchNorm kinds are refused."""
    if any(isinstance(m, torch.nn.modules.batchnorm._BatchNorm) and not isinstance(m, torch.nn.BatchNorm1d)
           for m in model.modules()):
        raise ValueError("CapturedTrainStep: only BatchNorm1d (MLP_BN) takes the padded batch's masked statistics")
    _check_no_bipartite_loops(model)


def _check_no_bipartite_loops(model: torch.nn.Module) -> None:
    """HetroGAT's GATConvs add the self loops (i, i) for i < min(N_src, N_dst) on bipartite relations (PyG 2.0.2,
    models.py:413-418): on a padded batch N_src / N_dst are the capacities, so real destination rows between the two
    real counts would gain a loop from a padding source row and their softmax would change.  The fused step
    (hgin/smallbatch.py SmallBatchStep / SmallBatchEval) counts the real rows on the device and takes HetroGAT; the
    captured padded path refuses it."""
    from .gat import GATConv
    if any(isinstance(m, GATConv) and m.add_self_loops for m in model.modules()):
        raise ValueError("captured padded steps: GATConv's bipartite self loops depend on the batch's real row counts, "
                         "which a padded batch hides — use SmallBatchStep / SmallBatchEval or eager steps")


class CapturedTrainStep:
    def __init__(self, model: torch.nn.Module, opt: torch.optim.Optimizer, store: GraphStore, batch_size: int,
                 warmup_ids: Sequence[Sequence[int]], warmup: int = 3):
        if not all(g.get("capturable", False) for g in opt.param_groups):
            raise ValueError("CapturedTrainStep needs a capturable optimizer (e.g. Adam(..., capturable=True))")
        if not warmup_ids:
            raise ValueError("CapturedTrainStep needs at least one warm-up batch")
        _check_row_independent(model)
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


def _forward_backward(model: torch.nn.Module, graph, distributed: bool = False):
    """train.py:33-43 without zero_grad / opt.step: forward (fused head + MAPE, §8 F3), sqrt, backward.

    ``distributed``: back-propagate the rank's path sum S_r = m_r * mape_r instead (hgin/dist.py) and return
    (S_r, m_r) for ``GradAllReducer.sync_sqrt_mean``."""
    if hasattr(model, "forward_loss"):
        _, loss_value = model.forward_loss(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"], graph.y,
                                           getattr(graph, "m_valid", None))
    else:
        loss_value = mape(model(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"]), graph.y.reshape(-1, 1))
    if not distributed:
        torch.sqrt(loss_value).backward()
        return loss_value.detach()
    m_valid = getattr(graph, "m_valid", None)
    m_local = (m_valid.to(torch.float32) if m_valid is not None
               else torch.full((), float(graph.y.numel()), dtype=torch.float32, device=loss_value.device))
    s_local = loss_value * m_local
    s_local.backward()
    return s_local.detach(), m_local


class CapturedStaticStep:
    """hipGraph replay of train.py's step on a resident graph whose tensors never move (cfg2-cfg5: one large
    static graph per rank, the bench workload).

    An eager step issues ~90 launches from Python (autograd, ctypes); a replay issues them as one graph.  At
    the bench sizes the two measure the same (cfg2 5.76 vs 5.74 ms, cfg5 101.4 vs 101.5 ms: the host runs
    ahead of a GPU-bound step, and the ~0.2 ms of kernel-to-kernel gaps per cfg2 step remain in a replay),
    so bench.py uses it only with ``--graph``.  Capture protocol (the standard whole-step one): a few eager warm-up steps on a side stream
    (CSR / CSC caches, allocator pools, optimizer state), gradients set to None, then forward + loss +
    backward captured — the captured backward (re)writes every .grad in place on each replay — followed by
    the optimizer step.  With a ``reducer`` (N > 1) the captured backward is that of the rank's path sum and the
    RCCL gradient all-reduce (+ the sqrt-loss scaling, hgin/dist.py) runs eagerly between two replays
    (forward/backward, then the optimizer), so no collective is captured.  The optimizer must be
    capturable (``torch.optim.Adam(..., capturable=True)``).  Every kernel is the eager step's, in the same
    order, so a replay equals an eager step with the same optimizer bit for bit (tests/test_gpu_model.py)."""

    def __init__(self, model: torch.nn.Module, opt: torch.optim.Optimizer, graph, reducer=None, warmup: int = 2):
        if not all(g.get("capturable", False) for g in opt.param_groups):
            raise ValueError("CapturedStaticStep needs a capturable optimizer (e.g. Adam(..., capturable=True))")
        self.model, self.opt, self.graph, self.reducer = model, opt, graph, reducer
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):
            for _ in range(max(int(warmup), 1)):
                train_step(model, opt, graph, reducer=reducer)
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        opt.zero_grad(set_to_none=True)
        self.fwd_bwd = torch.cuda.CUDAGraph()
        self.opt_graph: Optional[torch.cuda.CUDAGraph] = None
        with torch.cuda.graph(self.fwd_bwd):
            self.loss = _forward_backward(model, graph, distributed=reducer is not None)
            if reducer is None:
                opt.step()
        if reducer is not None:
            self.opt_graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.opt_graph, pool=self.fwd_bwd.pool()):
                opt.step()

    def step(self) -> torch.Tensor:
        """One training step; returns the device loss_value (no host sync)."""
        self.fwd_bwd.replay()
        if self.opt_graph is None:
            return self.loss
        loss_value = self.reducer.sync_sqrt_mean(*self.loss)
        self.opt_graph.replay()
        return loss_value


class CapturedEvalStep:
    """train.py's evaluation loops — ``test()`` (train.py:70-113, after ``model.eval()``, :192) and ``evaluate()``
    (:322-348) — as one batched-copy launch + one hipGraph replay per batch: the forward and the fused head + MAPE
    (F3, limited to the batch's paths by the padded batch's device count) under ``torch.no_grad()``, on the same
    static-capacity buffers as ``CapturedTrainStep``.  The replay also adds the batch's loss_value and its path-
    weighted form into device accumulators (the reference's ``running_loss += loss_value.item()`` and
    ``running_loss_mape += mape * n_paths``), so a whole evaluation pass syncs the host once, in ``result()``.

    The model must be in eval mode (BatchNorm then reads its running statistics and dropout is off: both
    row-independent, so the padded batch equals the exact one); GLOBAL_FEATS pools the padding path rows as a graph of
    their own (collate_into's padding id), so the real graphs' pooled features are the exact batch's."""

    def __init__(self, model: torch.nn.Module, store: GraphStore, batch_size: int,
                 warmup_ids: Sequence[Sequence[int]], warmup: int = 2):
        if model.training:
            raise ValueError("CapturedEvalStep: call model.eval() first (train.py:192, :329)")
        if not warmup_ids:
            raise ValueError("CapturedEvalStep needs at least one warm-up batch")
        _check_no_bipartite_loops(model)
        self.model, self.store = model, store
        self.batch: PaddedBatch = store.padded_batch(batch_size)
        dev = self.batch.y.device
        self.loss_sum = torch.zeros((), dtype=torch.float32, device=dev)
        self.loss_paths = torch.zeros((), dtype=torch.float32, device=dev)
        self.batches = 0
        self._warm = (list(warmup_ids), warmup)
        self._capture()

    def _capture(self) -> None:
        """Warm up on a side stream, then capture forward + fused head / MAPE + the accumulation once.  The graph holds
        the parameters' device pointers: they are recorded, and ``step`` re-captures if they move."""
        warmup_ids, warmup = self._warm
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side), torch.no_grad():
            for i in range(max(1, warmup)):
                self.store.collate_into(warmup_ids[i % len(warmup_ids)], self.batch)
                self._forward()
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph), torch.no_grad():
            self.out, self.loss = self._forward()
            self.loss_sum.add_(self.loss)
            self.loss_paths.add_(self.loss * self.batch.m_valid[0].to(torch.float32))
        self._ptrs = self._param_ptrs()

    def _param_ptrs(self):
        ps = list(self.model.parameters())
        return (ps[0].data_ptr(), ps[-1].data_ptr()) if ps else ()

    def _forward(self):
        b = self.batch
        return self.model.forward_loss(b.x_dict(), b.edge_index_dict(), b.batch["path"], b.y, b.m_valid)

    def step(self, ids: Sequence[int]) -> torch.Tensor:
        """Evaluate the graphs ``ids``; returns the batch's device loss_value (overwritten by the next step).  The
        predictions are ``self.out[:n_paths]`` until then.  If the parameters were re-allocated since the capture (a
        folding SmallBatchStep, model.to()), the step is re-captured first (the running sums are kept)."""
        if self._param_ptrs() != self._ptrs:
            acc = (self.loss_sum.clone(), self.loss_paths.clone())
            self._capture()
            self.loss_sum.copy_(acc[0])
            self.loss_paths.copy_(acc[1])
        self.store.collate_into(ids, self.batch)
        self.graph.replay()
        self.batches += 1
        return self.loss

    def reset(self) -> None:
        self.loss_sum.zero_()
        self.loss_paths.zero_()
        self.batches = 0

    def result(self, n_paths: int) -> tuple:
        """(average loss over the batches, path-weighted MAPE) = test()'s (average_loss, mape_loss) for a loss_func
        of MAPE; ``n_paths`` = the paths evaluated (the host knows the graphs).  One host sync."""
        s, w = float(self.loss_sum), float(self.loss_paths)
        return s / max(self.batches, 1), w / max(n_paths, 1)
