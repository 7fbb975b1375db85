"""Training-step harness mirroring the reference's ``train.py`` (train.py:12-13, 16-67, 140-148).

``train_step`` is one iteration of ``train_one_epoch``'s loop body: zero_grad, forward through the model
(``model(x_dict, edge_index_dict, path_batch)``, train.py:34), ``label = y.reshape(-1, 1)``, MAPE loss,
``sqrt``, backward, [gradient all-reduce across ranks], ``opt.step()``.  The reference additionally calls
``mape(out, label).item()`` every step (train.py:50); ``sync_metric=True`` reproduces that host sync, the
benchmark leaves it off.
"""
from __future__ import annotations

from typing import Optional

import torch

from .dist import GradAllReducer


def mape(preds: torch.Tensor, actuals: torch.Tensor) -> torch.Tensor:
    """train.py:12-13."""
    return 100.0 * torch.mean(torch.abs((preds - actuals) / actuals))


LOSSES = {"mape": mape}


def load_optimizer(config: dict, model: torch.nn.Module) -> torch.optim.Optimizer:
    """train.py:140-148."""
    kind = config.get("OPTIMIZER", "adam")
    lr, wd = config.get("LEARNING_RATE", 1e-3), config.get("WEIGHT_DECAY", 0)
    if kind == "adam":
        return torch.optim.Adam(lr=lr, params=model.parameters(), weight_decay=wd)
    if kind == "adamW":
        return torch.optim.AdamW(lr=lr, params=model.parameters(), weight_decay=wd)
    if kind == "sgd":
        return torch.optim.SGD(lr=lr, params=model.parameters(), weight_decay=wd)
    raise ValueError(f"unknown optimizer {kind!r}")


def train_step(model, opt, graph, loss_func=mape, reducer: Optional[GradAllReducer] = None,
               sync_metric: bool = False, fused_loss: bool = True):
    """One train.py:31-44 iteration.  ``fused_loss`` (default): when the loss is train.py's ``mape`` and the
    model offers ``forward_loss`` (hgin.HetroGIN), the readout head and the loss run fused (§8 F3)."""
    opt.zero_grad()
    label = graph.y.reshape(-1, 1)
    if fused_loss and loss_func is mape and hasattr(model, "forward_loss"):
        out, loss_value = model.forward_loss(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"], graph.y,
                                             getattr(graph, "m_valid", None))
    else:
        out = model(graph.x_dict(), graph.edge_index_dict(), graph.batch["path"])
        loss_value = loss_func(out, label)
    if reducer is None:
        loss = torch.sqrt(loss_value)
        loss.backward()
    else:
        # N ranks = one batch (hgin/dist.py): back-propagate this rank's path sum S_r = m_r * mape_r, then one
        # all-reduce turns the gradients into those of sqrt(batch mape) and returns the batch loss value
        m_valid = getattr(graph, "m_valid", None)
        m_local = (m_valid.to(torch.float32) if m_valid is not None
                   else torch.full((), float(label.numel()), dtype=torch.float32, device=loss_value.device))
        s_local = loss_value * m_local
        s_local.backward()
        loss_value = reducer.sync_sqrt_mean(s_local, m_local)
    opt.step()
    if sync_metric:
        return float(mape(out, label).item())
    return loss_value.detach()
