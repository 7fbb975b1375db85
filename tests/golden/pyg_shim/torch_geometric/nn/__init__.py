import torch
from . import conv  # noqa: F401
from .conv import MessagePassing, HeteroConv  # noqa: F401


def _pool(x, batch, reduce):
    size = int(batch.max().item()) + 1 if batch.numel() > 0 else 0
    out = torch.zeros(size, x.size(1), dtype=x.dtype)
    idx = batch.view(-1, 1).expand_as(x)
    return out.scatter_reduce(0, idx, x, reduce=reduce, include_self=False)


def global_mean_pool(x, batch):
    return _pool(x, batch, "mean")


def global_max_pool(x, batch):
    return _pool(x, batch, "amax")
