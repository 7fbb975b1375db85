import torch


def scatter(src, index, dim=-1, out=None, dim_size=None, reduce="sum"):
    """torch_scatter.scatter, reduce='sum' only: zeros().scatter_add_() after broadcasting index."""
    assert reduce in ("sum", "add") and out is None
    dim = dim if dim >= 0 else src.dim() + dim
    if index.dim() == 1:
        shape = [1] * src.dim()
        shape[dim] = -1
        index = index.view(shape).expand_as(src)
    size = list(src.size())
    size[dim] = dim_size if dim_size is not None else (int(index.max()) + 1 if index.numel() else 0)
    return torch.zeros(size, dtype=src.dtype, device=src.device).scatter_add_(dim, index, src)
