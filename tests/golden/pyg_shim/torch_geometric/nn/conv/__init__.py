import torch
from torch import Tensor


class MessagePassing(torch.nn.Module):
    """PyG 2.0.2 MessagePassing, restated for Tensor edge_index and aggr='add' only."""

    def __init__(self, aggr="add", flow="source_to_target", node_dim=-2, **kwargs):
        super().__init__()
        assert aggr == "add" and flow == "source_to_target"
        self.aggr = aggr
        self.flow = flow
        self.node_dim = node_dim
        self.trace = []  # fixture hook: every aggregate computed, in call order

    def propagate(self, edge_index, size=None, **kwargs):
        assert isinstance(edge_index, Tensor)
        assert edge_index.dtype == torch.long
        assert edge_index.dim() == 2
        assert edge_index.size(0) == 2
        x = kwargs["x"]
        if isinstance(x, Tensor):
            x = (x, x)
        x_j = x[0].index_select(self.node_dim, edge_index[0])
        msg = self.message(x_j)
        dim_size = x[1].size(self.node_dim) if x[1] is not None else (
            size[1] if size is not None else int(edge_index[1].max()) + 1)
        from torch_scatter import scatter
        out = scatter(msg, edge_index[1], dim=self.node_dim, dim_size=dim_size, reduce="sum")
        self.trace.append(out.detach().clone())
        return out

    def message(self, x_j):
        return x_j


class GATConv(torch.nn.Module):  # HetroGAT is out of scope
    def __init__(self, *a, **k):
        raise NotImplementedError("pyg_shim: GATConv is not restated")


from .hetero_conv import HeteroConv  # noqa: E402,F401
