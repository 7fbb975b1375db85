import math

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


def _glorot(t):
    """torch_geometric.nn.inits.glorot: U(-a, a), a = sqrt(6 / (size(-2) + size(-1)))."""
    if t is not None:
        a = math.sqrt(6.0 / (t.size(-2) + t.size(-1)))
        t.data.uniform_(-a, a)


class Linear(torch.nn.Module):
    """torch_geometric.nn.dense.linear.Linear (2.0.2), the bias-free glorot form GATConv uses.  in_channels = -1 is
    lazy: the weight is an UninitializedParameter until the first forward, whose pre-hook materialises it as
    [out, in] and initialises it (glorot, on the parameter's device RNG) — so lazy weights consume the RNG after
    everything the constructor initialised, in forward call order."""

    def __init__(self, in_channels, out_channels, bias=False, weight_initializer="glorot"):
        super().__init__()
        assert not bias and weight_initializer == "glorot"
        self.in_channels, self.out_channels = in_channels, out_channels
        if in_channels > 0:
            self.weight = torch.nn.Parameter(torch.Tensor(out_channels, in_channels))
        else:
            self.weight = torch.nn.parameter.UninitializedParameter()
            self._hook = self.register_forward_pre_hook(self._initialize)
        self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        if self.in_channels > 0:
            _glorot(self.weight)

    @torch.no_grad()
    def _initialize(self, module, inputs):
        if isinstance(self.weight, torch.nn.parameter.UninitializedParameter):
            self.in_channels = inputs[0].size(-1)
            self.weight.materialize((self.out_channels, self.in_channels))
            self.reset_parameters()
        self._hook.remove()
        delattr(self, "_hook")

    def forward(self, x):
        return torch.nn.functional.linear(x, self.weight, None)


def _softmax(src, index, num_nodes):
    """torch_geometric.utils.softmax (2.0.2, index form): per-destination max (torch_scatter max: 0 for empty
    groups), exp(src - max), per-destination sum, out / (sum + 1e-16)."""
    shape = (num_nodes,) + tuple(src.shape[1:])
    idx = index.view(-1, *([1] * (src.dim() - 1))).expand_as(src)
    src_max = torch.zeros(shape, dtype=src.dtype).scatter_reduce(0, idx, src, reduce="amax", include_self=False)
    out = (src - src_max.index_select(0, index)).exp()
    out_sum = torch.zeros(shape, dtype=src.dtype).scatter_add_(0, idx, out)
    return out / (out_sum.index_select(0, index) + 1e-16)


class GATConv(MessagePassing):
    """PyG 2.0.2 GATConv restated (heads, concat, negative_slope 0.2, dropout 0, add_self_loops, bias): the source
    and destination features go through lin_src / lin_dst (one shared Linear for an int in_channels), the per-node
    logits alpha = (x W^T . att).sum(-1); on a Tensor edge_index the self-loops are removed and (i, i) added for
    i < min(N_src, N_dst) — for a bipartite (two node types) relation too; then per edge alpha_j + alpha_i,
    leaky_relu(0.2), softmax over each destination's incoming edges, the message x_j * alpha summed into the
    destination; concat -> [N_dst, heads * C] (else the mean over heads), + bias."""

    def __init__(self, in_channels, out_channels, heads=1, concat=True, negative_slope=0.2, dropout=0.0,
                 add_self_loops=True, bias=True, **kwargs):
        kwargs.setdefault("aggr", "add")
        super().__init__(node_dim=0, **kwargs)
        self.in_channels, self.out_channels = in_channels, out_channels
        self.heads, self.concat, self.negative_slope = heads, concat, negative_slope
        self.dropout, self.add_self_loops = dropout, add_self_loops
        if isinstance(in_channels, int):
            self.lin_src = Linear(in_channels, heads * out_channels, bias=False, weight_initializer="glorot")
            self.lin_dst = self.lin_src
        else:
            self.lin_src = Linear(in_channels[0], heads * out_channels, False, weight_initializer="glorot")
            self.lin_dst = Linear(in_channels[1], heads * out_channels, False, weight_initializer="glorot")
        self.att_src = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        self.att_dst = torch.nn.Parameter(torch.Tensor(1, heads, out_channels))
        if bias and concat:
            self.bias = torch.nn.Parameter(torch.Tensor(heads * out_channels))
        elif bias:
            self.bias = torch.nn.Parameter(torch.Tensor(out_channels))
        else:
            self.register_parameter("bias", None)
        self.reset_parameters()

    def reset_parameters(self):
        self.lin_src.reset_parameters()
        self.lin_dst.reset_parameters()
        _glorot(self.att_src)
        _glorot(self.att_dst)
        if self.bias is not None:
            self.bias.data.fill_(0)

    def forward(self, x, edge_index, size=None):
        H, C = self.heads, self.out_channels
        if isinstance(x, Tensor):
            x_src = x_dst = self.lin_src(x).view(-1, H, C)
        else:
            x_src, x_dst = x
            x_src = self.lin_src(x_src).view(-1, H, C)
            if x_dst is not None:
                x_dst = self.lin_dst(x_dst).view(-1, H, C)
        alpha_src = (x_src * self.att_src).sum(dim=-1)
        alpha_dst = None if x_dst is None else (x_dst * self.att_dst).sum(-1)
        assert isinstance(edge_index, Tensor) and edge_index.dtype == torch.long
        if self.add_self_loops:
            num_nodes = x_src.size(0)
            if x_dst is not None:
                num_nodes = min(num_nodes, x_dst.size(0))
            num_nodes = min(size) if size is not None else num_nodes
            edge_index = edge_index[:, edge_index[0] != edge_index[1]]                      # remove_self_loops
            loop = torch.arange(num_nodes, dtype=torch.long)
            edge_index = torch.cat([edge_index, torch.stack([loop, loop], 0)], dim=1)      # add_self_loops
        n_dst = x_dst.size(0) if x_dst is not None else (size[1] if size is not None else x_src.size(0))
        j, i = edge_index[0], edge_index[1]
        alpha = alpha_src.index_select(0, j)
        if alpha_dst is not None:
            alpha = alpha + alpha_dst.index_select(0, i)
        alpha = torch.nn.functional.leaky_relu(alpha, self.negative_slope)
        alpha = _softmax(alpha, i, n_dst)
        self.alpha_trace = alpha.detach().clone()
        msg = x_src.index_select(0, j) * alpha.unsqueeze(-1)
        from torch_scatter import scatter
        out = scatter(msg, i, dim=0, dim_size=n_dst, reduce="sum")
        self.trace.append(out.detach().clone())
        out = out.view(-1, H * C) if self.concat else out.mean(dim=1)
        if self.bias is not None:
            out = out + self.bias
        return out


from .hetero_conv import HeteroConv  # noqa: E402,F401
