from collections import defaultdict

import torch


def _group(xs, aggr):
    if len(xs) == 0:
        return None
    if len(xs) == 1:
        return xs[0]
    out = torch.stack(xs, dim=0)
    return getattr(torch, aggr)(out, dim=0)


class HeteroConv(torch.nn.Module):
    """PyG 2.0.2 HeteroConv restated (see ../../../README.md)."""

    def __init__(self, convs, aggr="sum"):
        super().__init__()
        self.convs = torch.nn.ModuleDict({"__".join(k): v for k, v in convs.items()})
        self.aggr = aggr

    def reset_parameters(self):
        for conv in self.convs.values():
            conv.reset_parameters()

    def forward(self, x_dict, edge_index_dict):
        out_dict = defaultdict(list)
        for edge_type, edge_index in edge_index_dict.items():
            src, rel, dst = edge_type
            key = "__".join(edge_type)
            if key not in self.convs:
                continue
            conv = self.convs[key]
            if src == dst:
                out = conv(x_dict[src], edge_index)
            else:
                out = conv((x_dict[src], x_dict[dst]), edge_index)
            out_dict[dst].append(out)
        for k, v in out_dict.items():
            out_dict[k] = _group(v, self.aggr)
        return out_dict
