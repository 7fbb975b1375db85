"""Synthetic heterogeneous RouteNet-style graphs and PyG-style batch collation.

The reference's real data are GNNet-Challenge-2021 samples converted to PyG ``HeteroData`` with three
node types and six relations, in this insertion order (``dataset.py:112-117``):

    ('path','uses','link'), ('link','includes','path'), ('link','connects','node'),
    ('node','has','link'),  ('path','is_connected','node'), ('node','is_used','path')

``generateFiles.py:43-78`` adds every relation together with its reverse, so the reverse relations are
exact flips of the forward ones.  The dataset cannot be downloaded here (``downloadDataset.py:5-9``), so
the benchmark and the parity tests use synthetic graphs of the same schema:

* forward relations p->l, l->n, p->n: endpoints i.i.d. uniform (``torch.randint``) from one generator;
* reverse relations l->p, n->l (and n->p when requested): ``edge_index.flip(0)``;
* features ``randn``; labels ``rand + 0.5`` (keeps MAPE away from division by ~0).

``collate`` restates PyG's ``Batch.from_data_list`` for ``HeteroData`` (``dataset.py:239-244``): per node
type the features are concatenated and each relation's ``edge_index`` rows are offset by the running node
counts of its src / dst types; ``batch`` vectors record the graph of every node.
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Dict, List, Optional, Tuple

import torch

EdgeType = Tuple[str, str, str]

REL_PL: EdgeType = ("path", "uses", "link")
REL_LP: EdgeType = ("link", "includes", "path")
REL_LN: EdgeType = ("link", "connects", "node")
REL_NL: EdgeType = ("node", "has", "link")
REL_PN: EdgeType = ("path", "is_connected", "node")
REL_NP: EdgeType = ("node", "is_used", "path")
# dataset.py:112-117 insertion order
ALL_RELATIONS: List[EdgeType] = [REL_PL, REL_LP, REL_LN, REL_NL, REL_PN, REL_NP]
# the four relations HetroGIN convolves (models.py:286-298)
CONV_RELATIONS: List[EdgeType] = [REL_PL, REL_LP, REL_LN, REL_NL]
NODE_TYPES = ("path", "link", "node")


@dataclass
class GraphConfig:
    """One synthetic workload (sizes from BASELINE.json:configs)."""

    name: str
    n_path: int
    n_link: int
    n_node: int
    e_pl: int            # edges of path->link (and, flipped, link->path)
    e_ln: int            # edges of link->node (and, flipped, node->link)
    e_pn: int            # edges of path->node (0: relation absent)
    f_path: int
    f_link: int
    f_node: int
    hidden: int
    layers: int
    with_np: bool = False            # also carry node->path (flip of p->n)
    divided_features: bool = True    # config.json:18
    bl_features: bool = True         # config.json:17
    concat_path: bool = True         # config.json:24
    global_feats: bool = False       # config.json:25
    mlp_layers: List[int] = field(default_factory=lambda: [128, 32])   # config.json:26
    feat_dtype: str = "f32"          # "bf16": cfg5 storage (features, activations, gradients); fp32 params
    components: int = 1              # > 1: generated as this many independent, equal components (cfg4)

    @property
    def graph_edges(self) -> int:
        return 2 * self.e_pl + 2 * self.e_ln + self.e_pn * (2 if self.with_np else 1)

    @property
    def conv_edges(self) -> int:
        """Edges of the relations HetroGIN convolves (counted once per step)."""
        return 2 * self.e_pl + 2 * self.e_ln

    @property
    def nodes(self) -> int:
        return self.n_path + self.n_link + self.n_node

    def model_kwargs(self, input_channels: Dict[str, int]) -> dict:
        """Keyword arguments exactly as train.py:128-132 passes them."""
        return dict(input_channels=input_channels, node_embedding_size=self.hidden,
                    message_passing_layers=self.layers, dropout=0.0, concat_path=self.concat_path,
                    bl_features=self.bl_features, divided_features=self.divided_features,
                    global_feats=self.global_feats, mlp_layers=list(self.mlp_layers),
                    act="torch.nn.PReLU()", mlp_bn=False, mlp_head_act=None)


CONFIGS: Dict[str, GraphConfig] = {
    # configs[0]: 1k nodes / 5k edges, reference 7/7/3 layout, config.json flags, H=8, L=2
    "cfg1": GraphConfig("cfg1", 600, 300, 100, 2000, 500, 0, 7, 7, 3, 8, 2,
                        divided_features=False, bl_features=False),
    # configs[1]: 1M nodes / 10M edges, 5 relations, hidden 128, L=2
    "cfg2": GraphConfig("cfg2", 600_000, 300_000, 100_000, 3_000_000, 500_000, 3_000_000,
                        128, 128, 128, 128, 2),
    # configs[2]: 10M nodes / 100M edges, hidden 256, L=3
    "cfg3": GraphConfig("cfg3", 6_000_000, 3_000_000, 1_000_000, 30_000_000, 5_000_000, 30_000_000,
                        256, 256, 256, 256, 3),
    # cfg4 component: one eighth of cfg3 (one per GPU of the 8-GPU node)
    "cfg4c": GraphConfig("cfg4c", 750_000, 375_000, 125_000, 3_750_000, 625_000, 3_750_000,
                         256, 256, 256, 256, 3),
    # configs[3]: cfg3's 100M edges generated as 8 independent components; N GPUs take 8/N each
    "cfg4": GraphConfig("cfg4", 6_000_000, 3_000_000, 1_000_000, 30_000_000, 5_000_000, 30_000_000,
                        256, 256, 256, 256, 3, components=8),
    # configs[4]: cfg3 with bf16 node features + bf16 MFMA update (fp32 accumulate, fp32 master weights)
    "cfg5": GraphConfig("cfg5", 6_000_000, 3_000_000, 1_000_000, 30_000_000, 5_000_000, 30_000_000,
                        256, 256, 256, 256, 3, feat_dtype="bf16"),
    # cfg5 at cfg2 size (the bf16 counterpart of the headline fp32 config)
    "cfg2bf": GraphConfig("cfg2bf", 600_000, 300_000, 100_000, 3_000_000, 500_000, 3_000_000,
                          128, 128, 128, 128, 2, feat_dtype="bf16"),
}


def scaled_config(base: GraphConfig, factor: float, name: Optional[str] = None) -> GraphConfig:
    """Same schema, every count multiplied by ``factor`` (for bounded CPU samples and tests)."""
    import dataclasses
    s = lambda v: max(1, int(round(v * factor))) if v else 0  # noqa: E731
    return dataclasses.replace(base, name=name or f"{base.name}x{factor:g}", n_path=s(base.n_path),
                               n_link=s(base.n_link), n_node=s(base.n_node), e_pl=s(base.e_pl),
                               e_ln=s(base.e_ln), e_pn=s(base.e_pn))


@dataclass
class HeteroGraph:
    """Dict-of-tensors hetero graph (what ``HeteroData.x_dict`` / ``edge_index_dict`` expose)."""

    x: Dict[str, torch.Tensor]
    edge_index: Dict[EdgeType, torch.Tensor]
    y: torch.Tensor
    batch: Dict[str, torch.Tensor]

    def x_dict(self) -> Dict[str, torch.Tensor]:
        # A fresh dict per call, like HeteroData.x_dict: HetroGIN.forward assigns into it (models.py:333-342).
        return dict(self.x)

    def edge_index_dict(self) -> Dict[EdgeType, torch.Tensor]:
        return dict(self.edge_index)

    def to(self, device, non_blocking: bool = False) -> "HeteroGraph":
        mv = lambda t: t.to(device, non_blocking=non_blocking)  # noqa: E731
        return HeteroGraph({k: mv(v) for k, v in self.x.items()},
                           {k: mv(v) for k, v in self.edge_index.items()}, mv(self.y),
                           {k: mv(v) for k, v in self.batch.items()})

    def num_nodes(self, t: str) -> int:
        return int(self.x[t].shape[0])


def synthetic_graph(cfg: GraphConfig, seed: int = 0, device="cpu") -> HeteroGraph:
    """SURVEY.md §8.D generator: randint endpoints, flipped reverse relations, randn features."""
    g = torch.Generator(device=device).manual_seed(seed)
    ri = lambda hi, n: torch.randint(0, hi, (n,), generator=g, device=device, dtype=torch.long)  # noqa: E731
    pl = torch.stack([ri(cfg.n_path, cfg.e_pl), ri(cfg.n_link, cfg.e_pl)])
    ln = torch.stack([ri(cfg.n_link, cfg.e_ln), ri(cfg.n_node, cfg.e_ln)])
    ei: Dict[EdgeType, torch.Tensor] = {REL_PL: pl, REL_LP: pl.flip(0).contiguous(),
                                        REL_LN: ln, REL_NL: ln.flip(0).contiguous()}
    if cfg.e_pn:
        pn = torch.stack([ri(cfg.n_path, cfg.e_pn), ri(cfg.n_node, cfg.e_pn)])
        ei[REL_PN] = pn
        if cfg.with_np:
            ei[REL_NP] = pn.flip(0).contiguous()
    rn = lambda n, f: torch.randn(n, f, generator=g, device=device)  # noqa: E731
    x = {"path": rn(cfg.n_path, cfg.f_path), "link": rn(cfg.n_link, cfg.f_link),
         "node": rn(cfg.n_node, cfg.f_node)}
    if cfg.feat_dtype == "bf16":
        x = {t: v.to(torch.bfloat16) for t, v in x.items()}
    y = torch.rand(cfg.n_path, generator=g, device=device) + 0.5
    batch = {t: torch.zeros(x[t].shape[0], dtype=torch.long, device=device) for t in NODE_TYPES}
    return HeteroGraph(x, ei, y, batch)


def collate(graphs: List[HeteroGraph]) -> HeteroGraph:
    """PyG ``Batch.from_data_list`` for HeteroData (``dataset.py:239-244``), restated on dict-of-tensors.

    Node features concatenate per type in list order; every relation's ``edge_index[0]`` is offset by the
    running count of its src type and ``edge_index[1]`` by that of its dst type; ``batch[t]`` holds the
    graph index of every node.  Relations are kept in the first graph's insertion order.
    """
    if not graphs:
        raise ValueError("collate: empty list")
    types = list(graphs[0].x.keys())
    rels = list(graphs[0].edge_index.keys())
    inc = {t: 0 for t in types}
    xs = {t: [] for t in types}
    bs = {t: [] for t in types}
    es = {r: [] for r in rels}
    ys = []
    for gi, gr in enumerate(graphs):
        for r in rels:
            e = gr.edge_index[r]
            off = torch.tensor([[inc[r[0]]], [inc[r[2]]]], dtype=e.dtype, device=e.device)
            es[r].append(e + off)
        for t in types:
            n = gr.x[t].shape[0]
            xs[t].append(gr.x[t])
            bs[t].append(torch.full((n,), gi, dtype=torch.long, device=gr.x[t].device))
            inc[t] += n
        ys.append(gr.y)
    return HeteroGraph({t: torch.cat(xs[t]) for t in types}, {r: torch.cat(es[r], 1) for r in rels},
                       torch.cat(ys), {t: torch.cat(bs[t]) for t in types})


def component_graph(cfg: GraphConfig, n_components: int, seed: int = 0, device="cpu") -> HeteroGraph:
    """cfg split into ``n_components`` independent graphs, collated."""
    part = scaled_config(cfg, 1.0 / n_components, name=f"{cfg.name}/{n_components}")
    return collate([synthetic_graph(part, seed=seed + i, device=device) for i in range(n_components)])


def rank_components(cfg: GraphConfig, rank: int, world: int, device="cpu", n_components: Optional[int] = None
                    ) -> Tuple[HeteroGraph, List[int]]:
    """The components of ``cfg`` (generated as ``n_components`` equal independent graphs, default
    ``cfg.components``) that rank ``rank`` of ``world`` owns — a contiguous block of n / world components,
    component c always drawn from seed 1000 + c — collated into one batch.  The union over the ranks is the
    same graph for every world size, so N GPUs split ONE fixed workload (strong scaling)."""
    n = int(n_components or cfg.components)
    if n < 1 or n % world:
        raise ValueError(f"{n} components cannot be split evenly over {world} ranks")
    per = n // world
    ids = list(range(rank * per, (rank + 1) * per))
    import dataclasses
    part = dataclasses.replace(scaled_config(cfg, 1.0 / n, name=f"{cfg.name}/{n}"), components=1)
    return collate([synthetic_graph(part, seed=1000 + c, device=device) for c in ids]), ids
