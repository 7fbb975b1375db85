"""ORACLE — test infrastructure only.  numpy restatement of PyG 2.0.x ``Batch.from_data_list`` for the
reference's ``HeteroData`` graphs (what ``torch_geometric.loader.DataLoader`` / ``Collater`` does at
``dataset.py:239-244``; consumed at ``train.py:25-28``).

Only ``tests/`` may import it.  It is written independently of the product's ``hgin.data.collate`` (a
per-graph loop) and of ``hgin.store.GraphStore.collate`` (device descriptors): this one is vectorised over
the whole batch, the way PyG 2.0.x's ``torch_geometric/data/collate.py`` states the rule (PyG is not
installed and cannot be fetched; restated from its published algorithm):

* every node-level attribute of a node type (``x``, ``y``) is concatenated along dim 0 in list order
  (``__cat_dim__`` = 0);
* ``edge_index`` of a relation ``(src, rel, dst)`` is concatenated along dim -1 (``__cat_dim__`` = -1 for
  keys containing ``index``) after adding the increment ``__inc__`` = ``[[num_nodes(src)], [num_nodes(dst)]]``
  cumulated over the PRECEDING graphs (``incs = cumsum([0] + inc[:-1])``);
* ``batch`` of a node type = ``repeat_interleave(arange(num_graphs), num_nodes)``; relation order and node-type
  order are those of the first graph (``HeteroData`` keeps insertion order, ``dataset.py:89-117``).

Inputs are dicts of numpy arrays: ``{"x": {type: [n, F]}, "edge_index": {rel: [2, E] int64}, "y": [n_path]}``.
"""
from __future__ import annotations

from typing import Dict, List

import numpy as np


def collate(graphs: List[dict]) -> dict:
    if not graphs:
        raise ValueError("empty data list")
    types = list(graphs[0]["x"].keys())
    rels = list(graphs[0]["edge_index"].keys())
    n_nodes = {t: np.array([g["x"][t].shape[0] for g in graphs], np.int64) for t in types}
    # increments of the graphs BEFORE each graph (exclusive cumulative sum)
    incs = {t: np.concatenate([[0], np.cumsum(n_nodes[t])[:-1]]).astype(np.int64) for t in types}
    out_x = {t: np.concatenate([g["x"][t] for g in graphs], 0) for t in types}
    out_batch = {t: np.repeat(np.arange(len(graphs), dtype=np.int64), n_nodes[t]) for t in types}
    out_e: Dict[tuple, np.ndarray] = {}
    for r in rels:
        src, _, dst = r
        counts = np.array([g["edge_index"][r].shape[1] for g in graphs], np.int64)
        cat = np.concatenate([g["edge_index"][r] for g in graphs], 1).astype(np.int64) if counts.sum() else \
            np.zeros((2, 0), np.int64)
        shift = np.stack([np.repeat(incs[src], counts), np.repeat(incs[dst], counts)])
        out_e[r] = cat + shift
    out_y = np.concatenate([g["y"] for g in graphs], 0)
    return {"x": out_x, "edge_index": out_e, "y": out_y, "batch": out_batch}


def from_graph(g) -> dict:
    """A hgin.data.HeteroGraph (CPU tensors) as the numpy dicts this module takes."""
    return {"x": {t: v.numpy() for t, v in g.x.items()},
            "edge_index": {r: e.numpy() for r, e in g.edge_index.items()}, "y": g.y.numpy()}
