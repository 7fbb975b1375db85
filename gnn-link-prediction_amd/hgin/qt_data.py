"""Synthetic RouteNet-style homogeneous samples for the queueing-theory baseline (§8 F4).

The reference builds, per simulation, a networkx DiGraph whose vertices are network nodes ``n_i``, links
``l_i_j`` and paths (flows) ``p_s_d_f`` (``generateFiles.py:26-101``), converts it with
``from_networkx`` (``generateFiles.py:183-231``) and keeps the homogeneous ``edge_index`` (edges in the
graph's adjacency order: by source vertex in insertion order, then successors in insertion order), a
per-edge ``edge_type`` (0: path<->link, 1: path<->node, 2: node<->link) and a per-vertex ``type``
(0 path, 1 link, 2 node, ``generateFiles.py:213-221``).  ``QTBaseline`` (``models.py:42-158``) reads
``edge_index``, ``edge_type``, ``type``, ``P`` (path features [n_paths, 3]: AvgPktsLambda, PktsGen,
AvgBw / 1000, ``dataset.py:66-73``) and ``L`` (link capacity [n_links, 1], ``dataset.py:85``).

This module generates such samples without networkx or the dataset: a random strongly connected topology,
shortest-path routes, one flow per ordered node pair, with the same vertex / edge insertion rules, so the
edge order (which QTBaseline's per-position grouping depends on) has the reference's structure.
"""
from __future__ import annotations

from collections import deque
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np
import torch


@dataclass
class RouteSample:
    edge_index: torch.Tensor   # int64 [2, E]
    edge_type: torch.Tensor    # int64 [E]
    type: torch.Tensor         # int64 [N]
    P: torch.Tensor            # float32 [n_paths, 3]
    L: torch.Tensor            # float32 [n_links, 1]

    @property
    def num_nodes(self) -> int:
        return int(self.type.numel())


class _OrderedDiGraph:
    """Insertion-ordered adjacency (what networkx.DiGraph iteration order amounts to)."""

    def __init__(self):
        self.succ: Dict[str, Dict[str, int]] = {}

    def add_node(self, v: str) -> None:
        self.succ.setdefault(v, {})

    def add_edge(self, u: str, v: str, edge_type: int) -> None:
        self.add_node(u)
        self.add_node(v)
        self.succ[u][v] = edge_type     # re-adding keeps the original position (attribute update)

    def has_succ(self, u: str, v: str) -> bool:
        return v in self.succ.get(u, {})


def _topology(n: int, rng: np.random.Generator) -> List[Tuple[int, int]]:
    """Bidirectional ring + random bidirectional chords (strongly connected)."""
    edges = set()
    for i in range(n):
        edges.add((i, (i + 1) % n))
        edges.add(((i + 1) % n, i))
    for _ in range(n):
        a, b = rng.integers(0, n, 2)
        if a != b:
            edges.add((int(a), int(b)))
            edges.add((int(b), int(a)))
    return sorted(edges)


def _routes(n: int, edges: List[Tuple[int, int]]) -> Dict[Tuple[int, int], List[int]]:
    adj: Dict[int, List[int]] = {i: [] for i in range(n)}
    for a, b in edges:
        adj[a].append(b)
    routes = {}
    for s in range(n):
        prev = {s: -1}
        q = deque([s])
        while q:
            u = q.popleft()
            for v in adj[u]:
                if v not in prev:
                    prev[v] = u
                    q.append(v)
        for d in range(n):
            if d != s:
                path, v = [], d
                while v != -1:
                    path.append(v)
                    v = prev[v]
                routes[(s, d)] = path[::-1]
    return routes


def route_sample(n_nodes: int = 10, seed: int = 0, flows_per_pair: int = 1) -> RouteSample:
    """One simulation-shaped sample with ``n_nodes`` network nodes (paths = flows_per_pair * n(n-1))."""
    rng = np.random.default_rng(seed)
    topo = _topology(n_nodes, rng)
    topo_set = set(topo)
    routes = _routes(n_nodes, topo)
    g = _OrderedDiGraph()
    cap: Dict[str, float] = {}
    pfeat: Dict[str, Tuple[float, float, float]] = {}
    for i in range(n_nodes):                                   # generateFiles.py:32-34
        g.add_node(f"n_{i}")
    for s in range(n_nodes):                                   # generateFiles.py:36-78
        for d in range(n_nodes):
            if s == d:
                continue
            if (s, d) in topo_set:
                lname = f"l_{s}_{d}"
                g.add_node(lname)
                cap[lname] = float(rng.choice([10000.0, 25000.0, 40000.0, 100000.0]))
                g.add_edge(f"n_{s}", lname, 2)
                g.add_edge(lname, f"n_{d}", 2)
            for f in range(flows_per_pair):
                pname = f"p_{s}_{d}_{f}"
                g.add_node(pname)
                # packets/s and bits/s / 1000 at the GNNet scale: link loads rho = T / (capacity / 1000)
                # land around 0.1-1 (dataset.py:68-73, models.py:75-77)
                lam = float(rng.uniform(0.05, 1.0))
                pfeat[pname] = (lam, lam * float(rng.uniform(0.9, 1.1)), float(rng.uniform(0.1, 1.5)))
                r = routes[(s, d)]
                for h1, h2 in zip(r[:-1], r[1:]):
                    n1, n2, lk = f"n_{h1}", f"n_{h2}", f"l_{h1}_{h2}"
                    if not g.has_succ(pname, n1):
                        g.add_edge(pname, n1, 1)
                        g.add_edge(n1, pname, 1)
                    if not g.has_succ(pname, n2):
                        g.add_edge(pname, n2, 1)
                        g.add_edge(n2, pname, 1)
                    g.add_edge(pname, lk, 0)
                    g.add_edge(lk, pname, 0)
    names = list(g.succ.keys())                                 # convert_node_labels_to_integers order
    idx = {v: i for i, v in enumerate(names)}
    src, dst, et = [], [], []
    for u in names:
        for v, t in g.succ[u].items():
            src.append(idx[u])
            dst.append(idx[v])
            et.append(t)
    vtype = [0 if v[0] == "p" else (1 if v[0] == "l" else 2) for v in names]
    P = [pfeat[v] for v in names if v[0] == "p"]
    L = [[cap[v]] for v in names if v[0] == "l"]
    return RouteSample(torch.tensor([src, dst], dtype=torch.long), torch.tensor(et, dtype=torch.long),
                       torch.tensor(vtype, dtype=torch.long), torch.tensor(P, dtype=torch.float32),
                       torch.tensor(L, dtype=torch.float32))


def collate_routes(samples: List[RouteSample]) -> RouteSample:
    """Disjoint union (ids offset per sample), as PyG's Batch of homogeneous Data does."""
    off = 0
    ei, et, ty, P, L = [], [], [], [], []
    for s in samples:
        ei.append(s.edge_index + off)
        et.append(s.edge_type)
        ty.append(s.type)
        P.append(s.P)
        L.append(s.L)
        off += s.num_nodes
    return RouteSample(torch.cat(ei, 1), torch.cat(et), torch.cat(ty), torch.cat(P), torch.cat(L))
