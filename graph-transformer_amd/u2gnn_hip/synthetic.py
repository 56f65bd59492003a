"""Synthetic stand-ins for the datasets the container lacks (COLLAB, REDDITMULTI5K;
reference .MISSING_LARGE_BLOBS), shaped by their published statistics.

Graphs are generated lazily and deterministically per graph id (numpy default_rng([seed, gid])),
so a batch only materialises its own graphs.  The store exposes the GraphStore interface
used by BatchLoader (n_nodes, node_start, deg, labels, assemble).
"""
from __future__ import annotations

import numpy as np

from .batching import HostBatch


class SyntheticStore:
    def __init__(self, n_graphs: int, mean_nodes: float, min_nodes: int, max_nodes: int, avg_edges: float,
                 n_classes: int, d: int, seed: int = 0, dist: str = "gamma", feature: str = "degree_onehot"):
        rng = np.random.default_rng(seed)
        if dist == "gamma":
            base = rng.gamma(2.0, 1.0, size=n_graphs)
        else:
            base = rng.lognormal(0.0, 1.0, size=n_graphs)
        # scale so that the mean AFTER clipping equals the published mean (bisection)
        lo, hi = 1e-3, 10.0 * max_nodes
        for _ in range(60):
            mid = 0.5 * (lo + hi)
            if np.clip(np.round(base * mid), min_nodes, max_nodes).mean() < mean_nodes:
                lo = mid
            else:
                hi = mid
        self.n_nodes = np.clip(np.round(base * hi), min_nodes, max_nodes).astype(np.int64)
        self.node_start = np.zeros(n_graphs + 1, dtype=np.int64)
        np.cumsum(self.n_nodes, out=self.node_start[1:])
        self.labels = rng.integers(0, n_classes, size=n_graphs).astype(np.int64)
        pairs = (self.n_nodes * (self.n_nodes - 1) // 2).astype(np.float64)
        self.p_edge = min(1.0, avg_edges * n_graphs / max(pairs.sum(), 1.0))
        self.seed, self.d, self.feature = seed, d, feature
        self.graphs = range(n_graphs)   # len() for the permutation
        self._cache = {}

    def graph(self, gid: int):
        """(nbr CSR start [n+1], neighbour ids [2E], degree [n], features [n, d]) of graph gid.
        Edge order mimics load_data: forward upper-triangle edges, then the reversed ones."""
        c = self._cache.get(gid)
        if c is not None:
            return c
        n = int(self.n_nodes[gid])
        r = np.random.default_rng([self.seed, gid])
        iu, ju = np.triu_indices(n, 1)
        keep = r.random(len(iu)) < self.p_edge
        src = np.concatenate([iu[keep], ju[keep]])
        dst = np.concatenate([ju[keep], iu[keep]])
        order = np.argsort(src, kind="stable")
        nbr = dst[order].astype(np.int64)
        deg = np.bincount(src, minlength=n).astype(np.int64)
        start = np.zeros(n + 1, dtype=np.int64)
        np.cumsum(deg, out=start[1:])
        if self.feature == "degree_onehot":
            X = np.zeros((n, self.d), dtype=np.float32)
            X[np.arange(n), np.minimum(deg, self.d - 1)] = 1.0
        else:  # REDDIT: all tags equal -> tile(X, 4) * 0.01
            X = np.full((n, self.d), 0.01, dtype=np.float32)
        c = (start, nbr, deg, X)
        if len(self._cache) < 4096:
            self._cache[gid] = c
        return c

    def degrees_of(self, ids):
        return np.concatenate([self.graph(int(i))[2] for i in ids])

    def assemble(self, graph_ids, num_neighbors: int, rng=np.random, with_input_y: bool = False) -> HostBatch:
        ids = np.asarray(graph_ids, dtype=np.int64)
        parts = [self.graph(int(i)) for i in ids]
        sizes = self.n_nodes[ids]
        offsets = np.zeros(len(ids) + 1, dtype=np.int64)
        np.cumsum(sizes, out=offsets[1:])
        N = int(offsets[-1])
        k = num_neighbors
        X = np.concatenate([p[3] for p in parts], 0)
        deg = np.concatenate([p[2] for p in parts])
        ebase = np.concatenate([[0], np.cumsum([len(p[1]) for p in parts])])
        nbr_start = np.concatenate([p[0][:-1] + ebase[j] for j, p in enumerate(parts)])
        nbr = np.concatenate([p[1] for p in parts])
        input_x = np.repeat(np.arange(N, dtype=np.int64)[:, None], k + 1, axis=1)
        live = np.nonzero(deg > 0)[0]
        if len(live):
            draws = rng.randint(0, deg[live][:, None], size=(len(live), k))
            gpos = np.repeat(np.arange(len(ids)), sizes)[live]
            input_x[live, 1:] = nbr[nbr_start[live][:, None] + draws] + offsets[gpos][:, None]
        iy = None
        if with_input_y:
            iy = np.concatenate([np.arange(self.node_start[i], self.node_start[i + 1]) for i in ids])
        return HostBatch(input_x, offsets, X, self.labels[ids], ids, iy)


def collab_like(seed: int = 0) -> SyntheticStore:
    """COLLAB: 5000 graphs, 3 classes, mean 74.49 nodes in [32, 492], 2457.78 edges/graph,
    degree-as-tag one-hot over d = 367 tags."""
    return SyntheticStore(5000, 74.49, 32, 492, 2457.78, 3, 367, seed=seed, dist="gamma")


def reddit5k_like(seed: int = 0) -> SyntheticStore:
    """REDDITMULTI5K: 4999 graphs, 5 classes, mean 508.52 nodes in [22, 3648], 594.87 edges
    per graph, X = 0.01 * ones[n, 4]."""
    return SyntheticStore(4999, 508.52, 22, 3648, 594.87, 5, 4, seed=seed, dist="lognormal", feature="reddit")


class _Graph:
    """The attributes GraphStore reads from a util.S2VGraph."""

    def __init__(self, n, label, X, src, dst):
        self.n, self.label, self.node_features = n, label, X
        self.edge_mat = np.stack([src, dst])


def as_graph_store(s: "SyntheticStore"):
    """The same synthetic graphs as a GraphStore (the real-dataset path: native batch assembly into
    page-locked buffers, features gathered on the GPU) -- bench.py's on-the-fly pipeline line."""
    from .batching import GraphStore
    gs = []
    for gid in range(len(s.graphs)):
        start, nbr, deg, X = s.graph(gid)
        src = np.repeat(np.arange(len(deg)), deg)
        gs.append(_Graph(len(deg), int(s.labels[gid]), X, src, nbr))
    return GraphStore(gs)
