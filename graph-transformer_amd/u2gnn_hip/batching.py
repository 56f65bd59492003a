"""Host batch assembly, vectorised and bit-exact with the reference's per-node Python loop.

Reference: get_batch_data / Batch_Loader (train_pytorch_U2GNN_Sup.py:58-126,
train_pytorch_U2GNN_UnSup.py:59-134).  The reference builds a dict of neighbour lists over
the concatenated edge_mat (forward edges then reversed, in file order) and draws
``np.random.choice(nbrs, k, replace=True)`` node by node from the global numpy stream.
``np.random.randint(0, deg[:, None], size=(n, k))`` consumes that stream identically (one
bounded draw per element, row-major; deg == 1 draws nothing in both), so the vectorised
version below yields the same ``input_x`` and leaves the stream in the same state.

``GraphStore`` precomputes, once per dataset, each graph's neighbour CSR in reference order,
so a batch costs O(N*k) numpy work instead of a Python loop over every directed edge.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import List, Optional, Sequence

import numpy as np


@dataclass
class HostBatch:
    input_x: np.ndarray      # int64 [N, k+1]
    offsets: np.ndarray      # int64 [B+1]
    X_concat: np.ndarray     # f32 [N, d]
    labels: np.ndarray       # int64 [B]
    graph_ids: np.ndarray    # int64 [B] (indices into the store's graph list)
    input_y: Optional[np.ndarray] = None   # int64 [N] global node ids (UnSup)

    @property
    def N(self):
        return int(self.offsets[-1])


class GraphStore:
    """Per-dataset arrays: node features, labels, neighbour CSR in the reference's order."""

    def __init__(self, graphs: Sequence, reddit_tile: int = 0):
        self.graphs = list(graphs)
        n = np.array([g.n if hasattr(g, "n") else len(g.g) for g in self.graphs], dtype=np.int64)
        self.n_nodes = n
        self.node_start = np.zeros(len(n) + 1, dtype=np.int64)
        np.cumsum(n, out=self.node_start[1:])
        self.labels = np.array([g.label for g in self.graphs], dtype=np.int64)
        feats = np.concatenate([g.node_features for g in self.graphs], 0).astype(np.float32)
        if reddit_tile:
            # train_pytorch_U2GNN_Sup.py:93-95 (REDDIT*): tile to 4 columns, scale 0.01
            feats = (np.tile(feats, reddit_tile) * 0.01).astype(np.float32)
        self.X = feats
        # neighbour lists: stable sort of each graph's edge_mat by source keeps file order
        deg_all = np.zeros(int(self.node_start[-1]), dtype=np.int64)
        nbr_chunks = []
        for gi, g in enumerate(self.graphs):
            em = np.asarray(g.edge_mat, dtype=np.int64).reshape(2, -1)
            if em.shape[1] == 0:
                nbr_chunks.append(np.zeros(0, dtype=np.int64))
                continue
            order = np.argsort(em[0], kind="stable")
            nbr_chunks.append(em[1][order])
            deg_all[self.node_start[gi]:self.node_start[gi + 1]] = np.bincount(em[0], minlength=int(n[gi]))
        self.deg = deg_all
        self.nbr = np.concatenate(nbr_chunks) if nbr_chunks else np.zeros(0, dtype=np.int64)  # local ids
        self.nbr_start = np.zeros(len(deg_all) + 1, dtype=np.int64)
        np.cumsum(deg_all, out=self.nbr_start[1:])
        self.d = self.X.shape[1]

    def degrees_of(self, ids) -> np.ndarray:
        return np.concatenate([self.deg[self.node_start[i]:self.node_start[i + 1]] for i in ids])

    def assemble(self, graph_ids: Sequence[int], num_neighbors: int, rng=np.random,
                 with_input_y: bool = False) -> HostBatch:
        """get_batch_data for the graphs ``graph_ids`` (in that order)."""
        ids = np.asarray(graph_ids, dtype=np.int64)
        sizes = self.n_nodes[ids]
        offsets = np.zeros(len(ids) + 1, dtype=np.int64)
        np.cumsum(sizes, out=offsets[1:])
        N = int(offsets[-1])
        # global node ids of the batch nodes (contiguous per graph)
        gnode = np.concatenate([np.arange(self.node_start[i], self.node_start[i + 1]) for i in ids]) if N else \
            np.zeros(0, dtype=np.int64)
        X = self.X[gnode]
        deg = self.deg[gnode]
        k = num_neighbors
        input_x = np.repeat(np.arange(N, dtype=np.int64)[:, None], k + 1, axis=1)
        live = np.nonzero(deg > 0)[0]
        if len(live):
            draws = rng.randint(0, deg[live][:, None], size=(len(live), k))
            base = self.nbr_start[gnode[live]]
            local = self.nbr[base[:, None] + draws]                 # neighbour id within its graph
            gpos = np.repeat(np.arange(len(ids)), sizes)[live]      # batch graph index of each node
            input_x[live, 1:] = local + offsets[gpos][:, None]
        iy = gnode.copy() if with_input_y else None
        return HostBatch(input_x, offsets, X, self.labels[ids], ids, iy)


class BatchLoader:
    """Batch_Loader of train_pytorch_U2GNN_Sup.py:120-126: a permutation of the (train) graph
    list from the global numpy stream, first batch_size of it, then get_batch_data."""

    def __init__(self, store: GraphStore, batch_size: int, num_neighbors: int, rng=np.random,
                 with_input_y: bool = False):
        self.store, self.bs, self.k, self.rng, self.iy = store, batch_size, num_neighbors, rng, with_input_y

    def __call__(self) -> HostBatch:
        sel = self.rng.permutation(len(self.store.graphs))[:self.bs]
        return self.store.assemble(sel, self.k, self.rng, self.iy)

    def replay(self) -> None:
        """Consume exactly the numpy draws of one batch without building it (data-parallel
        ranks skip the batches of other ranks this way)."""
        sel = self.rng.permutation(len(self.store.graphs))[:self.bs]
        deg = self.store.degrees_of(sel)
        live = deg[deg > 0]
        if len(live):
            self.rng.randint(0, live[:, None], size=(len(live), self.k))
