"""Host batch assembly, vectorised and bit-exact with the reference's per-node Python loop.

Reference: get_batch_data / Batch_Loader (train_pytorch_U2GNN_Sup.py:58-126,
train_pytorch_U2GNN_UnSup.py:59-134).  The reference builds a dict of neighbour lists over
the concatenated edge_mat (forward edges then reversed, in file order) and draws
``np.random.choice(nbrs, k, replace=True)`` node by node from the global numpy stream.
``np.random.randint(0, deg[:, None], size=(n, k))`` consumes that stream identically (one
bounded draw per element, row-major; deg == 1 draws nothing in both), so the vectorised
version below yields the same ``input_x`` and leaves the stream in the same state.

``GraphStore`` precomputes, once per dataset, each graph's neighbour CSR in reference order,
so a batch costs O(N*k) work instead of a Python loop over every directed edge.  The production
path (``assemble``) runs that O(N*k) loop natively (csrc/batch_assembly.cpp, u2gnn_batch_assemble):
it continues numpy's MT19937 state in C++ exactly as the randint call below does, ~10x faster than
numpy's broadcast randint (which alone costs ~2 ms per 64-graph COLLAB batch, more than a GPU
step); ``assemble_numpy`` is the numpy form, kept as the readable statement and the test reference.
"""
from __future__ import annotations

import ctypes

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
    gnode: Optional[np.ndarray] = None     # int64 [N] dataset node id of each row (native assembly)
    pinned: Optional["PinnedSlot"] = None  # page-locked buffers the arrays above live in

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
        self.nbr = np.ascontiguousarray(np.concatenate(nbr_chunks) if nbr_chunks else np.zeros(0, dtype=np.int64),
                                        dtype=np.int64)   # local ids
        self.nbr_start = np.zeros(len(deg_all) + 1, dtype=np.int64)
        np.cumsum(deg_all, out=self.nbr_start[1:])
        self.d = self.X.shape[1]

    def degrees_of(self, ids) -> np.ndarray:
        return np.concatenate([self.deg[self.node_start[i]:self.node_start[i + 1]] for i in ids])

    def assemble(self, graph_ids: Sequence[int], num_neighbors: int, rng=np.random,
                 with_input_y: bool = False, gather_x: bool = True, out=None) -> HostBatch:
        """get_batch_data for the graphs ``graph_ids`` (in that order), natively (see module doc).
        gather_x=False leaves X_concat None and returns the rows' dataset node ids in ``gnode`` (the
        caller gathers the features on the GPU from a device-resident copy of ``X``).  out: a
        PinnedSlot whose page-locked buffers receive input_x / offsets / gnode / labels (no copy
        before the asynchronous H2D of DeviceBatch.from_store)."""
        from ._lib import lus_lib
        ids = np.ascontiguousarray(graph_ids, dtype=np.int64)
        st = rng.get_state()
        if st[0] != "MT19937":
            raise ValueError("the reference stream is numpy's legacy MT19937 RandomState")
        key = np.array(st[1], dtype=np.uint32)
        pos = ctypes.c_int32(int(st[2]))
        k = int(num_neighbors)
        N = int(self.n_nodes[ids].sum())
        if out is not None:
            out.wait()   # the slot's previous H2D copies are done
            offsets, input_x, gnode = out.views(len(ids), N, k)
            labels = out.labels_view(len(ids))
            np.take(self.labels, ids, out=labels)
        else:
            offsets = np.empty(len(ids) + 1, dtype=np.int64)
            input_x = np.empty((N, k + 1), dtype=np.int64)
            gnode = np.empty(N, dtype=np.int64)
            labels = self.labels[ids]
        p = lambda a: a.ctypes.data  # noqa: E731
        rc = lus_lib().u2gnn_batch_assemble(p(key), ctypes.byref(pos), p(ids), len(ids), p(self.n_nodes),
                                            p(self.node_start), p(self.deg), p(self.nbr_start), p(self.nbr), k, N,
                                            p(offsets), p(input_x), p(gnode))
        if rc != 0:
            raise ValueError(f"u2gnn_batch_assemble failed ({rc})")
        rng.set_state((st[0], key, pos.value, st[3], st[4]))
        X = self.X[gnode] if gather_x else None
        iy = (gnode if out is not None else gnode.copy()) if with_input_y else None
        hb = HostBatch(input_x, offsets, X, labels, ids, iy, gnode)
        hb.pinned = out
        return hb

    def assemble_numpy(self, graph_ids: Sequence[int], num_neighbors: int, rng=np.random,
                       with_input_y: bool = False) -> HostBatch:
        """get_batch_data for the graphs ``graph_ids`` (in that order), numpy form."""
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


class PinnedSlot:
    """Page-locked host buffers for one in-flight batch (input_x, offsets, gnode, labels) and the
    event recorded after their H2D copies; a ring of these lets the host assemble batch i+1 while
    the copies of batch i are still queued, without a synchronous pageable copy."""

    def __init__(self, max_rows: int, max_graphs: int, k: int):
        import torch
        self.ix = torch.empty(max_rows * (k + 1), dtype=torch.int64, pin_memory=True)
        self.gnode = torch.empty(max_rows, dtype=torch.int64, pin_memory=True)
        self.offsets = torch.empty(max_graphs + 1, dtype=torch.int64, pin_memory=True)
        self.labels = torch.empty(max_graphs, dtype=torch.int64, pin_memory=True)
        self.event = None

    def wait(self):
        if self.event is not None:
            self.event.synchronize()
            self.event = None

    def views(self, n_graphs: int, N: int, k: int):
        return (self.offsets.numpy()[:n_graphs + 1], self.ix.numpy()[:N * (k + 1)].reshape(N, k + 1),
                self.gnode.numpy()[:N])

    def labels_view(self, n_graphs: int):
        return self.labels.numpy()[:n_graphs]


class BatchLoader:
    """Batch_Loader of train_pytorch_U2GNN_Sup.py:120-126: a permutation of the (train) graph
    list from the global numpy stream, first batch_size of it, then get_batch_data."""

    def __init__(self, store: GraphStore, batch_size: int, num_neighbors: int, rng=np.random,
                 with_input_y: bool = False, gather_x: bool = True, native: bool = True):
        """gather_x=False: X_concat is left to the GPU (DeviceBatch.from_store); native=False: the
        numpy form of the assembly (measurements and tests)."""
        self.store, self.bs, self.k, self.rng, self.iy = store, batch_size, num_neighbors, rng, with_input_y
        self.gather_x, self.native = gather_x, native
        self.ring, self.slot = None, 0
        if not gather_x and native and isinstance(store, GraphStore):
            # batches bound for DeviceBatch.from_store are written straight into page-locked buffers
            max_rows = int(np.sort(store.n_nodes)[::-1][:batch_size].sum())
            self.ring = [PinnedSlot(max_rows, batch_size, num_neighbors) for _ in range(3)]

    def __call__(self) -> HostBatch:
        sel = self.rng.permutation(len(self.store.graphs))[:self.bs]
        if isinstance(self.store, GraphStore):
            if not self.native:
                return self.store.assemble_numpy(sel, self.k, self.rng, self.iy)
            out = None
            if self.ring is not None:
                out = self.ring[self.slot]
                self.slot = (self.slot + 1) % len(self.ring)
            return self.store.assemble(sel, self.k, self.rng, self.iy, gather_x=self.gather_x, out=out)
        return self.store.assemble(sel, self.k, self.rng, self.iy)

    def replay(self) -> None:
        """Consume exactly the numpy draws of one batch without building it (data-parallel
        ranks skip the batches of other ranks this way)."""
        sel = self.rng.permutation(len(self.store.graphs))[:self.bs]
        deg = self.store.degrees_of(sel)
        live = deg[deg > 0]
        if len(live):
            self.rng.randint(0, live[:, None], size=(len(live), self.k))
