"""Host batch-assembly cost on the C4 COLLAB-like set through the real-dataset path (GraphStore built
from the synthetic graphs): per-batch milliseconds of BatchLoader and of the prefetching loader.
Usage: python tools/loader_bench.py [batches]"""
import os
import sys
import time

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import numpy as np  # noqa: E402

from u2gnn_hip.batching import BatchLoader, GraphStore  # noqa: E402
from u2gnn_hip.synthetic import collab_like  # noqa: E402


class _G:
    def __init__(self, n, label, X, src, dst):
        self.n, self.label, self.node_features = n, label, X
        self.edge_mat = np.stack([src, dst])


def collab_store():
    s = collab_like(seed=0)
    gs = []
    for gid in range(len(s.graphs)):
        start, nbr, deg, X = s.graph(gid)
        src = np.repeat(np.arange(len(deg)), deg)
        gs.append(_G(len(deg), int(s.labels[gid]), X, src, nbr))
    return GraphStore(gs)


def main():
    nb = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    t = time.perf_counter()
    store = collab_store()
    print(f"store build {time.perf_counter() - t:.1f} s", flush=True)
    np.random.seed(123)
    L = BatchLoader(store, 64, 16)
    L()
    t = time.perf_counter()
    for _ in range(nb):
        L()
    print(f"BatchLoader: {(time.perf_counter() - t) / nb * 1e3:.2f} ms/batch", flush=True)


if __name__ == "__main__":
    main()
