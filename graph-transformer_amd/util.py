"""Drop-in replacement of U2GNN_pytorch/util.py for the graph-classification hot path.

``load_data`` reads the GIN text format (util.py:54-158) WITHOUT networkx: it keeps the
insertion-ordered adjacency networkx would build, so the edge order of ``edge_mat``
(g.edges() then reversed, util.py:131-136), self-loop handling, and the degree-as-tag
quirk (tags listed in networkx NODE-INSERTION order, util.py:140-142) are identical to the
reference.  ``separate_data`` / ``separate_data_idx`` keep the sklearn StratifiedKFold
split (util.py:160-186).  ``get_gm`` (pyriemann) is out of scope.
"""
import os

import numpy as np

DATASET_ROOT = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "dataset")


class S2VGraph(object):
    """util.py:18-34 (``g`` is replaced by the node count ``n``; ``len(graph.g)`` users use ``n``)."""

    def __init__(self, n, label, node_tags=None, node_features=None):
        self.label = label
        self.n = n
        self.node_tags = node_tags
        self.neighbors = []
        self.node_features = 0
        self.edge_mat = 0
        self.max_neighbor = 0


class _InsertionGraph:
    """The subset of networkx.Graph semantics load_data relies on."""

    def __init__(self):
        self.adj = {}

    def add_node(self, u):
        if u not in self.adj:
            self.adj[u] = {}

    def add_edge(self, u, v):
        self.add_node(u)
        self.add_node(v)
        self.adj[u][v] = None
        self.adj[v][u] = None

    def edges(self):
        seen = set()
        out = []
        for u, nb in self.adj.items():
            for v in nb:
                if v not in seen:
                    out.append((u, v))
            seen.add(u)
        return out

    def degrees(self):
        return [len(nb) + (1 if u in nb else 0) for u, nb in self.adj.items()]


def load_data(dataset, degree_as_tag, root=None):
    """util.py:54-158.  Returns (list of S2VGraph, number of classes)."""
    path = dataset if dataset.endswith(".txt") else os.path.join(root or DATASET_ROOT, dataset, dataset + ".txt")
    print('loading data')
    g_list = []
    label_dict = {}
    feat_dict = {}
    with open(path, 'r') as f:
        n_g = int(f.readline().strip())
        for _ in range(n_g):
            n, l = [int(w) for w in f.readline().strip().split()]
            if l not in label_dict:
                label_dict[l] = len(label_dict)
            g = _InsertionGraph()
            node_tags = []
            for j in range(n):
                g.add_node(j)
                row = f.readline().strip().split()
                tmp = int(row[1]) + 2
                row = [int(w) for w in row[:tmp]]
                if row[0] not in feat_dict:
                    feat_dict[row[0]] = len(feat_dict)
                node_tags.append(feat_dict[row[0]])
                for k in range(2, len(row)):
                    g.add_edge(j, row[k])
            assert len(g.adj) == n
            s = S2VGraph(n, l, node_tags)
            s._g = g
            g_list.append(s)

    for s in g_list:
        g = s._g
        s.label = label_dict[s.label]
        edges = [list(pair) for pair in g.edges()]
        s.neighbors = [[] for _ in range(s.n)]
        for i, j in edges:
            s.neighbors[i].append(j)
            s.neighbors[j].append(i)
        s.max_neighbor = max(len(x) for x in s.neighbors) if s.n else 0
        edges.extend([[i, j] for j, i in edges])
        s.edge_mat = np.transpose(np.array(edges, dtype=np.int32).reshape(-1, 2), (1, 0))
        s._deg = g.degrees()

    if degree_as_tag:
        for s in g_list:
            s.node_tags = list(s._deg)

    tagset = set([])
    for s in g_list:
        tagset = tagset.union(set(s.node_tags))
    tagset = list(tagset)
    tag2index = {tagset[i]: i for i in range(len(tagset))}
    for s in g_list:
        s.node_features = np.zeros((len(s.node_tags), len(tagset)), dtype=np.float32)
        s.node_features[range(len(s.node_tags)), [tag2index[tag] for tag in s.node_tags]] = 1
        del s._g, s._deg

    print('# classes: %d' % len(label_dict))
    print('# maximum node tag: %d' % len(tagset))
    print("# data: %d" % len(g_list))
    return g_list, len(label_dict)


def separate_data_idx(graph_list, fold_idx, seed=0):
    """util.py:176-186."""
    assert 0 <= fold_idx < 10, "fold_idx must be from 0 to 9."
    from sklearn.model_selection import StratifiedKFold
    skf = StratifiedKFold(n_splits=10, shuffle=True, random_state=seed)
    labels = [graph.label for graph in graph_list]
    idx_list = list(skf.split(np.zeros(len(labels)), labels))
    return idx_list[fold_idx]


def separate_data(graph_list, fold_idx, seed=0):
    """util.py:160-173."""
    train_idx, test_idx = separate_data_idx(graph_list, fold_idx, seed)
    return [graph_list[i] for i in train_idx], [graph_list[i] for i in test_idx]


class Namespace:
    def __init__(self, **kwargs):
        self.__dict__.update(kwargs)

    def update(self, **kwargs):
        self.__dict__.update(kwargs)
