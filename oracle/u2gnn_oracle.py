"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference U2GNN hot path (shaginhekvs/Graph-Transformer,
PyTorch implementation).  Only tests/, __graft_entry__.smoke() and bench.py's
``cpu_baseline`` leg may import this module, and only as the checker / CPU
baseline — the product path (graph-transformer_amd/) never imports it and
fails loudly when its HIP library is missing.

What is restated (file:line relative to /root/reference):

* GIN-format loader                     U2GNN_pytorch/util.py:54-158
* stratified 10-fold split              U2GNN_pytorch/util.py:160-186
* batch assembly + neighbour sampling   U2GNN_pytorch/train_pytorch_U2GNN_Sup.py:58-126
                                        U2GNN_pytorch/train_pytorch_U2GNN_UnSup.py:59-134
* Sup model forward                     U2GNN_pytorch/pytorch_U2GNN_Sup.py:30-46
  (torch.nn.TransformerEncoderLayer post-LN semantics, nhead=1, ReLU, eps=1e-5,
   batch_first=False => sequence = all N nodes, batch = the k+1 slots)
* label smoothing / soft cross-entropy  pytorch_U2GNN_Sup.py:48-60, train_pytorch_U2GNN_Sup.py:140-142
* clip_grad_norm_(0.5) + Adam           train_pytorch_U2GNN_Sup.py:145,160-161 (torch semantics)
* sampled softmax                       U2GNN_pytorch/sampled_softmax.py:36-56
* UnSup composite (a12 of SURVEY §8)    pytorch_U2GNN_UnSup.py:52-69 + U2GNN_tf/model_U2GNN_Unsup_multi.py:43-58
* UnSup evaluation (§8(f) row 3)        train_pytorch_U2GNN_UnSup.py:82-94 (graph_pool over all graphs),
                                        :164-188 (spmm + 10-fold LogisticRegression(liblinear, tol=1e-3))

The model restatement computes ALL k+1 neighbour slots with dropout p=0.5 when
``train=True`` so that its cost is the reference's cost (used as the CPU
baseline); ``slots=1`` restricts to slot 0, which is exactly equal on outputs
 and is what parity tests use to stay fast.

Parity pins: tests/golden/*.npz produced by tests/golden/make_goldens.py from
the reference's own ``pytorch_U2GNN_Sup.TransformerU2GNN`` and
``sampled_softmax.SampledSoftmax`` (imported from /root/reference in the
survey container) and the reference C++ sampler built by
oracle/build_ref_sampler.sh.  The loader/batch assembly restatement is pinned
by the published dataset statistics only (the reference ``util.py`` imports
``pyriemann``, absent in the image; no stand-in is used) — see DESIGN.md.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field
from typing import Dict, List, Optional, Sequence

import numpy as np
import torch
import torch.nn.functional as F

# ----------------------------------------------------------------------------
# Loader  (util.py:54-158)
# ----------------------------------------------------------------------------


@dataclass
class OracleGraph:
    label: int
    n: int
    node_tags: list
    edges: list                 # networkx g.edges() order
    edge_mat: np.ndarray = None  # int32 [2, 2E]: forward edges then reversed (util.py:131-136)
    node_features: np.ndarray = None
    degrees: list = field(default_factory=list)


def load_data(path: str, degree_as_tag: bool):
    """util.py:54-158.  Uses networkx exactly like the reference so edge order,
    self-loop handling and degree-as-tag are identical."""
    import networkx as nx

    g_list = []
    label_dict: Dict[int, int] = {}
    feat_dict: Dict[int, int] = {}
    with open(path, "r") as f:
        n_g = int(f.readline().strip())
        for _ in range(n_g):
            row = f.readline().strip().split()
            n, l = [int(w) for w in row]
            if l not in label_dict:
                label_dict[l] = len(label_dict)
            g = nx.Graph()
            node_tags = []
            for j in range(n):
                g.add_node(j)
                row = f.readline().strip().split()
                tmp = int(row[1]) + 2
                if tmp == len(row):
                    row = [int(w) for w in row]
                else:
                    row = [int(w) for w in row[:tmp]]
                if row[0] not in feat_dict:
                    feat_dict[row[0]] = len(feat_dict)
                node_tags.append(feat_dict[row[0]])
                for k in range(2, len(row)):
                    g.add_edge(j, row[k])
            assert len(g) == n
            og = OracleGraph(label=l, n=n, node_tags=node_tags, edges=[])
            og._g = g
            g_list.append(og)

    for og in g_list:
        g = og._g
        og.label = label_dict[og.label]
        edges = [list(pair) for pair in g.edges()]
        edges.extend([[i, j] for j, i in edges])
        og.edges = edges
        og.edge_mat = np.transpose(np.array(edges, dtype=np.int32), (1, 0))
        og.degrees = list(dict(g.degree).values())

    if degree_as_tag:
        for og in g_list:
            og.node_tags = list(og.degrees)

    tagset = set([])
    for og in g_list:
        tagset = tagset.union(set(og.node_tags))
    tagset = list(tagset)
    tag2index = {tagset[i]: i for i in range(len(tagset))}
    for og in g_list:
        og.node_features = np.zeros((len(og.node_tags), len(tagset)), dtype=np.float32)
        og.node_features[range(len(og.node_tags)), [tag2index[t] for t in og.node_tags]] = 1
        del og._g
    return g_list, len(label_dict)


def separate_data_idx(labels: Sequence[int], fold_idx: int, seed: int = 0):
    """util.py:176-186 (sklearn StratifiedKFold(10, shuffle=True, random_state=seed))."""
    from sklearn.model_selection import StratifiedKFold

    skf = StratifiedKFold(n_splits=10, shuffle=True, random_state=seed)
    idx_list = list(skf.split(np.zeros(len(labels)), labels))
    return idx_list[fold_idx]


# ----------------------------------------------------------------------------
# Batch assembly, sequential  (train_pytorch_U2GNN_Sup.py:58-126)
# ----------------------------------------------------------------------------


def get_batch_data_seq(batch_graph, num_neighbors: int, reddit: bool = False,
                       feature_dim_size: Optional[int] = None, rng=np.random):
    """Per-node Python loop with the global numpy stream, like the reference.
    Returns (input_x int64[N,k+1], offsets int64[B+1], X_concat f32[N,d], labels int64[B])."""
    X_concat = np.concatenate([g.node_features for g in batch_graph], 0)
    if reddit:
        X_concat = np.tile(X_concat, feature_dim_size) * 0.01
    start = [0]
    for i, g in enumerate(batch_graph):
        start.append(start[i] + g.n)
    edge_mat = np.concatenate([g.edge_mat + start[i] for i, g in enumerate(batch_graph)], 1)
    rows, cols = edge_mat[0, :], edge_mat[1, :]
    adj: Dict[int, list] = {}
    for i in range(len(rows)):
        if rows[i] not in adj:
            adj[rows[i]] = []
        adj[rows[i]].append(cols[i])
    nbrs = []
    for u in range(X_concat.shape[0]):
        if u in adj:
            nbrs.append([u] + list(rng.choice(adj[u], num_neighbors, replace=True)))
        else:
            nbrs.append([u for _ in range(num_neighbors + 1)])
    input_x = np.array(nbrs, dtype=np.int64)
    labels = np.array([g.label for g in batch_graph], dtype=np.int64)
    return input_x, np.array(start, dtype=np.int64), X_concat.astype(np.float32), labels


def pool_matrix(offsets: np.ndarray) -> torch.Tensor:
    """Dense equivalent of get_graphpool (train_pytorch_U2GNN_Sup.py:73-89)."""
    B = len(offsets) - 1
    N = int(offsets[-1])
    P = torch.zeros(B, N)
    for b in range(B):
        P[b, offsets[b]:offsets[b + 1]] = 1.0
    return P


# ----------------------------------------------------------------------------
# Model  (pytorch_U2GNN_Sup.py:7-46 + torch TransformerEncoderLayer semantics)
# ----------------------------------------------------------------------------

def _drop(x, p, train, mask=None):
    if not train or p == 0.0:
        return x
    if mask is not None:
        return x * mask * (1.0 / (1.0 - p))
    return F.dropout(x, p, True)


def encoder_layer(x: torch.Tensor, prm: Dict[str, torch.Tensor], train: bool, p: float = 0.5,
                  masks: Optional[Dict[str, torch.Tensor]] = None) -> torch.Tensor:
    """One post-LN encoder layer on x[S, B, d] (S = nodes, B = neighbour slots).

    torch.nn.TransformerEncoderLayer(d, nhead=1, ff, dropout=0.5), norm_first=False,
    ReLU, layer_norm_eps=1e-5 (instantiated at pytorch_U2GNN_Sup.py:20).
    ``masks`` (optional, slot-0 only, shapes [S,S] / [S,d] / [S,ff]) replaces the random
    dropout masks of slot 0 for exact train-mode parity tests.  Test-only key ``"relu"`` ([S,ff] of 0/1):
    the ReLU's on/off decision of slot 0 taken from outside (a GPU run's), instead of the sign of the
    pre-activation -- the diagnostic that isolates ReLU boundary flips (tests/test_train_parity_gpu.py);
    test-only key ``"pre_out"`` (a list): slot 0's FFN pre-activations [S, ff] are appended to it."""
    S, B, d = x.shape
    W, b = prm["in_proj_weight"], prm["in_proj_bias"]
    qkv = x @ W.t() + b                                     # [S,B,3d]
    q, k, v = qkv[..., :d], qkv[..., d:2 * d], qkv[..., 2 * d:]
    q = q.permute(1, 0, 2)
    k = k.permute(1, 0, 2)
    v = v.permute(1, 0, 2)                                  # [B,S,d]
    scores = torch.bmm(q, k.transpose(1, 2)) / math.sqrt(d)  # head_dim = d (nhead=1)
    attn = torch.softmax(scores, dim=-1)
    if train and p > 0:
        if masks is not None:
            m = torch.ones_like(attn)
            m = torch.bernoulli(torch.full_like(attn, 1 - p)) if B > 1 else m
            m[0] = masks["attn"]
            attn = attn * m / (1 - p)
        else:
            attn = F.dropout(attn, p, True)
    o = torch.bmm(attn, v).permute(1, 0, 2)                 # [S,B,d]
    sa = o @ prm["out_proj.weight"].t() + prm["out_proj.bias"]

    def site_mask(name, like):
        if masks is None or not (train and p > 0):
            return None
        m = torch.bernoulli(torch.full_like(like, 1 - p)) if B > 1 else torch.ones_like(like)
        m[:, 0] = masks[name]
        return m

    x = F.layer_norm(x + _drop(sa, p, train, site_mask("drop1", sa)), (d,),
                     prm["norm1.weight"], prm["norm1.bias"], 1e-5)
    pre = x @ prm["linear1.weight"].t() + prm["linear1.bias"]
    if masks is not None and "pre_out" in masks:   # test-only: record slot 0's pre-activations [S, ff]
        masks["pre_out"].append(pre[:, 0].detach().clone())
    if masks is not None and "relu" in masks:
        on = (pre > 0).to(pre.dtype)
        on[:, 0] = masks["relu"]
        h = pre * on
    else:
        h = torch.relu(pre)
    h = _drop(h, p, train, site_mask("drop_ff", h))
    ff = h @ prm["linear2.weight"].t() + prm["linear2.bias"]
    x = F.layer_norm(x + _drop(ff, p, train, site_mask("drop2", ff)), (d,),
                     prm["norm2.weight"], prm["norm2.bias"], 1e-5)
    return x


def layer_params(sd: Dict[str, torch.Tensor], l: int, t: int) -> Dict[str, torch.Tensor]:
    pre = f"u2gnn_layers.{l}.layers.{t}."
    keys = ["self_attn.in_proj_weight", "self_attn.in_proj_bias", "self_attn.out_proj.weight",
            "self_attn.out_proj.bias", "linear1.weight", "linear1.bias", "linear2.weight",
            "linear2.bias", "norm1.weight", "norm1.bias", "norm2.weight", "norm2.bias"]
    out = {}
    for k in keys:
        out[k.replace("self_attn.", "")] = sd[pre + k]
    return out


def sup_forward(sd: Dict[str, torch.Tensor], input_x: torch.Tensor, offsets: np.ndarray,
                X_concat: torch.Tensor, num_layers: int, num_timesteps: int, train: bool,
                dropout: float = 0.5, slots: Optional[int] = None,
                masks: Optional[dict] = None, attention: str = "nodes") -> torch.Tensor:
    """pytorch_U2GNN_Sup.py:30-46.  ``sd`` uses the reference state_dict keys.
    ``masks[(l, t)]`` feeds encoder_layer; ``masks[('head', l)]`` is the [B,d] mask of
    the graph-embedding dropout (pytorch_U2GNN_Sup.py:42).
    attention="neighbors": the paper semantics (U2GNN_tf/model_U2GNN_Sup_multi.py:14-45) restated
    on the same torch encoder by feeding the gathered window transposed, [k+1, N, d], so each node
    attends over its own k+1 tokens (no TF oracle here, parity of this mode is
    unpinned by the reference)."""
    if slots is not None:
        input_x = input_x[:, :slots]
    P = pool_matrix(offsets).to(X_concat.dtype)
    scores = 0
    inp = F.embedding(input_x, X_concat)                   # [N, k+1, d]
    nb = attention == "neighbors"
    for l in range(num_layers):
        x = inp.transpose(0, 1) if nb else inp
        for t in range(num_timesteps):
            x = encoder_layer(x, layer_params(sd, l, t), train, 0.5,
                              None if masks is None else masks[(l, t)])
        out = x[0] if nb else x[:, 0, :]                  # slot 0
        inp = F.embedding(input_x, out)
        ge = P @ out
        hm = None if masks is None else masks.get(("head", l))
        ge = _drop(ge, dropout, train, hm)
        scores = scores + ge @ sd[f"predictions.{l}.weight"].t() + sd[f"predictions.{l}.bias"]
    return scores


def label_smoothing(labels: torch.Tensor, classes: int, smoothing: float = 0.1) -> torch.Tensor:
    """pytorch_U2GNN_Sup.py:48-60."""
    t = torch.full((labels.shape[0], classes), smoothing / (classes - 1))
    t.scatter_(1, labels.view(-1, 1), 1.0 - smoothing)
    return t


def soft_cross_entropy(pred: torch.Tensor, soft_targets: torch.Tensor) -> torch.Tensor:
    """train_pytorch_U2GNN_Sup.py:140-142."""
    return torch.mean(torch.sum(-soft_targets * torch.log_softmax(pred, dim=1), 1))


def clip_and_adam(params: List[torch.Tensor], grads: List[torch.Tensor], state: dict, lr: float,
                  max_norm: float = 0.5, betas=(0.9, 0.999), eps: float = 1e-8):
    """torch.nn.utils.clip_grad_norm_(max_norm) followed by torch.optim.Adam.step()
    (defaults: no weight decay, no amsgrad).  In-place on params; state holds m, v, step."""
    total = torch.norm(torch.stack([torch.norm(g.double(), 2) for g in grads]), 2)
    coef = min(1.0, max_norm / (float(total) + 1e-6))
    state["step"] = state.get("step", 0) + 1
    step = state["step"]
    bc1 = 1 - betas[0] ** step
    bc2 = 1 - betas[1] ** step
    for i, (p, g) in enumerate(zip(params, grads)):
        g = g * coef
        m = state.setdefault(("m", i), torch.zeros_like(p))
        v = state.setdefault(("v", i), torch.zeros_like(p))
        m.mul_(betas[0]).add_(g, alpha=1 - betas[0])
        v.mul_(betas[1]).addcmul_(g, g, value=1 - betas[1])
        denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
        p.addcdiv_(m, denom, value=-lr / bc1)
    return float(total)


# ----------------------------------------------------------------------------
# Sampled softmax  (sampled_softmax.py:36-56)  and the UnSup composite (a12)
# ----------------------------------------------------------------------------

def sampled_softmax_logits(inputs: torch.Tensor, labels: torch.Tensor, weight: torch.Tensor,
                           sample_ids: torch.Tensor) -> torch.Tensor:
    """-log(exp(x.w_y) / sum_s exp(x.w_s)), exactly the reference expression (no max
    subtraction, no logQ correction, no accidental-hit removal)."""
    tw = weight.index_select(0, labels)
    sw = weight.index_select(0, sample_ids)
    true_logits = torch.exp(torch.sum(inputs * tw, dim=1))
    sample_logits = torch.exp(inputs @ sw.t())
    return -torch.log(true_logits / torch.sum(sample_logits, dim=1))


def unsup_forward(sd: Dict[str, torch.Tensor], weight: torch.Tensor, input_x: torch.Tensor,
                  X_concat: torch.Tensor, input_y: torch.Tensor, sample_ids: torch.Tensor,
                  num_layers: int, num_timesteps: int, train: bool, dropout: float = 0.5,
                  slots: Optional[int] = None, masks: Optional[dict] = None) -> torch.Tensor:
    """UnSup composite: per-layer slot-0 outputs concatenated to [N, d*L] -> dropout ->
    SampledSoftmax; loss = sum of logits (train_pytorch_U2GNN_UnSup.py:155-156)."""
    if slots is not None:
        input_x = input_x[:, :slots]
    inp = F.embedding(input_x, X_concat)
    outs = []
    for l in range(num_layers):
        x = inp
        for t in range(num_timesteps):
            x = encoder_layer(x, layer_params(sd, l, t), train, 0.5,
                              None if masks is None else masks[(l, t)])
        out = x[:, 0, :]
        outs.append(out)
        inp = F.embedding(input_x, out)
    ov = torch.cat(outs, dim=1)
    hm = None if masks is None else masks.get("ss")
    ov = _drop(ov, dropout, train, hm)
    return sampled_softmax_logits(ov, input_y, weight, sample_ids)


# ----------------------------------------------------------------------------
# UnSup evaluation  (train_pytorch_U2GNN_UnSup.py:82-94, 164-188)
# ----------------------------------------------------------------------------

def unsup_evaluate(weight: torch.Tensor, n_nodes: Sequence[int], labels: Sequence[int], seed: int = 0):
    """evaluate(): graph_pool = sparse [G, V] of ones over every graph's nodes (get_graphpool over ALL
    graphs, nodes contiguous in dataset order); graph embeddings = torch.spmm(graph_pool, ss.weight);
    per fold of separate_data_idx (StratifiedKFold(10, shuffle, seed 0)) a
    LogisticRegression(solver="liblinear", tol=0.001) fit on the train graphs, scored on the test
    graphs.  Returns the 10 accuracies (mean / stdev are statistics.mean / statistics.stdev of them)."""
    from sklearn.linear_model import LogisticRegression
    n_nodes = np.asarray(n_nodes, dtype=np.int64)
    start = np.concatenate([[0], np.cumsum(n_nodes)])
    rows = np.repeat(np.arange(len(n_nodes)), n_nodes)
    idx = torch.from_numpy(np.stack([rows, np.arange(int(start[-1]))]))
    graph_pool = torch.sparse_coo_tensor(idx, torch.ones(int(start[-1])), (len(n_nodes), int(start[-1])))
    emb = torch.spmm(graph_pool, weight.float()).numpy()
    labels = np.asarray(labels)
    accs = []
    for fold in range(10):
        tr, te = separate_data_idx(labels, fold)
        cls = LogisticRegression(solver="liblinear", tol=0.001)
        cls.fit(emb[tr], labels[tr])
        accs.append(float(cls.score(emb[te], labels[te])))
    return accs
