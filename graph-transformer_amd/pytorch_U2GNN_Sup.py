"""Drop-in replacement of U2GNN_pytorch/pytorch_U2GNN_Sup.py on MI355X.

Same class name, constructor, ``forward(input_x, graph_pool, X_concat)`` signature,
parameter construction order (so ``torch.manual_seed`` gives identical initial weights) and
state_dict keys as the reference (pytorch_U2GNN_Sup.py:7-46).  The torch.nn encoder modules
are only parameter containers here: the computation runs on the gfx950 kernels of
libu2gnn_hip.so through ``u2gnn_hip.core.SupCore`` (no CPU fallback — the forward raises if
the HIP library or a GPU is missing).

Extra keywords (not in the reference): ``precision`` = "fp32" (exact fp32 matrix cores,
the parity path), "bf16x3" (split-bf16, ~2^-16 per product), "mixed" (bf16x3 with the
attention-backward products dS, dQ, dK on plain bf16; an experiment, see
u2gnn_hip.engine.MIXED_BF16_ROLES), "fwd32" (exact fp32 forward products, bf16x3 backward: the
forward's ReLU decisions carry fp32 rounding only), "fwd6" (the forward products on the
three-plane bf16x6 split -- fp32-accurate products on bf16 matrix cores -- bf16x3 backward) or "bf16" (experiments
only); ``attention`` = "nodes" (the fork's semantics: the encoder's sequence axis is
the node axis, pytorch_U2GNN_Sup.py:35) or "neighbors" (the paper / TF semantics: each node
attends over its own k+1 sampled neighbours, U2GNN_tf/model_U2GNN_Sup_multi.py:14-45).
"""
import torch
import torch.nn as nn
from torch.nn import TransformerEncoder, TransformerEncoderLayer

from u2gnn_hip.core import DeviceBatch, FlatParams, SupCore


class _SupFunction(torch.autograd.Function):
    @staticmethod
    def forward(fctx, core, batch, train, seed, names, *params):
        scores, ctx = core.forward(batch, train, need_ctx=True, seed=seed)
        fctx.core, fctx.ctx, fctx.names, fctx.params = core, ctx, names, params
        return scores

    @staticmethod
    def backward(fctx, dscores):
        params = fctx.params
        grads = {n: torch.empty_like(p) for n, p in zip(fctx.names, params)}
        fctx.core.backward(fctx.ctx, dscores.contiguous(), grads)
        fctx.ctx = None
        return (None, None, None, None, None) + tuple(grads[n] for n in fctx.names)


class TransformerU2GNN(nn.Module):

    def __init__(self, feature_dim_size, ff_hidden_size, num_classes,
                 num_self_att_layers, dropout, num_U2GNN_layers, precision="fp32", attention="nodes"):
        super(TransformerU2GNN, self).__init__()
        self.feature_dim_size = feature_dim_size
        self.ff_hidden_size = ff_hidden_size
        self.num_classes = num_classes
        self.num_self_att_layers = num_self_att_layers
        self.num_U2GNN_layers = num_U2GNN_layers
        self.dropout_p = dropout
        self.precision = precision
        if attention not in ("nodes", "neighbors"):
            raise ValueError(f"attention must be 'nodes' or 'neighbors', got {attention!r}")
        self.attention = attention
        # parameter containers built in the reference's order (identical init under a seed)
        self.u2gnn_layers = torch.nn.ModuleList()
        for _ in range(self.num_U2GNN_layers):
            encoder_layers = TransformerEncoderLayer(d_model=self.feature_dim_size, nhead=1,
                                                     dim_feedforward=self.ff_hidden_size, dropout=0.5)
            self.u2gnn_layers.append(TransformerEncoder(encoder_layers, self.num_self_att_layers,
                                                        enable_nested_tensor=False))
        self.predictions = torch.nn.ModuleList()
        self.dropouts = torch.nn.ModuleList()
        for _ in range(self.num_U2GNN_layers):
            self.predictions.append(nn.Linear(self.feature_dim_size, self.num_classes))
            self.dropouts.append(nn.Dropout(dropout))
        self._core = None

    @property
    def core(self) -> SupCore:
        if self._core is None:
            self._core = SupCore(self, self.precision)
        return self._core

    def flatten_parameters(self) -> FlatParams:
        """Move all parameters into one flat device buffer (for the fused clip+Adam)."""
        return FlatParams(self)

    def forward(self, input_x, graph_pool, X_concat):
        if isinstance(input_x, DeviceBatch):
            batch = input_x
        else:
            batch = DeviceBatch.from_reference_inputs(input_x, graph_pool, X_concat)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self.training else 0
        if torch.is_grad_enabled() and any(p.requires_grad for p in self.parameters()):
            names, params = zip(*self.named_parameters())
            return _SupFunction.apply(self.core, batch, self.training, seed, names, *params)
        scores, _ = self.core.forward(batch, self.training, need_ctx=False, seed=seed)
        return scores


def label_smoothing(true_labels: torch.Tensor, classes: int, smoothing=0.1):
    """pytorch_U2GNN_Sup.py:48-60: confidence 1-smoothing on the true class,
    smoothing/(classes-1) elsewhere."""
    assert 0 <= smoothing < 1
    true_dist = torch.full((true_labels.size(0), classes), smoothing / (classes - 1), device=true_labels.device)
    true_dist.scatter_(1, true_labels.data.unsqueeze(1), 1.0 - smoothing)
    return true_dist
