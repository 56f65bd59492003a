"""Drop-in replacement of U2GNN_pytorch/pytorch_U2GNN_UnSup.py on MI355X.

Constructor and forward signature of the fork (pytorch_U2GNN_UnSup.py:14-15, :52):
``TransformerU2GNN(vocab_size, feature_dim_size, ff_hidden_size, sampled_num, num_self_att_layers,
num_U2GNN_layers, dropout, device, sampler_type='default', loss_type='default', adj_mat=None,
single_layer_only=True)`` and ``forward(X_concat, input_x, input_y, args=None) -> (logits, weight)``.

The shipped fork cannot run (NameError on SampledSoftmax, a [vocab,d]*[N,d] product, a 3-D tensor
into SampledSoftmax — SURVEY.md §0.3).  This module implements its working semantics, which are
also the original U2GNN's (U2GNN_tf/model_U2GNN_Unsup_multi.py:43-62): concatenated slot-0
outputs of every U2GNN layer -> dropout -> SampledSoftmax(vocab, sampled_num, d*L).  The fork-only
pieces (cross-layer ``self_attn`` and the ``weight`` table it multiplies) are still constructed so
fork state_dicts load, but they are not on the loss path (node-level research, OUT of scope), and
``sampler_type``/``loss_type`` other than 'default' raise NotImplementedError.
"""
import math

import torch
import torch.nn as nn
from torch.nn import TransformerEncoder, TransformerEncoderLayer

from sampled_softmax import SampledSoftmax
from u2gnn_hip import kernels as K
from u2gnn_hip.core import DeviceBatch
from u2gnn_hip.engine import site_seed
from u2gnn_hip.unsup import SITE_SS_DROP, UnSupCore


class _EncodeFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, core, batch, train, seed, names, *params):
        OV, sctx = core.encode(batch, train, True, seed)
        fctx.core, fctx.sctx, fctx.names, fctx.params = core, sctx, names, params
        return OV

    @staticmethod
    def backward(fctx, dOV):
        grads = {n: torch.zeros_like(p) for n, p in zip(fctx.names, fctx.params)}
        fctx.core.encode_backward(fctx.sctx, dOV.contiguous(), grads)
        fctx.sctx = None
        return (None, None, None, None, None) + tuple(grads[n] for n in fctx.names)


class _DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(fctx, x, p, seed):
        x = x.contiguous()
        y = torch.empty_like(x)
        K.dropout(x, x.shape[1], y, x.shape[1], x.shape[0], x.shape[1], p, seed)
        fctx.p, fctx.seed = p, seed
        return y

    @staticmethod
    def backward(fctx, dy):
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        K.dropout(dy, dy.shape[1], dx, dy.shape[1], dy.shape[0], dy.shape[1], fctx.p, fctx.seed)
        return dx, None, None


class TransformerU2GNN(nn.Module):

    def __init__(self, vocab_size, feature_dim_size, ff_hidden_size, sampled_num,
                 num_self_att_layers, num_U2GNN_layers, dropout, device, sampler_type='default',
                 loss_type='default', adj_mat=None, single_layer_only=True, precision="fp32", attention="nodes"):
        super(TransformerU2GNN, self).__init__()
        if sampler_type != 'default' or loss_type != 'default':
            raise NotImplementedError("only sampler_type='default', loss_type='default' (graph-level U2GNN) "
                                      "are on the MI355X path; neighbour/contrastive/gae are node-level research")
        self.feature_dim_size = feature_dim_size
        if attention not in ("nodes", "neighbors"):
            raise ValueError(f"attention must be 'nodes' or 'neighbors', got {attention!r}")
        self.attention = attention
        self.self_attn = nn.MultiheadAttention(self.feature_dim_size, 1, dropout=dropout)
        self.ff_hidden_size = ff_hidden_size
        self.num_self_att_layers = num_self_att_layers
        self.num_U2GNN_layers = num_U2GNN_layers
        self.vocab_size = vocab_size
        self.sampled_num = sampled_num
        self.device = device
        self.single_layer_only = single_layer_only
        self.dropout_p = dropout
        self.precision = precision
        self.u2gnn_layers = torch.nn.ModuleList()
        self.adj_mat = adj_mat
        self.loss_type = loss_type
        self.weight = nn.Parameter(torch.Tensor(vocab_size, feature_dim_size))
        for _ in range(self.num_U2GNN_layers):
            encoder_layers = TransformerEncoderLayer(d_model=self.feature_dim_size, nhead=1,
                                                     dim_feedforward=self.ff_hidden_size, dropout=0.5)
            self.u2gnn_layers.append(TransformerEncoder(encoder_layers, self.num_self_att_layers,
                                                        enable_nested_tensor=False))
        self.dropouts = nn.Dropout(dropout)
        self.ss = SampledSoftmax(self.vocab_size, self.sampled_num, self.feature_dim_size * self.num_U2GNN_layers,
                                 self.device)
        self.reset_parameters()
        self._core = None

    def reset_parameters(self):
        stdv = math.sqrt(6.0 / (self.weight.size(0) + self.weight.size(1)))
        self.weight.data.uniform_(-stdv, stdv)

    @property
    def core(self) -> UnSupCore:
        if self._core is None:
            self._core = UnSupCore(self, self.precision)
        return self._core

    def trainable_names(self):
        """Parameters on the loss path (encoders + ss.weight)."""
        return [n for n, _ in self.named_parameters() if n.startswith("u2gnn_layers.") or n == "ss.weight"]

    def forward(self, X_concat, input_x, input_y, args=None):
        if isinstance(X_concat, DeviceBatch):
            b = X_concat
        else:
            N = X_concat.shape[0]
            if input_x.numel() and (int(input_x.min()) < 0 or int(input_x.max()) >= N):
                raise IndexError("index out of range in self (input_x entry outside [0, N))")
            b = DeviceBatch(N, 1, input_x.contiguous(), X_concat.to(torch.float32).contiguous(), None, None, None,
                            None, input_y)
        seed = int(torch.randint(0, 2 ** 62, (1,)).item()) if self.training else 0
        names = [n for n in self.trainable_names() if n.startswith("u2gnn_layers.")]
        params = [dict(self.named_parameters())[n] for n in names]
        if torch.is_grad_enabled():
            OV = _EncodeFn.apply(self.core, b, self.training, seed, names, *params)
        else:
            OV, _ = self.core.encode(b, self.training, False, seed)
        if self.training and self.dropout_p > 0:
            OV = _DropoutFn.apply(OV, self.dropout_p, site_seed(seed, 0, 0, SITE_SS_DROP))
        logits = self.ss(OV, b.input_y)
        return logits, self.weight
