"""Drop-in replacement of U2GNN_pytorch/sampled_softmax.py (SampledSoftmax, :11-56) on MI355X.

Same constructor ``SampledSoftmax(ntokens, nsampled, nhid, device)``, ``weight`` parameter and
init (uniform +-sqrt(6/(ntokens+nhid)), :25-27), ``forward(inputs, labels)`` and
``sampled(inputs, labels, sample_values)``.  The loss kernel (u2gnn_sampled_softmax_fwd/bwd)
computes  -log(exp(x.w_y) / sum_s exp(x.w_s)) = logsumexp_s(x.w_s) - x.w_y  per row, which is
the reference expression whenever the reference is finite (the reference has no max
subtraction and overflows to inf/NaN for large logits; this does not).

Differences by design: ``forward`` does not copy ``labels`` to the host — the reference does
(:31) only to compute expected counts the loss never uses; the sampler's random stream
(consumed by ``sample`` alone) is unchanged by that.
"""
import math

import numpy as np
import torch
import torch.nn as nn

from log_uniform import LogUniformSampler
from u2gnn_hip import kernels as K


class _SampledSoftmaxFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, inputs, labels, sample_ids, weight):
        x = inputs.contiguous()
        n, D = x.shape
        S = sample_ids.numel()
        loss = torch.empty(n, device=x.device, dtype=torch.float32)
        prob = torch.empty(n, S, device=x.device, dtype=torch.float32)
        K.sampled_softmax_fwd(x, D, labels, sample_ids, S, weight, weight.stride(0), loss, prob, n, D)
        ctx.save_for_backward(x, labels, sample_ids, weight, prob)
        return loss

    @staticmethod
    def backward(ctx, dloss):
        x, labels, sample_ids, weight, prob = ctx.saved_tensors
        n, D = x.shape
        dx = torch.empty_like(x)
        dW = torch.zeros_like(weight)
        K.sampled_softmax_bwd(x, D, labels, sample_ids, sample_ids.numel(), weight, weight.stride(0), prob,
                              dloss.contiguous(), dx, D, dW, dW.stride(0), n, D)
        return dx, None, None, dW


class SampledSoftmax(nn.Module):
    def __init__(self, ntokens, nsampled, nhid, device):
        super(SampledSoftmax, self).__init__()
        self.ntokens = ntokens
        self.nsampled = nsampled
        self.device = device
        self.sampler = LogUniformSampler(self.ntokens)
        self.weight = nn.Parameter(torch.Tensor(ntokens, nhid))
        self.reset_parameters()

    def reset_parameters(self):
        stdv = math.sqrt(6.0 / (self.weight.size(0) + self.weight.size(1)))
        self.weight.data.uniform_(-stdv, stdv)

    def draw_samples(self):
        ids, _ = self.sampler.sample_set_order(self.nsampled)
        return ids

    def forward(self, inputs, labels):
        ids = self.draw_samples()
        return self.sampled(inputs, labels, (ids, None, None))

    def sampled(self, inputs, labels, sample_values):
        assert inputs.device == labels.device
        sample_ids = sample_values[0]
        if not torch.is_tensor(sample_ids):
            sample_ids = torch.as_tensor(np.asarray(sample_ids, dtype=np.int64))
        sample_ids = sample_ids.to(inputs.device, non_blocking=True)
        return _SampledSoftmaxFn.apply(inputs, labels, sample_ids, self.weight)
