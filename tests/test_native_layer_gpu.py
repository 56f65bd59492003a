"""The native layer executor (csrc/encoder_layer.cpp) issues exactly the kernel sequence of the
Python orchestration (u2gnn_hip/engine.py): same tiles, split counts and reduction order, so
outputs, input gradients and every parameter gradient must be bit-identical."""
import pytest
import torch

pytestmark = pytest.mark.gpu

from u2gnn_hip import native  # noqa: E402
from u2gnn_hip.engine import (SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF, Dims, LayerParams, OffPath,  # noqa: E402
                              PackedLayer, encoder_layer_backward, encoder_layer_forward, site_seed)


def _layer(d, ff, seed):
    torch.manual_seed(seed)
    layer = torch.nn.TransformerEncoderLayer(d, 1, ff, 0.5).cuda()
    with torch.no_grad():
        for prm in (layer.norm1.weight, layer.norm1.bias, layer.norm2.weight, layer.norm2.bias):
            prm.add_(0.1 * torch.randn_like(prm))
    return layer


def _zeros_like_params(p: LayerParams) -> LayerParams:
    return LayerParams(*[torch.full_like(t, float("nan")) for t in p.tensors()])


# d = 19, 4: fused LN and the small-width attention (small_layer.hip); (1920, 4, 1024): the C5 layer (long reductions batched at the end of a one-stream backward)
# (80, 136, 1024) and (100, 100, 256): C2-class layers (round 5): one query block, the unsplit fused
# softmax.P.V, FFN2 split-K + slab LayerNorm at dp = 192 / 128, the tiny direct dX1 product (ff = 256)
@pytest.mark.parametrize("N,d,ff", [(300, 67, 128), (1000, 367, 1024), (300, 19, 128), (1920, 4, 1024),
                                    (80, 136, 1024), (100, 100, 256)])
@pytest.mark.parametrize("prec", ["bf16x3", "fp32", "mixed", "fwd32", "fwd6", "fwdh"])
@pytest.mark.parametrize("train", [True, False])
@pytest.mark.parametrize("side", [False, True])
def test_native_layer_matches_python_orchestration(N, d, ff, prec, train, side):
    layer = _layer(d, ff, 5)
    p = LayerParams.from_encoder_layer(layer)
    dims = Dims(N, d, ff)
    packed = PackedLayer(d, ff, "cuda")
    packed.pack(p)
    seeds = {s: site_seed(77, 0, 1, s) for s in (SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2)}
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.zeros(dims.Np, dims.dp, device="cuda")
    X[:N, :d] = torch.randn(N, d, device="cuda", generator=g)
    dY = torch.zeros(dims.Np, dims.dp, device="cuda")
    dY[:N, :d] = torch.randn(N, d, device="cuda", generator=g)

    Y_ref, ctx_ref = encoder_layer_forward(X, packed, p, dims, train, seeds, True, prec)
    g_ref = _zeros_like_params(p)
    dX_ref = encoder_layer_backward(dY, ctx_ref, packed, p, g_ref, dims, prec)

    Y, ctx = native.layer_forward(X, packed, p, dims, train, seeds, True, prec, 0.5)
    g_nat = _zeros_like_params(p)
    off = OffPath(X.device) if side else None
    dX = native.layer_backward(dY, ctx, packed, p, g_nat, dims, prec, side=off.side if off else None)
    if off is not None:
        off.join()
    torch.cuda.synchronize()
    assert torch.equal(Y, Y_ref)
    assert torch.equal(dX, dX_ref)
    for name, a, b in zip(("in_w", "in_b", "out_w", "out_b", "l1_w", "l1_b", "l2_w", "l2_b", "n1_w", "n1_b", "n2_w",
                           "n2_b"), g_nat.tensors(), g_ref.tensors()):
        assert torch.isfinite(a).all(), name
        assert torch.equal(a, b), name


def test_native_forward_without_ctx_matches():
    N, d, ff = 500, 67, 128
    layer = _layer(d, ff, 9)
    p = LayerParams.from_encoder_layer(layer)
    dims = Dims(N, d, ff)
    packed = PackedLayer(d, ff, "cuda")
    packed.pack(p)
    X = torch.zeros(dims.Np, dims.dp, device="cuda")
    X[:N, :d] = torch.randn(N, d, device="cuda")
    Y_ref, _ = encoder_layer_forward(X, packed, p, dims, False, {}, False, "bf16x3")
    Y, c = native.layer_forward(X, packed, p, dims, False, {}, False, "bf16x3", 0.5)
    assert c is None
    assert torch.equal(Y, Y_ref)


def test_mixed_precision_only_changes_attention_backward():
    """precision "mixed": the forward is the bf16x3 forward bit for bit; the backward differs
    (dS, dQ, dK on plain bf16) but stays within bf16 rounding of the bf16x3 backward."""
    N, d, ff = 1000, 367, 1024
    layer = _layer(d, ff, 5)
    p = LayerParams.from_encoder_layer(layer)
    dims = Dims(N, d, ff)
    packed = PackedLayer(d, ff, "cuda")
    packed.pack(p)
    seeds = {s: site_seed(77, 0, 1, s) for s in (SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2)}
    g = torch.Generator(device="cuda").manual_seed(3)
    X = torch.zeros(dims.Np, dims.dp, device="cuda")
    X[:N, :d] = torch.randn(N, d, device="cuda", generator=g)
    dY = torch.zeros(dims.Np, dims.dp, device="cuda")
    dY[:N, :d] = torch.randn(N, d, device="cuda", generator=g)
    out = {}
    for prec in ("bf16x3", "mixed"):
        Y, ctx = native.layer_forward(X, packed, p, dims, True, seeds, True, prec, 0.5)
        gg = _zeros_like_params(p)
        dX = native.layer_backward(dY, ctx, packed, p, gg, dims, prec)
        torch.cuda.synchronize()
        out[prec] = (Y, dX, gg)
    assert torch.equal(out["mixed"][0], out["bf16x3"][0])
    a, b = out["mixed"][1], out["bf16x3"][1]
    assert not torch.equal(a, b)
    assert ((a - b).abs().max() / b.abs().max()).item() < 2e-2
    # the FFN weight gradients do not depend on the attention backward at all
    assert torch.equal(out["mixed"][2].l1_w, out["bf16x3"][2].l1_w)
    assert not torch.equal(out["mixed"][2].in_w, out["bf16x3"][2].in_w)


def test_probe_times_every_launch_of_a_role():
    """u2gnn_probe_arm/collect (bench.py's live roofline timing): every dS / QK launch of the
    executor is bracketed by events on its own stream; capacity caps the count."""
    from u2gnn_hip import _lib
    N, d, ff = 1000, 367, 1024
    layer = _layer(d, ff, 5)
    p = LayerParams.from_encoder_layer(layer)
    dims = Dims(N, d, ff)
    packed = PackedLayer(d, ff, "cuda")
    packed.pack(p)
    seeds = {s: site_seed(77, 0, 1, s) for s in (SITE_ATTN, SITE_DROP1, SITE_DROPFF, SITE_DROP2)}
    X = torch.zeros(dims.Np, dims.dp, device="cuda")
    X[:N, :d] = torch.randn(N, d, device="cuda")
    dY = torch.zeros_like(X)
    dY[:N, :d] = torch.randn(N, d, device="cuda")
    for role, cap, runs, want in ((_lib.ROLE_DS, 8, 3, 3), (_lib.ROLE_QK, 2, 3, 2), (_lib.ROLE_DK, 4, 2, 2)):
        native.probe_arm(role, cap)
        off = OffPath(X.device)
        for _ in range(runs):
            Y, ctx = native.layer_forward(X, packed, p, dims, True, seeds, True, "bf16x3", 0.5)
            g = _zeros_like_params(p)
            native.layer_backward(dY, ctx, packed, p, g, dims, "bf16x3", side=off.side)
        off.join()
        ms, n = native.probe_collect()
        assert n == want and ms > 0.0, (role, n, ms)
    assert native.probe_collect() == (0.0, 0)   # disarmed
