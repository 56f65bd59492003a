"""The oracle restatement is pinned against the REFERENCE-generated golden fixtures (CPU only)."""
import ctypes
import os

import numpy as np
import pytest
import torch

from oracle import u2gnn_oracle as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _close(a, b, tol=1e-4):
    a, b = torch.as_tensor(a).double(), torch.as_tensor(b).double()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item() <= tol


@pytest.mark.parametrize("name", ["mutag_sup", "mutag_sup_L2T2", "imdbb_sup"])
@pytest.mark.parametrize("slots", [None, 1])
def test_oracle_sup_forward_and_grads(golden_dir, name, slots):
    z = dict(np.load(os.path.join(golden_dir, name + ".npz")))
    bs, k, T, ff, L, d, C, _ = [int(x) for x in z["meta"]]
    sd = {kk[5:]: torch.from_numpy(v).clone().requires_grad_(True) for kk, v in z.items() if kk.startswith("init.")}
    s = O.sup_forward(sd, torch.from_numpy(z["b0_input_x"]), z["b0_offsets"], torch.from_numpy(z["b0_X"]), L, T,
                      train=False, slots=slots)
    assert _close(s.detach(), z["scores"])
    loss = O.soft_cross_entropy(s, O.label_smoothing(torch.from_numpy(z["b0_labels"]), C))
    assert abs(loss.item() - float(z["loss"])) < 1e-4 * max(1, abs(float(z["loss"])))
    loss.backward()
    for kk, v in sd.items():
        assert _close(v.grad, z["grad." + kk], 1e-3), kk
    # clip + Adam restatement == torch clip_grad_norm_ + Adam (reference train step)
    params = list(sd.values())
    total = O.clip_and_adam([p.detach() for p in params], [p.grad for p in params], {}, float(z["lr"]))
    assert abs(total - float(z["grad_norm"])) < 1e-4 * float(z["grad_norm"])
    # Adam's first step moves every entry by ~lr*sign(g) when |g| >> eps, so entries whose
    # true gradient is zero (e.g. the key bias: softmax is shift-invariant) carry rounding-noise
    # gradients whose sign can flip: bound those by 2*lr, the rest to 1e-4.
    lr = float(z["lr"])
    for kk, v in sd.items():
        g = torch.from_numpy(z["grad." + kk]).abs()
        sig = g > 1e-4 * max(g.max().item(), 1e-30)
        a, r = v.detach(), torch.from_numpy(z["after." + kk])
        assert (a - r)[sig].abs().max().item() <= 1e-4 if sig.any() else True, kk
        assert (a - r).abs().max().item() <= 2 * lr + 1e-6, kk


def test_oracle_unsup_and_sampled_softmax(golden_dir):
    z = dict(np.load(os.path.join(golden_dir, "sampled_softmax.npz")))
    x = torch.from_numpy(z["inputs"]).requires_grad_(True)
    w = torch.from_numpy(z["weight"]).requires_grad_(True)
    lg = O.sampled_softmax_logits(x, torch.from_numpy(z["labels"]), w, torch.from_numpy(z["sample_ids"]))
    assert _close(lg.detach(), z["logits"])
    lg.sum().backward()
    assert _close(x.grad, z["grad_inputs"], 1e-4) and _close(w.grad, z["grad_weight"], 1e-4)
    u = dict(np.load(os.path.join(golden_dir, "ptc_unsup.npz")))
    bs, k, T, ff, L, d, V = [int(v) for v in u["meta"]]
    sd = {kk[5:]: torch.from_numpy(v) for kk, v in u.items() if kk.startswith("init.u2gnn")}
    lg = O.unsup_forward(sd, torch.from_numpy(u["init.ss.weight"]), torch.from_numpy(u["input_x"]),
                         torch.from_numpy(u["X"]), torch.from_numpy(u["input_y"]), torch.from_numpy(u["sample_ids"]),
                         L, T, train=False)
    assert _close(lg, u["logits"], 1e-4)


def _oracle_lib():
    path = os.path.join(REPO, "oracle", "liblus_oracle.so")
    if not os.path.exists(path):
        import subprocess
        subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "liblus_oracle.so"])
    lib = ctypes.CDLL(path)
    lib.lus_oracle_create.restype = ctypes.c_void_p
    lib.lus_oracle_create.argtypes = [ctypes.c_int64, ctypes.c_uint32]
    lib.lus_oracle_sample.argtypes = [ctypes.c_void_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_void_p]
    lib.lus_oracle_expected_count.argtypes = [ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p, ctypes.c_int64,
                                              ctypes.c_void_p]
    lib.lus_oracle_destroy.argtypes = [ctypes.c_void_p]
    return lib


def test_c_oracle_sampler_vs_reference_sets(golden_dir):
    """oracle/log_uniform_oracle.c reproduces the reference C++ sampler's sets exactly."""
    z = dict(np.load(os.path.join(golden_dir, "sampler.npz")))
    lib = _oracle_lib()
    for V in (8792, 2542091):
        h = lib.lus_oracle_create(V, 1111)
        for c in range(3):
            out = np.zeros(512, np.int64)
            nt = ctypes.c_int32()
            assert lib.lus_oracle_sample(h, 512, out.ctypes.data, ctypes.byref(nt)) == 0
            ref = z[f"V{V}_c{c}_ids_order"]
            assert np.array_equal(out, np.sort(ref))
            ec = np.zeros(512, np.float32)
            lib.lus_oracle_expected_count(h, nt.value, ref.ctypes.data, 512, ec.ctypes.data)
            assert np.array_equal(ec, z[f"V{V}_c{c}_sample_freq"])
        lib.lus_oracle_destroy(h)


def test_oracle_neighbors_mode_matches_torch_encoder_on_transposed_window():
    """Paper semantics restated: the oracle's encoder on the transposed window [k+1, N, d] equals
    torch.nn.TransformerEncoder (the reference's module, eval mode) fed the same tensor, and the
    attention="neighbors" forward uses exactly that (slot 0 = sequence position 0)."""
    import torch
    from oracle import u2gnn_oracle as O
    torch.manual_seed(3)
    d, ff, T, N, k = 12, 32, 2, 9, 4
    enc = torch.nn.TransformerEncoder(torch.nn.TransformerEncoderLayer(d, 1, ff, 0.5), T,
                                      enable_nested_tensor=False).eval()
    x = torch.randn(N, k + 1, d)
    ref = enc(x.transpose(0, 1))
    sd = {f"u2gnn_layers.0.{kk}": v for kk, v in enc.state_dict().items()}
    y = x.transpose(0, 1)
    for t in range(T):
        y = O.encoder_layer(y, O.layer_params(sd, 0, t), train=False)
    assert torch.allclose(y, ref, atol=1e-5)
    # full forward: pooled slot-0 rows through the head
    input_x = torch.randint(0, N, (N, k + 1))
    input_x[:, 0] = torch.arange(N)
    X = torch.randn(N, d)
    sd["predictions.0.weight"], sd["predictions.0.bias"] = torch.randn(3, d), torch.randn(3)
    offsets = np.array([0, 4, N])
    scores = O.sup_forward(sd, input_x, offsets, X, 1, T, train=False, attention="neighbors")
    out = enc(torch.nn.functional.embedding(input_x, X).transpose(0, 1))[0]
    exp = O.pool_matrix(offsets) @ out @ sd["predictions.0.weight"].t() + sd["predictions.0.bias"]
    assert torch.allclose(scores, exp, atol=1e-5)
