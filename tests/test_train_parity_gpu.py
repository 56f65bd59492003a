"""Train-mode (dropout on) parity of the WHOLE training step in the precision the bench times.

The reference trains with model.train() and p = 0.5 at every encoder dropout site
(pytorch_U2GNN_Sup.py:20, train_pytorch_U2GNN_Sup.py:150-161).  Torch's CPU Bernoulli stream cannot be
reproduced on the GPU, so the oracle restatement is run with the exact masks the kernels draw
(u2gnn_dropout_mask of every site seed) and the step is compared end to end: scores, loss, every
parameter gradient, the clip norm and the parameters after clip_grad_norm_(0.5) + Adam.

Cases: the reference-golden batches mutag_sup_L2T2 (L = 2, T = 2) and imdbb_sup (C2), and one full C4
batch (N ~ 4.8K, d = 367, T = 4) -- in fp32 and in bf16x3 (the bench's precision).

Tolerance: max|ours - oracle| / max(1, max|oracle|) per tensor, TOL = 1e-3 (north_star), for every
quantity of every case except where TOL_TRAIN below says otherwise; the reason for each exception is
measured and written beside it.  U2GNN_PARITY_REPORT=<path> appends the measured
per-tensor errors as JSON lines (profiles/ evidence)."""
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

DEV = "cuda"
TOL = 1e-3


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item()


def _kernel_masks(seed, L, T, N, B, d, ff):
    from u2gnn_hip import kernels as K
    from u2gnn_hip.engine import SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF, SITE_HEAD, row_pad, rup, site_seed
    Np, dp, ffp = row_pad(N), rup(d, 64), rup(ff, 64)

    def mk(s, r, c):
        return K.dropout_mask(s, r, c, 0.5).float().cpu()
    masks = {}
    for l in range(L):
        for t in range(T):
            masks[(l, t)] = {"attn": mk(site_seed(seed, l, t, SITE_ATTN), Np, Np)[:N, :N],
                             "drop1": mk(site_seed(seed, l, t, SITE_DROP1), Np, dp)[:N, :d],
                             "drop_ff": mk(site_seed(seed, l, t, SITE_DROPFF), Np, ffp)[:N, :ff],
                             "drop2": mk(site_seed(seed, l, t, SITE_DROP2), Np, dp)[:N, :d]}
        masks[("head", l)] = mk(site_seed(seed, l, 0, SITE_HEAD), B, dp)[:, :d]
    return masks


def _case(name, golden_dir):
    """-> (init state_dict, dims (L, T, d, ff, C), input_x, offsets, X, labels, lr)."""
    if name == "c4":
        from pytorch_U2GNN_Sup import TransformerU2GNN
        from u2gnn_hip.batching import BatchLoader
        from u2gnn_hip.synthetic import collab_like
        np.random.seed(123)
        hb = BatchLoader(collab_like(), 64, 16)()
        torch.manual_seed(123)
        m = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1)
        sd = {k: v.detach().clone() for k, v in m.state_dict().items()}
        return sd, (1, 4, 367, 1024, 3), hb.input_x, hb.offsets, hb.X_concat, hb.labels, 5e-4
    z = dict(np.load(os.path.join(golden_dir, name + ".npz")))
    bs, k, T, ff, L, d, C, fold = [int(x) for x in z["meta"]]
    sd = {kk[5:]: torch.from_numpy(v) for kk, v in z.items() if kk.startswith("init.")}
    return sd, (L, T, d, ff, C), z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"], float(z["lr"])


# Measured exceptions to TOL (case, precision) -> {quantity: bound}; everything not listed is held at 1e-3.
# C4 in bf16x3 (round 4, profiles/r04/train_parity_*.jsonl): scores 2.3e-6, loss 1.5e-7, clip norm 6.3e-6, every
# gradient except linear1's <= 5.2e-4 -- but linear1.weight / .bias gradients 9e-5 .. 1.66e-2: a few of the
# N x ff = 5 M pre-activations per layer lie within the 2^-16 product error of zero and switch the ReLU
# (test_c4_bf16x3_train_deviation_is_the_relu_boundary: with the GPU's ReLU decisions in the oracle every
# gradient is back under 1e-3).  Adam's first step moves every element by lr * g / |g|, so an element whose
# gradient changes sign moves 2 lr = 1e-3 the other way: the post-Adam parameters measured 9.9e-4.  fp32 holds
# 1e-3 everywhere (max 4.1e-6) and is the parity path; bench.py reports its C4 rate beside the headline.
_L1 = {f"grad.u2gnn_layers.0.layers.{t}.linear1.{w}": 2.5e-2 for t in range(4) for w in ("weight", "bias")}
_AFTER = {f"after.{n}": 1.5e-3 for n in
          [f"u2gnn_layers.0.layers.{t}.{k}" for t in range(4) for k in
           ("self_attn.in_proj_weight", "self_attn.in_proj_bias", "self_attn.out_proj.weight", "self_attn.out_proj.bias",
            "linear1.weight", "linear1.bias", "linear2.weight", "linear2.bias", "norm1.weight", "norm1.bias",
            "norm2.weight", "norm2.bias")] + ["predictions.0.weight", "predictions.0.bias"]}
TOL_TRAIN = {("c4", "bf16x3"): dict(_L1, **_AFTER)}


@pytest.mark.parametrize("precision", ["fp32", "bf16x3"])
@pytest.mark.parametrize("name", ["mutag_sup_L2T2", "imdbb_sup", "c4"])
def test_train_mode_step_matches_oracle_with_kernel_masks(golden_dir, name, precision):
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip import kernels as K
    from u2gnn_hip.core import DeviceBatch, FusedAdam
    sd0, (L, T, d, ff, C), input_x, offsets, X, labels, lr = _case(name, golden_dir)
    m = TransformerU2GNN(d, ff, C, T, 0.5, L, precision=precision)
    m.load_state_dict(sd0)
    m = m.to(DEV).train()
    flat = m.flatten_parameters()
    b = DeviceBatch.from_offsets(input_x, offsets, X, labels, device=DEV)
    seed = 987654321
    scores, ctx = m.core.forward(b, train=True, need_ctx=True, seed=seed)
    dsc = torch.empty_like(scores)
    loss = torch.zeros(1, device=DEV)
    K.smoothed_ce(scores, b.labels, b.B, C, 0.1, loss, dsc)
    m.core.backward(ctx, dsc, flat.grads)
    scores_c = scores.detach().cpu().clone()
    grads_c = {n: flat.grads[n].detach().cpu().clone() for n in flat.names}
    opt = FusedAdam(flat, lr=lr, max_norm=0.5)
    opt.step()
    after = {n: p.detach().cpu().clone() for n, p in m.named_parameters()}

    torch.set_num_threads(min(16, os.cpu_count()))
    masks = _kernel_masks(seed, L, T, b.N, b.B, d, ff)
    prm = {k: v.detach().clone().double().float().requires_grad_(True) for k, v in sd0.items()}
    ref = O.sup_forward(prm, torch.from_numpy(np.asarray(input_x)), offsets, torch.from_numpy(np.asarray(X)), L, T,
                        train=True, dropout=0.5, slots=1, masks=masks)
    lref = O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(np.asarray(labels)), C))
    lref.backward()
    names = [n for n, _ in m.named_parameters()]
    state = {}
    p_ref = [prm[n].detach().clone() for n in names]
    gnorm_ref = O.clip_and_adam(p_ref, [prm[n].grad for n in names], state, lr)

    err = {"scores": rel_err(scores_c, ref.detach()),
           "loss": abs(loss.item() - lref.item()) / max(1.0, abs(lref.item())),
           "grad_norm": abs(opt.grad_norm() - gnorm_ref) / max(1.0, gnorm_ref)}
    for n in names:
        err["grad." + n] = rel_err(grads_c[n], prm[n].grad)
    for n, p in zip(names, p_ref):
        err["after." + n] = rel_err(after[n], p)
    rep = os.environ.get("U2GNN_PARITY_REPORT")
    if rep:
        with open(rep, "a") as f:
            f.write(json.dumps({"case": name, "precision": precision, "N": b.N, "errors": err}) + "\n")
    bounds = TOL_TRAIN.get((name, precision), {})
    bad = {k: v for k, v in err.items() if v > bounds.get(k, TOL)}
    assert not bad, f"{name} {precision}: above tolerance: {bad}"


def test_c4_bf16x3_train_deviation_is_the_relu_boundary(golden_dir):
    """Where bf16x3 misses 1e-3 in train mode (C4: linear1 gradients, see TOL_TRAIN), the cause is the
    ReLU's on/off decision of pre-activations within ~1e-5 of zero: split-bf16 products perturb them at the
    2^-16 level and a flipped unit moves its row of dW1 by dH[n, j] X1[n, :].  Taking the ReLU decision of
    the GPU run into the oracle (masks["relu"], from the saved dropped-ReLU image Hd: Hd > 0 is relu' * keep)
    and comparing again must put EVERY quantity within 1e-3 -- the remaining difference is the continuous
    2^-16 error of the products."""
    import u2gnn_hip.native as native
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip import kernels as K
    from u2gnn_hip.core import DeviceBatch
    sd0, (L, T, d, ff, C), input_x, offsets, X, labels, lr = _case("c4", golden_dir)
    m = TransformerU2GNN(d, ff, C, T, 0.5, L, precision="bf16x3")
    m.load_state_dict(sd0)
    m = m.to(DEV).train()
    flat = m.flatten_parameters()
    b = DeviceBatch.from_offsets(input_x, offsets, X, labels, device=DEV)
    seed = 987654321
    prev = native.set_enabled(False)   # the Python orchestration (bit-identical to the executor) exposes Hd
    try:
        scores, ctx = m.core.forward(b, train=True, need_ctx=True, seed=seed)
        dsc = torch.empty_like(scores)
        loss = torch.zeros(1, device=DEV)
        K.smoothed_ce(scores, b.labels, b.B, C, 0.1, loss, dsc)
        m.core.backward(ctx, dsc, flat.grads)
        torch.cuda.synchronize()
    finally:
        native.set_enabled(prev)
    grads_c = {n: flat.grads[n].detach().cpu().clone() for n in flat.names}
    masks = _kernel_masks(seed, L, T, b.N, b.B, d, ff)
    for t in range(T):
        masks[(0, t)]["relu"] = (ctx["stack"]["layers"][0][t].Hd[:b.N, :ff].detach().cpu() > 0).float()
    torch.set_num_threads(min(16, os.cpu_count()))
    prm = {k: v.detach().clone().requires_grad_(True) for k, v in sd0.items()}
    ref = O.sup_forward(prm, torch.from_numpy(np.asarray(input_x)), offsets, torch.from_numpy(np.asarray(X)), L, T,
                        train=True, dropout=0.5, slots=1, masks=masks)
    O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(np.asarray(labels)), C)).backward()
    err = {n: rel_err(grads_c[n], prm[n].grad) for n in flat.names}
    rep = os.environ.get("U2GNN_PARITY_REPORT")
    if rep:
        with open(rep, "a") as f:
            f.write(json.dumps({"case": "c4_relu_injected", "precision": "bf16x3", "N": b.N, "errors": err}) + "\n")
    bad = {k: v for k, v in err.items() if v > TOL}
    assert not bad, f"with the GPU's ReLU decisions injected: {bad}"
