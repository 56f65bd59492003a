"""Train-mode parity per precision policy on the C4 benchmark batch.

The step (dropout on, the kernels' own masks injected into the oracle restatement) is run through the
Python orchestration with per-role precision overrides (engine.ROLE_PREC) on top of bf16x3, and every
quantity the parity test checks (scores, loss, every gradient, the clip norm, the post-Adam parameters)
is compared with the oracle: max|ours - oracle| / max(1, max|oracle|).  The oracle run depends only on
the dropout seed, so it is computed once per seed and shared by all policies.
Usage (GPU box): python tools/prec_train_probe.py [--seeds 987654321,5] > gpurun_out/prec_train.jsonl
"""
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402

FWD = ("in_proj", "qk", "pv", "out_proj", "ffn1", "ffn2")
POLICIES = {   # name -> (layer precision, role overrides)
    "bf16x3": ("bf16x3", {}),
    "ffn1": ("bf16x3", {"ffn1": "fp32"}),
    "fwd_proj": ("bf16x3", {r: "fp32" for r in ("in_proj", "out_proj", "ffn1", "ffn2")}),
    "fwd_attn": ("bf16x3", {r: "fp32" for r in ("qk", "pv")}),
    "fwd_all": ("bf16x3", {r: "fp32" for r in FWD}),
    "fp32": ("fp32", {}),
    "x6_proj": ("bf16x3", {r: "bf16x6" for r in ("in_proj", "out_proj", "ffn1", "ffn2")}),
    "x6_all": ("bf16x3", {r: "bf16x6" for r in FWD}),
    "fwd6": ("fwd6", {}),
    "fwdh": ("fwdh", {}),
    "fwdh_3pass": ("fwdh", {}),   # the three-pass attention forward (engine.FUSED_MIN_NP raised for this policy)
    "fwd32": ("fwd32", {}),
    "x6_nopv": ("bf16x3", {r: "bf16x6" for r in ("in_proj", "qk", "out_proj", "ffn1", "ffn2")}),
    "x6_noqk": ("bf16x3", {r: "bf16x6" for r in ("in_proj", "pv", "out_proj", "ffn1", "ffn2")}),
}


def rel_err(a, b):
    a = torch.as_tensor(a).double().cpu()
    b = torch.as_tensor(b).double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item()


def main():
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip import engine, native
    from u2gnn_hip import kernels as K
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch, FusedAdam
    from u2gnn_hip.engine import SITE_ATTN, SITE_DROP1, SITE_DROP2, SITE_DROPFF, SITE_HEAD, row_pad, rup, site_seed
    from u2gnn_hip.synthetic import collab_like
    seeds = [987654321]
    only = None
    fp64 = "--fp64" in sys.argv
    for i, a in enumerate(sys.argv):
        if a == "--seeds":
            seeds = [int(x) for x in sys.argv[i + 1].split(",")]
        if a == "--policies":
            only = sys.argv[i + 1].split(",")
    native.set_enabled(False)
    fused_min_np = engine.FUSED_MIN_NP
    dev = "cuda"
    torch.set_num_threads(min(16, os.cpu_count()))
    np.random.seed(123)
    hb = BatchLoader(collab_like(), 64, 16)()
    torch.manual_seed(123)
    m0 = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1)
    sd0 = {k: v.detach().clone() for k, v in m0.state_dict().items()}
    L, T, d, ff, C, lr = 1, 4, 367, 1024, 3, 5e-4
    names = [n for n, _ in m0.named_parameters()]

    def masks_for(seed, N, B):
        Np, dp, ffp = row_pad(N), rup(d, 64), rup(ff, 64)

        def mk(s, r, c):
            return K.dropout_mask(s, r, c, 0.5).float().cpu()
        ms = {}
        for t in range(T):
            ms[(0, t)] = {"attn": mk(site_seed(seed, 0, t, SITE_ATTN), Np, Np)[:N, :N],
                          "drop1": mk(site_seed(seed, 0, t, SITE_DROP1), Np, dp)[:N, :d],
                          "drop_ff": mk(site_seed(seed, 0, t, SITE_DROPFF), Np, ffp)[:N, :ff],
                          "drop2": mk(site_seed(seed, 0, t, SITE_DROP2), Np, dp)[:N, :d]}
        ms[("head", 0)] = mk(site_seed(seed, 0, 0, SITE_HEAD), B, dp)[:, :d]
        return ms

    captured = []
    relu0 = torch.relu

    def capture(x):
        captured.append(x[:, 0].detach().double().clone())
        return relu0(x)

    def flips(on_gpu, pre, keep):
        """ReLU decisions of kept units that differ from the sign of `pre` (a list per layer)."""
        n, mx = 0, 0.0
        for t in range(T):
            diff = keep[t] & (on_gpu[t] != (pre[t] > 0))
            n += int(diff.sum())
            if diff.any():
                mx = max(mx, float(pre[t][diff].abs().max()))
        return n, mx

    for seed in seeds:
        b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=dev)
        t0 = time.time()
        masks = masks_for(seed, b.N, b.B)
        prm = {k: v.detach().clone().requires_grad_(True) for k, v in sd0.items()}
        captured.clear()
        torch.relu = capture
        ref = O.sup_forward(prm, torch.from_numpy(np.asarray(hb.input_x)), hb.offsets,
                            torch.from_numpy(np.asarray(hb.X_concat)), L, T, train=True, dropout=0.5, slots=1,
                            masks=masks)
        torch.relu = relu0
        pre32 = list(captured)
        keep = [masks[(0, t)]["drop_ff"] > 0 for t in range(T)]
        lref = O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(np.asarray(hb.labels)), C))
        lref.backward()
        p_ref = [prm[n].detach().clone() for n in names]
        gnorm_ref = O.clip_and_adam(p_ref, [prm[n].grad for n in names], {}, lr)
        print(json.dumps({"seed": seed, "oracle_s": round(time.time() - t0, 1), "N": b.N}), flush=True)
        ref64 = None
        if fp64:
            m64 = {k: v.double() for k, v in masks.items() if k[0] == "head"}
            m64.update({k: {kk: vv.double() for kk, vv in v.items()} for k, v in masks.items() if k[0] != "head"})
            p64 = {k: v.detach().clone().double().requires_grad_(True) for k, v in sd0.items()}
            captured.clear()
            torch.relu = capture
            r64 = O.sup_forward(p64, torch.from_numpy(np.asarray(hb.input_x)), hb.offsets,
                                torch.from_numpy(np.asarray(hb.X_concat)).double(), L, T, train=True, dropout=0.5,
                                slots=1, masks=m64)
            torch.relu = relu0
            pre64 = list(captured)
            l64 = O.soft_cross_entropy(r64, O.label_smoothing(torch.from_numpy(np.asarray(hb.labels)), C).double())
            l64.backward()
            ref64 = {"scores": r64.detach()}
            ref64.update({"grad." + n: p64[n].grad for n in names})
            e = {"scores": rel_err(ref.detach(), ref64["scores"])}
            e.update({"grad." + n: rel_err(prm[n].grad, p64[n].grad) for n in names})
            worst = max(e, key=e.get)
            print(json.dumps({"seed": seed, "policy": "oracle_fp32_vs_fp64", "max_err": e[worst], "worst": worst,
                              "linear1_grad": max(v for k, v in e.items() if "linear1" in k),
                              "pass_1e-3": e[worst] <= 1e-3,
                              "relu_flips_vs_fp64": flips([p > 0 for p in pre32], pre64, keep)}), flush=True)
        for pname, (base, roles) in POLICIES.items():
            if only and pname not in only:
                continue
            engine.ROLE_PREC.clear()
            engine.ROLE_PREC.update(roles)
            engine.FUSED_MIN_NP = 1 << 30 if pname.endswith("_3pass") else fused_min_np
            m = TransformerU2GNN(d, ff, C, T, 0.5, L, precision=base)
            m.load_state_dict(sd0)
            m = m.to(dev).train()
            flat = m.flatten_parameters()
            scores, ctx = m.core.forward(b, train=True, need_ctx=True, seed=seed)
            dsc = torch.empty_like(scores)
            loss = torch.zeros(1, device=dev)
            K.smoothed_ce(scores, b.labels, b.B, C, 0.1, loss, dsc)
            m.core.backward(ctx, dsc, flat.grads)
            grads = {n: flat.grads[n].detach().cpu().clone() for n in flat.names}
            opt = FusedAdam(flat, lr=lr, max_norm=0.5)
            opt.step()
            after = {n: p.detach().cpu().clone() for n, p in m.named_parameters()}
            err = {"scores": rel_err(scores, ref.detach()),
                   "loss": abs(loss.item() - lref.item()) / max(1.0, abs(lref.item())),
                   "grad_norm": abs(opt.grad_norm() - gnorm_ref) / max(1.0, gnorm_ref)}
            for n in names:
                err["grad." + n] = rel_err(grads[n], prm[n].grad)
            for n, p in zip(names, p_ref):
                err["after." + n] = rel_err(after[n], p)
            if ref64 is not None:
                e64 = [rel_err(scores, ref64["scores"])] + [rel_err(grads[n], ref64["grad." + n]) for n in names]
                err64 = max(e64)
            on_gpu = [(ctx["stack"]["layers"][0][t].Hd[:b.N, :ff].detach().cpu() > 0) for t in range(T)]
            fl32 = flips(on_gpu, pre32, keep)
            fl64 = flips(on_gpu, pre64, keep) if ref64 is not None else None
            worst = max(err, key=err.get)
            l1 = max(v for k, v in err.items() if k.startswith("grad.") and "linear1" in k)
            other = max(v for k, v in err.items() if k.startswith("grad.") and "linear1" not in k)
            aft = max(v for k, v in err.items() if k.startswith("after."))
            print(json.dumps({"seed": seed, "policy": pname, "max_err": err[worst], "worst": worst,
                              "linear1_grad": l1, "other_grad": other, "after": aft, "scores": err["scores"],
                              "pass_1e-3": err[worst] <= 1e-3,
                              "vs_fp64": err64 if ref64 is not None else None,
                              "relu_flips_vs_oracle32": fl32, "relu_flips_vs_fp64": fl64}), flush=True)
            del m, flat, ctx
            engine.ROLE_PREC.clear()


if __name__ == "__main__":
    main()
