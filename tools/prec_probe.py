"""Parity error of each GEMM role in plain bf16 (the rest bf16x3) on the C4 benchmark batch.

For every role of engine.ROLES (and a few combinations) run the C4 full batch (eval mode) through the
Python orchestration and report max|x - ref| / max(1, max|ref|) over scores, loss and every parameter
gradient against the fp32-MFMA run (itself checked against the oracle restatement once).
Usage (GPU box): python tools/prec_probe.py [--oracle] > gpurun_out/prec_probe.log
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def err(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).abs().max() / max(1.0, b.abs().max().item())).item()


def main():
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip import engine, native
    from u2gnn_hip import kernels as K
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.synthetic import collab_like
    native.set_enabled(False)
    dev = "cuda"
    np.random.seed(123)
    loaders = BatchLoader(collab_like(), 64, 16)
    hbs = [loaders() for _ in range(2)]
    torch.manual_seed(123)
    base = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1)
    sd = {k: v.detach().clone() for k, v in base.state_dict().items()}

    def run(prec, roles, hb, train=False):
        engine.ROLE_BF16.clear()
        engine.ROLE_BF16.update(roles)
        m = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1, precision=prec)
        m.load_state_dict(sd)
        m = m.to(dev).eval()
        flat = m.flatten_parameters()
        b = DeviceBatch.from_offsets(hb.input_x, hb.offsets, hb.X_concat, hb.labels, device=dev)
        scores, ctx = m.core.forward(b, train=train, need_ctx=True, seed=7)
        dsc = torch.empty_like(scores)
        loss = torch.zeros(1, device=dev)
        K.smoothed_ce(scores, b.labels, b.B, 3, 0.1, loss, dsc)
        m.core.backward(ctx, dsc, flat.grads)
        torch.cuda.synchronize()
        out = {"scores": scores.detach().cpu(), "loss": loss.cpu()}
        for n, _ in m.named_parameters():
            out[n] = flat.grads[n].detach().cpu().clone()
        return out

    def report(tag, o, ref):
        e = {k: err(o[k], ref[k]) for k in ref}
        worst = max(e, key=e.get)
        print(json.dumps({"tag": tag, "max_err": e[worst], "worst": worst,
                          "scores": e["scores"], "loss": e["loss"]}), flush=True)
        return e[worst]

    if "--mixed" in sys.argv:
        # joint error of the attention-backward roles in plain bf16, eval and train mode (same
        # dropout masks in every run: counter-based), several batches
        more = [loaders() for _ in range(2)]
        for bi, hb in enumerate(hbs + more):
            for train in (False, True):
                ref = run("fp32", [], hb, train)
                report(f"b{bi} train={train} bf16x3", run("bf16x3", [], hb, train), ref)
                for combo in (["ds", "dq", "dk"], ["ds", "dq", "dk", "dv"], ["dq", "dk"], ["dq", "dk", "dv"]):
                    report(f"b{bi} train={train} bf16:{'+'.join(combo)}", run("bf16x3", combo, hb, train), ref)
        return
    for bi, hb in enumerate(hbs):
        ref = run("fp32", [], hb)
        if "--oracle" in sys.argv and bi == 0:
            from oracle import u2gnn_oracle as O
            torch.set_num_threads(min(16, os.cpu_count()))
            sdg = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
            r = O.sup_forward(sdg, torch.from_numpy(hb.input_x), hb.offsets, torch.from_numpy(hb.X_concat), 1, 4,
                              train=False, slots=1)
            lref = O.soft_cross_entropy(r, O.label_smoothing(torch.from_numpy(hb.labels), 3))
            lref.backward()
            oref = {"scores": r.detach(), "loss": lref.detach().reshape(1)}
            for k, v in sdg.items():
                oref[k] = v.grad
            report(f"b{bi} fp32 vs oracle", ref, oref)
        report(f"b{bi} bf16x3", run("bf16x3", [], hb), ref)
        report(f"b{bi} bf16 (all)", run("bf16", [], hb), ref)
        for role in engine.ROLES:
            report(f"b{bi} bf16:{role}", run("bf16x3", [role], hb), ref)
        for combo in (["qk", "pv"], ["qk", "pv", "ds", "dv", "dq", "dk"],
                      ["in_proj", "out_proj", "ffn1", "ffn2"],
                      ["ffn2_dx", "ffn1_dx", "out_dx", "in_dx"],
                      ["ffn2_dw", "ffn1_dw", "out_dw", "in_dw"]):
            report(f"b{bi} bf16:{'+'.join(combo)}", run("bf16x3", combo, hb), ref)


if __name__ == "__main__":
    main()
