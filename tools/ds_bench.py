"""Micro-benchmark: the attention dS GEMM of a C4 layer (dS = Pd o (dO.V^T - delta), signed
probability image, Np = 4864, dp = 384) and the scores GEMM S = Q K^T with the softmax row partials
(EPI_STORE_ROWSTAT) on each tile code, HIP-event device time per launch and algorithmic TFLOP/s (real
N = 4776, d = 367), with a bit-identity check of every tile against the first one.
Usage: python tools/ds_bench.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import _lib as E  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, N, d = 4864, 384, 4776, 367
FL = 2.0 * N * N * d


def timed(run, reps=20):
    for _ in range(3):
        run()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        run()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / reps * 1e3


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    dO = torch.randn(Np, dp, device="cuda", generator=g)
    QKV = torch.randn(Np, 3 * dp, device="cuda", generator=g)
    Pd = torch.rand(Np, Np, device="cuda", generator=g) * 1e-3
    delta = torch.randn(Np, device="cuda", generator=g)
    out = torch.empty(Np, Np, device="cuda")
    ref = None
    for tile in (128, 256, 64):
        def run():
            K.gemm(dO, QKV[:, 2 * dp:], out, Np, Np, dp, dp, 3 * dp, Np, trans_b=True,
                   epilogue=E.EPI_ATTN_DS_SIGNED, aux0=Pd, rowvec=delta, ld_aux=Np, p_drop=0.5,
                   precision="bf16x3", tile=tile)
        us = timed(run)
        same = "" if ref is None else f" identical to tile 128: {torch.equal(out, ref)}"
        if ref is None:
            ref = out.clone()
        print(f"dS tile {tile:3d}: {us:7.1f} us {FL / us / 1e6:6.1f} TF{same}", flush=True)
    S = torch.empty(Np, Np, device="cuda")
    rp = torch.empty(Np, 2 * (Np // 32), device="cuda")
    ref = None
    for tile in (256, 128):
        def run():
            K.gemm(QKV[:, :dp], QKV[:, dp:2 * dp], S, Np, Np, dp, 3 * dp, 3 * dp, Np, trans_b=True,
                   epilogue=E.EPI_STORE_ROWSTAT, rowpart=rp, n_valid=N, precision="bf16x3", tile=tile)
        S.zero_()
        rp.zero_()
        us = timed(run)
        cur = (S.clone(), rp[:, :2 * (Np // 64)].clone())
        same = "" if ref is None else \
            f" identical to tile 256: S {torch.equal(cur[0], ref[0])} rowstat {torch.equal(cur[1], ref[1])}"
        if ref is None:
            ref = cur
        print(f"QK tile {tile:3d}: {us:7.1f} us {FL / us / 1e6:6.1f} TF{same}", flush=True)


if __name__ == "__main__":
    main()
