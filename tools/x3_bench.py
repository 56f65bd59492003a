"""Micro-benchmark + correctness of the 256x256 x3 kernel (gemm_x3.hip, tile code 300) on the NT
attention products of a C4 layer (S = Q.K^T; dS = dO.V^T with the signed-image epilogue) against the
production fp32-operand BF16X3 kernel (gemm.hip).  Usage: python tools/x3_bench.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import _lib as E  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402

TILE = int(os.environ.get("XB_TILE", "301"))
REPS = int(os.environ.get("XB_REPS", "20"))


def to_x2(X):
    out = torch.empty(X.shape[0], 2 * X.shape[1], device=X.device, dtype=torch.bfloat16)
    K.split_x2(X, X.stride(0), out, out.stride(0), X.shape[0], X.shape[1])
    return out


def timeit(fn):
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(REPS):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / REPS * 1e3   # us


def err(a, ref):
    return ((a.double() - ref).abs().max() / ref.abs().max()).item()


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    for (Np, dp, N, d) in [(4864, 384, 4776, 367), (2048, 384, 2048, 384), (8192, 384, 8192, 384)]:
        FL = 2.0 * N * N * d
        QKV = torch.randn(Np, 3 * dp, device="cuda", generator=g)
        QKV2 = to_x2(QKV)
        Q, Kt, V = QKV[:, :dp], QKV[:, dp:2 * dp], QKV[:, 2 * dp:]
        Q2, K2 = QKV2[:, :2 * dp], QKV2[:, 2 * dp:4 * dp]
        ld3, ld3x = 3 * dp, QKV2.stride(0)
        out = torch.empty(Np, Np, device="cuda")
        out3 = torch.empty(Np, Np, device="cuda")
        ref = Q.double() @ Kt.double().t()
        base = lambda: K.gemm(Q, Kt, out, Np, Np, dp, ld3, ld3, Np, trans_b=True, precision="bf16x3", tile=256)  # noqa: E731
        x3 = lambda: K.gemm(Q2, K2, out3, Np, Np, dp, ld3x, ld3x, Np, trans_b=True, precision="bf16x3", tile=TILE)  # noqa: E731
        base()
        x3()
        torch.cuda.synchronize()
        eb, e3 = err(out, ref), err(out3, ref)
        tb, t3 = timeit(base), timeit(x3)
        print(f"QK^T Np={Np}: base {tb:7.1f} us {FL / tb / 1e6:6.1f} TF err {eb:.2e} | x3 {t3:7.1f} us "
              f"{FL / t3 / 1e6:6.1f} TF err {e3:.2e} | x{tb / t3:.2f}", flush=True)
        # dS = P o (dO V^T - delta) on the signed image (kept: P/(1-p), dropped: -P)
        dO = torch.randn(Np, dp, device="cuda", generator=g)
        dO2 = to_x2(dO)
        V2 = QKV2[:, 4 * dp:]
        Pimg = torch.rand(Np, Np, device="cuda", generator=g) * 1e-3
        Pimg = torch.where(torch.rand(Np, Np, device="cuda", generator=g) < 0.5, -Pimg, Pimg)
        delta = torch.randn(Np, device="cuda", generator=g)
        dsb = lambda: K.gemm(dO, V, out, Np, Np, dp, dp, ld3, Np, trans_b=True, epilogue=E.EPI_ATTN_DS_SIGNED,  # noqa: E731
                             aux0=Pimg, rowvec=delta, ld_aux=Np, p_drop=0.5, precision="bf16x3", tile=128)
        ds3 = lambda: K.gemm(dO2, V2, out3, Np, Np, dp, 2 * dp, ld3x, Np, trans_b=True,  # noqa: E731
                             epilogue=E.EPI_ATTN_DS_SIGNED, aux0=Pimg, rowvec=delta, ld_aux=Np, p_drop=0.5,
                             precision="bf16x3", tile=TILE)
        dsb()
        ds3()
        torch.cuda.synchronize()
        G = dO.double() @ V.double().t()
        x = Pimg.double()
        refd = torch.where(x < 0, x * delta.double()[:, None], x * (G - 0.5 * delta.double()[:, None]))
        eb, e3 = err(out, refd), err(out3, refd)
        tb, t3 = timeit(dsb), timeit(ds3)
        print(f"dS   Np={Np}: base {tb:7.1f} us {FL / tb / 1e6:6.1f} TF err {eb:.2e} | x3 {t3:7.1f} us "
              f"{FL / t3 / 1e6:6.1f} TF err {e3:.2e} | x{tb / t3:.2f}", flush=True)
        del QKV, QKV2, out, out3, ref, Pimg, G, x, refd


if __name__ == "__main__":
    main()
