"""Micro-benchmark: the N^2 attention products of a C4 layer (Np = 4864, dp = 384) on the fp32-operand
BF16X3 kernel (gemm.hip) vs the pre-split x2 kernel (gemm_x2.hip), HIP-event device time per launch
and algorithmic TFLOP/s (real N = 4776, d = 367).  Usage: python tools/x2_bench.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import _lib as E  # noqa: E402
from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, N, d = 4864, 384, 4776, 367
REPS = int(os.environ.get("XB_REPS", "20"))
FL = 2.0 * N * N * d


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


def main():
    g = torch.Generator(device="cuda").manual_seed(0)
    r = lambda *s: torch.randn(*s, device="cuda", generator=g)  # noqa: E731
    QKV, Pd, dO, S = r(Np, 3 * dp), r(Np, Np).abs() * 1e-3, r(Np, dp), r(Np, Np)
    QKV2, Pd2, dO2 = to_x2(QKV), to_x2(Pd), to_x2(dO)
    Q, Kt, V = QKV[:, :dp], QKV[:, dp:2 * dp], QKV[:, 2 * dp:]
    Q2, K2, V2 = QKV2[:, :2 * dp], QKV2[:, 2 * dp:4 * dp], QKV2[:, 4 * dp:]
    out = torch.empty(Np, Np, device="cuda")
    out2 = torch.empty(Np, 2 * Np, device="cuda", dtype=torch.bfloat16)
    slabs = torch.empty(4, Np, dp, device="cuda")
    delta, rs = r(Np), torch.stack([S.max(1).values, torch.full((Np,), 1e-3, device="cuda")], 1).contiguous()
    ld3, ld3x = 3 * dp, QKV2.stride(0)
    rows = []

    CODES = [int(c) for c in os.environ.get("XB_CODES", "256,130,261,263").split(",")]

    def row(name, fa, fb):
        ta = timeit(fa)
        best = None
        for code in CODES:
            try:
                tb = timeit(lambda: fb(code))
            except Exception as e:   # tile code not applicable to this shape
                print(f"{name:8s} x2[{code}] n/a ({e})", flush=True)
                continue
            print(f"{name:8s} bf16x3 {ta:7.1f} us {FL / ta / 1e6:6.1f} TF | x2[{code}] {tb:7.1f} us "
                  f"{FL / tb / 1e6:6.1f} TF | x{ta / tb:.2f}", flush=True)
            best = tb if best is None else min(best, tb)
        rows.append((name, ta, best))

    row("QK^T", lambda: K.gemm(Q, Kt, out, Np, Np, dp, ld3, ld3, Np, trans_b=True, precision="bf16x3", tile=256),
        lambda c: K.gemm(Q2, K2, out, Np, Np, dp, ld3x, ld3x, Np, trans_b=True, precision="bf16x3", tile=c))
    row("P.V", lambda: K.gemm(Pd, V, slabs, Np, dp, Np, Np, ld3, dp, precision="bf16x3", tile=256, split_k=4,
                              slab_stride=Np * dp, clamp_a=True),
        lambda c: K.gemm(Pd2, V2, slabs, Np, dp, Np, 2 * Np, ld3x, dp, precision="bf16x3", tile=c, split_k=4,
                       slab_stride=Np * dp))
    row("dV", lambda: K.gemm(Pd, dO, slabs, Np, dp, Np, Np, dp, dp, trans_a=True, precision="bf16x3", tile=256,
                             split_k=4, slab_stride=Np * dp, clamp_a=True),
        lambda c: K.gemm(Pd2, dO2, slabs, Np, dp, Np, 2 * Np, 2 * dp, dp, trans_a=True, precision="bf16x3", tile=c,
                       split_k=4, slab_stride=Np * dp))
    row("dQ", lambda: K.gemm(Pd, Kt, slabs, Np, dp, Np, Np, ld3, dp, precision="bf16x3", tile=256, split_k=4,
                             slab_stride=Np * dp),
        lambda c: K.gemm(Pd2, K2, slabs, Np, dp, Np, 2 * Np, ld3x, dp, precision="bf16x3", tile=c, split_k=4,
                       slab_stride=Np * dp))
    row("dS", lambda: K.gemm(dO, V, out, Np, Np, dp, dp, ld3, Np, trans_b=True, epilogue=E.EPI_ATTN_DS_SIGNED,
                             aux0=Pd, rowvec=delta, ld_aux=Np, p_drop=0.5, precision="bf16x3", tile=128),
        lambda c: K.gemm(dO2, V2, None, Np, Np, dp, 2 * dp, ld3x, Np, trans_b=True, epilogue=E.EPI_ATTN_DS_RECOMP,
                       aux0=S, ld_aux=Np, rowvec=delta, rowstat=rs, m_valid=N, n_valid=N, p_drop=0.5, seed=3,
                       precision="bf16x3", tile=c, Cx2=out2, ldcx2=2 * Np))
    sm_old = timeit(lambda: K.attn_softmax_fwd(S, Np, None, out, Np, N, Np, N, Np, 0.5, 9))
    sm_new = timeit(lambda: K.attn_softmax_x2_fwd(S, Np, out2, 2 * Np, rs, N, Np, N, Np, 0.5, 9))
    print(f"softmax  signed {sm_old:7.1f} us | x2 {sm_new:7.1f} us", flush=True)
    ta = sum(a for _, a, _ in rows) + sm_old
    tb = sum(b for _, _, b in rows) + sm_new
    print(f"total (QK, PV, dV, dQ, dS, softmax; dK ~ dV) bf16x3 {ta:.1f} us | x2 {tb:.1f} us")


if __name__ == "__main__":
    main()
