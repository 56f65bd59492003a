"""GEMM micro-benchmark on the C4 attention / projection / weight-gradient shapes: device time of
u2gnn_gemm per (precision, tile, split) via HIP events.  Usage: python tools/gemm_bench.py [prec ...]"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, ffp = 4864, 384, 1024
SHAPES = [  # name, M, N, K, ta, tb, [(split, tile), ...] (tile 129 = 128x128 with a 16-deep K step)
    ("QK^T  NT", Np, Np, dp, False, True, [(1, 128), (1, 256), (1, 129)]),
    ("dS    NT", Np, Np, dp, False, True, [(1, 128), (1, 256)], 6),   # dO.V^T, attention-dS epilogue (Pd)
    ("dSkb  NT", Np, Np, dp, False, True, [(1, 128), (1, 256)], 7),   # same, dropout keep bits instead of Pd
    ("P.V   NN", Np, dp, Np, False, False, [(4, 128), (4, 256), (4, 129)]),
    ("P.Vc  NN", Np, dp, Np, False, False, [(4, 256)], 8),   # A = signed probability image (clamp_a)
    ("dVc   TN", Np, dp, Np, True, False, [(4, 256)], 8),
    ("dV    TN", Np, dp, Np, True, False, [(4, 128), (4, 256), (4, 129)]),
    ("dWin  TN", 3 * dp, dp, Np, True, False, [(8, 128), (8, 129), (16, 129)]),
    ("dW1   TN", ffp, dp, Np, True, False, [(16, 128), (16, 129)]),
    ("QKV   NT", Np, 3 * dp, dp, False, True, [(1, 64), (1, 128), (1, 256)]),
    ("FFN1  NT", Np, ffp, dp, False, True, [(1, 64), (1, 128), (1, 256)]),
    ("FFN2  NT", Np, dp, ffp, False, True, [(1, 64), (1, 128), (2, 129)]),
    # epilogue GEMMs of the layer as the executor issues them (dropout p = 0.5 where it applies)
    ("QKVb  NT", Np, 3 * dp, dp, False, True, [(1, 64), (1, 128), (1, 256)], 1),
    ("FFN1d NT", Np, ffp, dp, False, True, [(1, 64), (1, 128), (1, 256)], 3),
    ("outpr NT", Np, dp, dp, False, True, [(1, 64), (1, 128), (1, 256)], 2),
    ("FFN2r NT", Np, dp, ffp, False, True, [(1, 64), (1, 128), (1, 256)], 2),
    ("dH    NN", Np, ffp, dp, False, False, [(1, 64), (1, 128), (1, 256)], 4),
    ("dO    NN", Np, dp, dp, False, False, [(1, 64), (1, 128), (1, 256)]),
    # shallow-K backward products (dH.W1 -> dX1, dQKV.W_in -> dX)
    ("dX1   NN", Np, dp, ffp, False, False, [(1, 64), (1, 128), (2, 128), (4, 256)]),
    ("dXin  NN", Np, dp, 3 * dp, False, False, [(1, 64), (1, 128), (2, 128), (4, 256)]),
    # the same weight products with the weight stored transposed (NT): the k-contiguous B image
    ("dH-T  NT", Np, ffp, dp, False, True, [(1, 64), (1, 128)], 4),
    ("dO-T  NT", Np, dp, dp, False, True, [(1, 64), (1, 128)]),
    ("dX1-T NT", Np, dp, ffp, False, True, [(1, 64), (1, 128)]),
    ("dXin-T NT", Np, dp, 3 * dp, False, True, [(1, 64), (1, 128)]),
]


ONLY = os.environ.get("GB_ONLY")  # e.g. "QK^T,dV": restrict to shapes whose name starts with one of these
REPS = int(os.environ.get("GB_REPS", "20"))


def run(prec):
    g = torch.Generator(device="cuda").manual_seed(0)
    for name, M, N, Kd, ta, tb, cfgs, *epi in SHAPES:
        epi = epi[0] if epi else 0
        ext = {}
        if epi == 6:
            ext = dict(epilogue=6, aux0=torch.rand(M, N, device="cuda", generator=g),
                       aux1=torch.rand(M, N, device="cuda", generator=g),
                       rowvec=torch.randn(M, device="cuda", generator=g), ld_aux=N)
        elif epi == 7:
            ext = dict(epilogue=6, aux0=torch.rand(M, N, device="cuda", generator=g), p_drop=0.5,
                       keep=torch.randint(-2**31, 2**31 - 1, (M, N // 32), device="cuda", dtype=torch.int32,
                                          generator=g),
                       rowvec=torch.randn(M, device="cuda", generator=g), ld_aux=N)
        if epi in (1, 2, 3, 4):
            ext = dict(epilogue=epi, p_drop=0.5 if epi != 1 else 0.0, seed=7, ld_aux=N, alpha=0.05, scale_cols=dp)
            if epi in (1, 2, 3):
                ext["bias"] = torch.randn(N, device="cuda", generator=g)
            if epi in (2, 4):
                ext["aux0"] = torch.randn(M, N, device="cuda", generator=g)
        if epi == 8:
            ext, epi = dict(clamp_a=True), 0
        if ONLY and not any(name.startswith(o) for o in ONLY.split(",")):
            continue
        A = torch.randn(Kd, M, device="cuda", generator=g) if ta else torch.randn(M, Kd, device="cuda", generator=g)
        if ext.get("clamp_a"):
            ref_a = A.clamp(min=0)
        B = torch.randn(N, Kd, device="cuda", generator=g) if tb else torch.randn(Kd, N, device="cuda", generator=g)
        first = None
        for split, tile in cfgs:
            if prec == "fp32" and tile == 256:
                continue
            C = torch.empty(split, M, N, device="cuda")
            f = lambda: K.gemm(A, B, C, M, N, Kd, A.shape[1], B.shape[1], N, trans_a=ta, trans_b=tb,  # noqa: E731
                               split_k=split, slab_stride=M * N, tile=tile, precision=prec, **ext)
            for _ in range(3):
                f()
            torch.cuda.synchronize()
            s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            s.record()
            for _ in range(REPS):
                f()
            e.record()
            torch.cuda.synchronize()
            us = s.elapsed_time(e) / REPS * 1e3
            A_ = ref_a if ext.get("clamp_a") else A
            ref = (A_.t() if ta else A_).double() @ (B.t() if tb else B).double()
            if epi in (1, 2, 3, 4):   # dropout epilogues: timing only
                ref = None
            elif epi == 6:
                ref = ext["aux1"].double() * ref - ext["aux0"].double() * ext["rowvec"].double()[:, None]
            elif epi == 7:
                w = ext["keep"].to(torch.int64) & 0xFFFFFFFF
                kb = ((w[:, :, None] >> torch.arange(32, device="cuda")) & 1).reshape(M, -1).double()
                ref = ext["aux0"].double() * (kb * ref * 2 - ext["rowvec"].double()[:, None])
            err = float("nan") if ref is None else ((C.sum(0).double() - ref).abs().max() / ref.abs().max()).item()
            same = ""
            if split == 1:
                if first is None:
                    first = C.clone()
                else:
                    same = f"  same bits as tile {cfgs[0][1]}: {torch.equal(C, first)}"
            print(f"{prec:7s} {name}  M={M:5d} N={N:5d} K={Kd:5d} split={split:2d} tile={tile:3d}: {us:8.1f} us "
                  f"{2.0 * M * N * Kd / us / 1e6:7.1f} TF/s  relerr {err:.1e}{same}")


if __name__ == "__main__":
    for p in (sys.argv[1:] or ["bf16x3", "fp32"]):
        run(p)
