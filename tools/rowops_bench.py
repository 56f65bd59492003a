"""Isolated device time of the C4 row-wise kernels (LayerNorm fwd/bwd, split-K slab reduce, attention
softmax) next to same-byte torch copies and a tiny launch: REPS launches captured in one HIP graph
(no host launch cost in the timing), replayed and timed with HIP events.
Usage: python tools/rowops_bench.py"""
import os
import sys

sys.path[:0] = [os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "graph-transformer_amd")]
import torch  # noqa: E402

from u2gnn_hip import kernels as K  # noqa: E402

Np, dp, d, N = 4864, 384, 367, 4776
REPS = 50


def t(fn):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    gr = torch.cuda.CUDAGraph()
    with torch.cuda.graph(gr):
        for _ in range(REPS):
            fn()
    gr.replay()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    gr.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3 / REPS


def main():
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(0)
    Z = torch.randn(Np, dp, device=dev, generator=g)
    Y = torch.empty_like(Z)
    dY = torch.randn(Np, dp, device=dev, generator=g)
    dZ = torch.empty_like(Z)
    dZd = torch.empty_like(Z)
    gam = torch.randn(dp, device=dev, generator=g)
    bet = torch.randn(dp, device=dev, generator=g)
    mean = torch.empty(Np, device=dev)
    rstd = torch.empty(Np, device=dev)
    MB = Np * dp * 4 / 1e6
    rows = []
    rows.append(("tiny fill (launch floor)", t(lambda: mean[:64].zero_()), 0))
    rows.append(("copy 7.5 MB", t(lambda: Y.copy_(Z)), 2 * MB))
    rows.append(("ln_fwd", t(lambda: K.layernorm_fwd(Z, dp, gam, bet, Y, dp, mean, rstd, N, Np, d, dp)), 2 * MB))
    K.layernorm_fwd(Z, dp, gam, bet, Y, dp, mean, rstd, N, Np, d, dp)
    rows.append(("ln_bwd (+drop)", t(lambda: K.layernorm_bwd(dY, dp, Z, dp, mean, rstd, gam, dZ, dp, dZd, dp, 0.5, 7,
                                                            N, Np, d, dp)), 4 * MB))
    rows.append(("ln_bwd", t(lambda: K.layernorm_bwd(dY, dp, Z, dp, mean, rstd, gam, dZ, dp, None, 0, 0.0, 7,
                                                    N, Np, d, dp)), 3 * MB))
    slabs = torch.randn(4, Np, dp, device=dev, generator=g)
    rows.append(("slab_reduce x4", t(lambda: K.slab_reduce(slabs, 4, Np * dp, Np, dp, dp, (Np, Np), (dp, dp), Y, dp)),
                 5 * MB))
    spare = torch.empty(3, Np, dp, device=dev)
    rows.append(("copy 22.4 MB", t(lambda: spare.copy_(slabs[:3])), 6 * MB))
    S = torch.randn(Np, Np, device=dev, generator=g)
    Pd = torch.empty_like(S)
    SMB = Np * Np * 4 / 1e6
    rows.append(("attn_softmax_fwd (signed)", t(lambda: K.attn_softmax_fwd(S, Np, None, Pd, Np, N, Np, N, Np, 0.5, 11)),
                 2 * SMB))
    rows.append(("copy 94.6 MB", t(lambda: Pd.copy_(S)), 2 * SMB))
    # neighbour-mode token rows (82 K): bandwidth, not launch latency, decides here
    R = 82176
    Zt = torch.randn(R, dp, device=dev, generator=g)
    Yt, dYt = torch.empty_like(Zt), torch.randn(R, dp, device=dev, generator=g)
    dZt, dZdt = torch.empty_like(Zt), torch.empty_like(Zt)
    mt, rt = torch.empty(R, device=dev), torch.empty(R, device=dev)
    TMB = R * dp * 4 / 1e6
    rows.append(("ln_fwd 82K rows", t(lambda: K.layernorm_fwd(Zt, dp, gam, bet, Yt, dp, mt, rt, R - 66, R, d, dp)), 2 * TMB))
    rows.append(("ln_bwd (+drop) 82K rows", t(lambda: K.layernorm_bwd(dYt, dp, Zt, dp, mt, rt, gam, dZt, dp, dZdt, dp, 0.5,
                                                                     7, R - 66, R, d, dp)), 4 * TMB))
    rows.append(("copy 126 MB", t(lambda: Yt.copy_(Zt)), 2 * TMB))
    for name, us, mb in rows:
        bw = f"{mb / us:6.2f} TB/s" if mb else ""
        print(f"{name:28s} {us:8.2f} us  {mb:7.1f} MB  {bw}", flush=True)


if __name__ == "__main__":
    main()
