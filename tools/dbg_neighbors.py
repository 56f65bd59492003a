import os, sys, numpy as np, torch
sys.path[:0] = ["graph-transformer_amd", "."]
from oracle import u2gnn_oracle as O
from pytorch_U2GNN_Sup import TransformerU2GNN
from u2gnn_hip.core import DeviceBatch
from u2gnn_hip import kernels as K
z = dict(np.load("tests/golden/imdbb_sup.npz"))
d, C = int(z["meta"][5]), int(z["meta"][6])
for prec, L, T, side in [("bf16x3", 2, 2, "1"), ("bf16x3", 2, 2, "0"), ("fp32", 2, 2, "1")]:
    from u2gnn_hip import engine
    engine.set_overlap(side == "1")
    torch.manual_seed(7)
    m = TransformerU2GNN(d, 256, C, T, 0.5, L, precision=prec, attention="neighbors")
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    m = m.to("cuda").eval()
    flat = m.flatten_parameters()
    b = DeviceBatch.from_offsets(z["b0_input_x"], z["b0_offsets"], z["b0_X"], z["b0_labels"], device="cuda")
    scores, ctx = m.core.forward(b, train=False, need_ctx=True, seed=0)
    dsc = torch.empty_like(scores); loss = torch.zeros(1, device="cuda")
    K.smoothed_ce(scores, b.labels, b.B, C, 0.1, loss, dsc)
    m.core.backward(ctx, dsc, flat.grads)
    ref = O.sup_forward(sd, torch.from_numpy(z["b0_input_x"]), z["b0_offsets"], torch.from_numpy(z["b0_X"]), L, T, train=False, attention="neighbors")
    lref = O.soft_cross_entropy(ref, O.label_smoothing(torch.from_numpy(z["b0_labels"]), C)); lref.backward()
    print(prec, L, T, "side", side, "scores", (scores.cpu() - ref.detach()).abs().max().item())
    for n, _ in m.named_parameters():
        a, r = flat.grads[n].cpu().double(), sd[n].grad.double()
        e = (a - r).abs().max().item() / max(1.0, r.abs().max().item())
        if e > 1e-4: print("   ", n, e, r.abs().max().item())
