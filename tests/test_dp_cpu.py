"""Data-parallel plumbing on CPU with gloo, world_size 2 (RCCL is exercised on the GPU box by
bench.py under torch.distributed.run).  Checks: each rank's batches are exactly the consecutive
batches of the single reference stream, and the bucketed gradient all-reduce leaves every rank
with the mean of the per-rank gradients (computed here with the oracle)."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import util
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader, GraphStore
    from u2gnn_hip.core import FlatParams
    from u2gnn_hip.dp import GradAllReduce, OverlappedGradAllReduce, broadcast_params, rank_batches

    graphs, C = util.load_data("MUTAG", False)
    np.random.seed(123)
    mine = rank_batches(BatchLoader(GraphStore(graphs), 4, 4), world, rank, 2)
    torch.manual_seed(123 + rank)             # different init per rank -> broadcast must fix it
    m = TransformerU2GNN(7, 32, C, 1, 0.5, 1)
    flat = FlatParams(m)
    broadcast_params(flat)
    sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    b = mine[1]                                # second global step
    s = O.sup_forward(sd, torch.from_numpy(b.input_x), b.offsets, torch.from_numpy(b.X_concat), 1, 1, False, slots=1)
    loss = O.soft_cross_entropy(s, O.label_smoothing(torch.from_numpy(b.labels), C))
    loss.backward()
    for n in flat.names:
        flat.grads[n].copy_(sd[n].grad)
    GradAllReduce(bucket_mb=0.01)(flat)
    # overlapped form on a 2-timestep, 2-layer model with per-rank random gradients: per-layer
    # regions in backward order (as EncoderStack.grad_ready issues them), the head at the end;
    # must give the same buffer as the bucketed all-reduce, bit for bit
    m2 = TransformerU2GNN(7, 32, C, 2, 0.5, 2)
    f2 = FlatParams(m2)
    f2.gflat.copy_(torch.randn(f2.gflat.numel(), generator=torch.Generator().manual_seed(7 + rank)))
    mine_g = f2.gflat.clone()
    GradAllReduce(bucket_mb=0.001)(f2)
    g_after = f2.gflat.clone()
    f2.gflat.copy_(mine_g)
    ar = OverlappedGradAllReduce(f2)
    for l in reversed(range(2)):
        for t in reversed(range(2)):
            ar.layer_done(f"u2gnn_layers.{l}.layers.{t}.")
    ar(f2)
    assert torch.equal(f2.gflat, g_after)
    assert not ar.pending and not ar.launched
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), g=flat.gflat.numpy(), p=flat.flat.numpy(),
             ix=np.concatenate([x.input_x.ravel() for x in mine]))
    dist.destroy_process_group()


def test_gloo_world2_batches_and_grad_average(tmp_path):
    world = 2
    mp.spawn(_worker, args=(world, _free_port(), str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(os.path.join(tmp_path, f"r{i}.npz"))) for i in range(world)]
    assert np.array_equal(r[0]["g"], r[1]["g"]) and np.array_equal(r[0]["p"], r[1]["p"])
    # single-process reference: the same stream, 4 consecutive batches, mean grad of step 2
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    import util
    from oracle import u2gnn_oracle as O
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader, GraphStore
    graphs, C = util.load_data("MUTAG", False)
    np.random.seed(123)
    bl = BatchLoader(GraphStore(graphs), 4, 4)
    seq = [bl() for _ in range(4)]
    assert np.array_equal(r[0]["ix"], np.concatenate([seq[0].input_x.ravel(), seq[2].input_x.ravel()]))
    assert np.array_equal(r[1]["ix"], np.concatenate([seq[1].input_x.ravel(), seq[3].input_x.ravel()]))
    torch.manual_seed(123)
    m = TransformerU2GNN(7, 32, C, 1, 0.5, 1)
    grads = []
    for b in seq[2:4]:
        sd = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
        s = O.sup_forward(sd, torch.from_numpy(b.input_x), b.offsets, torch.from_numpy(b.X_concat), 1, 1, False,
                          slots=1)
        O.soft_cross_entropy(s, O.label_smoothing(torch.from_numpy(b.labels), C)).backward()
        grads.append(torch.cat([sd[n].grad.reshape(-1) for n, _ in m.named_parameters()]))
    mean = ((grads[0] + grads[1]) / 2).numpy()
    # flat buffer pads each tensor to 4 floats; compare the packed entries
    off, got = 0, []
    for n, p in m.named_parameters():
        got.append(r[0]["g"][off:off + p.numel()])
        off += (p.numel() + 3) // 4 * 4
    assert np.allclose(np.concatenate(got), mean, rtol=1e-5, atol=1e-6)
