"""Data-parallel path on real GPUs over RCCL (backend "nccl"), world_size 2 — runs only where at
least two devices are visible (the driver's multi-GPU node; skipped on a one-GPU box).

One C4-shaped training step per rank (its own batch of the single reference stream) through the
production path: the native layer executor with the parameter-gradient side stream and the
per-layer all-reduce issued under the backward (OverlappedGradAllReduce, bench.py's default for
N > 1) must leave exactly the same flat gradients, bit for bit, as the same step with the bucketed
all-reduce after the backward (GradAllReduce); both ranks must hold identical gradients and, after
clip + Adam, identical parameters."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def _worker(rank, world, port, out_dir):
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True")
    import u2gnn_hip  # noqa: F401  (hardware queues before HIP starts)
    import torch.distributed as dist
    dev = torch.device("cuda", rank)
    torch.cuda.set_device(dev)
    from u2gnn_hip.engine import side_stream
    side_stream(dev)
    dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.dp import GradAllReduce, OverlappedGradAllReduce, broadcast_params, rank_batches
    from u2gnn_hip.synthetic import collab_like
    from u2gnn_hip.train import SupTrainer

    np.random.seed(123)
    host = rank_batches(BatchLoader(collab_like(seed=0), 64, 16), world, rank, 1)   # C4 size: side stream on
    b = DeviceBatch.from_offsets(host[0].input_x, host[0].offsets, host[0].X_concat, host[0].labels, device=dev)
    out = {}
    for mode in ("overlap", "after"):
        torch.manual_seed(123)
        m = TransformerU2GNN(367, 1024, 3, 2, 0.5, 1, precision="bf16x3").to(dev).train()
        tr = SupTrainer(m, lr=5e-4, max_norm=0.5, seed=99 + rank)
        broadcast_params(tr.flat)
        if mode == "overlap":
            ar = OverlappedGradAllReduce(tr.flat)
            m.core.stack.grad_ready = ar.layer_done
            tr.grad_sync = ar
        else:
            tr.grad_sync = GradAllReduce(bucket_mb=8.0)
        tr.forward_backward(b, train=True)
        tr.grad_sync(tr.flat)
        torch.cuda.synchronize()
        g = tr.flat.gflat.detach().cpu().clone()
        tr.opt.step()
        torch.cuda.synchronize()
        out[mode] = (g.numpy(), tr.flat.flat.detach().cpu().numpy())
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), g_overlap=out["overlap"][0], g_after=out["after"][0],
             p_overlap=out["overlap"][1], p_after=out["after"][1])
    dist.destroy_process_group()


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2,
                    reason="needs two GPUs (RCCL over xGMI)")
def test_rccl_overlapped_allreduce_matches_bucketed(tmp_path, rdzv_port):
    world = 2
    mp.spawn(_worker, args=(world, rdzv_port, str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(os.path.join(tmp_path, f"r{i}.npz"))) for i in range(world)]
    for i in range(world):
        assert np.array_equal(r[i]["g_overlap"], r[i]["g_after"])
        assert np.array_equal(r[i]["p_overlap"], r[i]["p_after"])
    assert np.array_equal(r[0]["g_overlap"], r[1]["g_overlap"])
    assert np.array_equal(r[0]["p_overlap"], r[1]["p_overlap"])
    assert np.isfinite(r[0]["g_overlap"]).all() and np.abs(r[0]["g_overlap"]).max() > 0
