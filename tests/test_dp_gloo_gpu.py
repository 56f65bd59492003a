"""The product's own gradient exchange at world 2 on ONE GPU (VERDICT r4 missing #2): two ranks on cuda:0
over gloo, which reduces CUDA tensors in stream order (each collective waits for the stream current at the
call, the caller's stream waits for the collective), so the same code paths run as over RCCL on a node:

* C4 (U2GNN-Sup COLLAB): bench.py's N > 1 path -- the native layer executor with the parameter-gradient
  side stream, OverlappedGradAllReduce wired as stack.grad_ready (each layer's region all-reduced from the
  stream that wrote it, under the next layer's backward), then clip + Adam;
* C5 (U2GNN-UnSup REDDIT-M5K): UnSupGradSync, eager -- the encoder all-reduce and the ss.weight compact-row
  all-gather folded into the dense gradient, then clip + Adam.

Each rank trains batch r of the first global step of the single reference stream (dp.rank_batches) with
its own dropout seed.  Asserted: both ranks hold bit-identical gradients and parameters, equal to ONE
process taking the same two batches with the same seeds and stepping once with the mean gradient
(SURVEY.md §8(e) parity check; train_pytorch_U2GNN_Sup.py:159-161, train_pytorch_U2GNN_UnSup.py:155-159).
Sup: bit for bit.  UnSup: the encoder gradient bit for bit; the ss.weight rows within 1e-6 (the exchange folds
label and sample rows rank by rank, the single process adds them per batch -- a different fp32 order) and so
the clip norm and the post-Adam parameters within 1e-5."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WORLD = 2
SEED = {"c4": 1000, "c5": 2000}



def _c4_setup(world, rank, dev):
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.dp import rank_batches
    from u2gnn_hip.synthetic import collab_like
    from u2gnn_hip.train import SupTrainer
    np.random.seed(123)
    h = rank_batches(BatchLoader(collab_like(seed=0), 64, 16), world, rank, 1)[0]
    b = DeviceBatch.from_offsets(h.input_x, h.offsets, h.X_concat, h.labels, device=dev)
    torch.manual_seed(123)
    m = TransformerU2GNN(367, 1024, 3, 4, 0.5, 1, precision="bf16x3").to(dev).train()
    return b, SupTrainer(m, lr=5e-4, max_norm=0.5)


def _c5_setup(world, rank, dev):
    from pytorch_U2GNN_UnSup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.dp import rank_batches
    from u2gnn_hip.synthetic import reddit5k_like
    from u2gnn_hip.unsup import UnSupTrainer
    store = reddit5k_like(seed=0)
    V = int(store.node_start[-1])
    np.random.seed(123)
    h = rank_batches(BatchLoader(store, 4, 16, with_input_y=True), world, rank, 1)[0]
    torch.manual_seed(123)
    m = TransformerU2GNN(feature_dim_size=4, ff_hidden_size=1024, dropout=0.5, num_self_att_layers=4,
                         vocab_size=V, sampled_num=512, num_U2GNN_layers=1, device=dev, precision="bf16x3")
    draws = [m.ss.draw_samples() for _ in range(world)]   # one draw per batch of the global step, in order
    m = m.to(dev).train()
    b = DeviceBatch.from_offsets(h.input_x, h.offsets, h.X_concat, None, device=dev, input_y=h.input_y)
    sid = torch.from_numpy(np.asarray(draws[rank], dtype=np.int64)).to(dev)
    return b, sid, UnSupTrainer(m, lr=5e-3, max_norm=0.5), store


def _worker(rank, world, port, out_dir, case):
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True")
    import u2gnn_hip  # noqa: F401  (hardware queues before HIP starts)
    import torch.distributed as dist
    dev = torch.device("cuda", 0)   # both ranks on the one GPU
    torch.cuda.set_device(dev)
    from u2gnn_hip.engine import side_stream
    side_stream(dev)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from u2gnn_hip.dp import OverlappedGradAllReduce, UnSupGradSync, broadcast_params, max_batch_nodes
    if case == "c4":
        b, tr = _c4_setup(world, rank, dev)
        broadcast_params(tr.flat)
        ar = OverlappedGradAllReduce(tr.flat)
        tr.m.core.stack.grad_ready = ar.layer_done
        tr.grad_sync = ar
        tr.forward_backward(b, train=True, seed=SEED[case] + rank)
        tr.grad_sync(tr.flat)
        g = tr.flat.gflat.detach().cpu().clone()
        tr.opt.step()
    else:
        b, sid, tr, store = _c5_setup(world, rank, dev)
        broadcast_params(tr.flat)
        sync = UnSupGradSync(tr.flat, max_batch_nodes(store.node_start, 4))
        tr.grad_sync = tr.row_sync = sync
        tr.forward_backward(b, sid, train=True, seed=SEED[case] + rank)
        tr.grad_sync(tr.flat)
        g = tr.flat.gflat.detach().cpu().clone()
        tr.opt.step()
        tr.clear_row_grads()
        assert float(tr.flat.grads["ss.weight"].abs().max()) == 0.0
    torch.cuda.synchronize()
    np.savez(os.path.join(out_dir, f"{case}_r{rank}.npz"), g=g.numpy(), p=tr.flat.flat.detach().cpu().numpy())
    dist.destroy_process_group()


def _single_process(case, world):
    """One process, the same two batches and seeds, the mean gradient, one clip + Adam step."""
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    dev = torch.device("cuda", 0)
    gs = []
    tr = None
    for r in range(world):
        if case == "c4":
            b, t = _c4_setup(world, r, dev)
            tr = tr or t
            tr.flat.gflat.zero_()
            tr.forward_backward(b, train=True, seed=SEED[case] + r)
        else:
            b, sid, t, _ = _c5_setup(world, r, dev)
            tr = tr or t
            tr.flat.gflat.zero_()
            tr.forward_backward(b, sid, train=True, seed=SEED[case] + r)
        gs.append(tr.flat.gflat.detach().clone())
        if case == "c5":
            tr.clear_row_grads()
    tr.flat.gflat.copy_((gs[0] + gs[1]) * (1.0 / world))
    g = tr.flat.gflat.detach().cpu().clone()
    tr.opt.step()
    torch.cuda.synchronize()
    return g.numpy(), tr.flat.flat.detach().cpu().numpy(), tr


@pytest.mark.parametrize("case", ["c4", "c5"])
def test_gloo_world2_on_one_gpu_equals_one_process_mean_step(tmp_path, case, rdzv_port):
    mp.spawn(_worker, args=(WORLD, rdzv_port, str(tmp_path), case), nprocs=WORLD, join=True)
    r = [dict(np.load(os.path.join(tmp_path, f"{case}_r{i}.npz"))) for i in range(WORLD)]
    assert np.array_equal(r[0]["g"], r[1]["g"]), "ranks hold different gradients"
    assert np.array_equal(r[0]["p"], r[1]["p"]), "ranks hold different parameters"
    g_ref, p_ref, tr = _single_process(case, WORLD)
    assert np.isfinite(g_ref).all() and np.abs(g_ref).max() > 0
    if case == "c4":
        assert np.array_equal(r[0]["g"], g_ref)
        assert np.array_equal(r[0]["p"], p_ref)
        return
    gw = tr.flat.grads["ss.weight"]
    lo = (gw.data_ptr() - tr.flat.gflat.data_ptr()) // 4
    hi = lo + gw.numel()
    assert np.array_equal(r[0]["g"][:lo], g_ref[:lo]) and np.array_equal(r[0]["g"][hi:], g_ref[hi:])
    dw = np.abs(r[0]["g"][lo:hi] - g_ref[lo:hi]).max() / max(1.0, np.abs(g_ref[lo:hi]).max())
    assert dw <= 1e-6, f"ss.weight gradient rows {dw:.3g}"
    dp_ = np.abs(r[0]["p"] - p_ref).max() / max(1.0, np.abs(p_ref).max())
    assert dp_ <= 1e-5, f"post-Adam parameters {dp_:.3g}"
