"""Data-parallel plumbing on CPU with gloo, world_size 2 (RCCL is exercised on the GPU box by
bench.py under torch.distributed.run).  Checks: each rank's batches are exactly the consecutive
batches of the single reference stream, and the bucketed gradient all-reduce leaves every rank
with the mean of the per-rank gradients (computed here with the oracle)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))



def _worker(rank, world, port, out_dir):
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True")
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
    # buckets of adjacent layers (round 6): one bucket for this small model (the default 9 MB), a bucket per layer
    # (tiny), and every layer pair; the head joins the first bucket; twice each (the step resets the counters)
    for mb in (9.0, 1e-5, 0.02):
        ar = OverlappedGradAllReduce(f2, bucket_mb=mb)
        for rep in range(2):
            f2.gflat.copy_(mine_g)
            for l in reversed(range(2)):
                for t in reversed(range(2)):
                    ar.layer_done(f"u2gnn_layers.{l}.layers.{t}.")
            n_coll = len(ar.pending)
            ar(f2)
            assert torch.equal(f2.gflat, g_after), mb
            assert not ar.pending and not ar.launched
            assert n_coll == {9.0: 1, 1e-5: 4}.get(mb, n_coll), (mb, n_coll)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), g=flat.gflat.numpy(), p=flat.flat.numpy(),
             ix=np.concatenate([x.input_x.ravel() for x in mine]))
    dist.destroy_process_group()


def test_gloo_world2_batches_and_grad_average(tmp_path, rdzv_port):
    world = 2
    mp.spawn(_worker, args=(world, rdzv_port, str(tmp_path)), nprocs=world, join=True)
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


def _unsup_grads(rank_batch, sids, sd, W):
    """Oracle (train_pytorch_U2GNN_UnSup.py:149-157, eval mode): dense gradients of the summed
    sampled-softmax loss of one batch w.r.t. the encoder parameters and ss.weight."""
    from oracle import u2gnn_oracle as O
    enc = {k: v.detach().clone().requires_grad_(True) for k, v in sd.items()}
    w = W.detach().clone().requires_grad_(True)
    b = rank_batch
    loss = O.unsup_forward(enc, w, torch.from_numpy(b.input_x), torch.from_numpy(b.X_concat),
                           torch.from_numpy(b.input_y), torch.from_numpy(sids), 1, 1, train=False, slots=1).sum()
    loss.backward()
    return {k: v.grad for k, v in enc.items()}, w.grad


def _unsup_setup(world, rank, steps=2):
    import util
    from log_uniform import LogUniformSampler
    from pytorch_U2GNN_UnSup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader, GraphStore
    from u2gnn_hip.dp import rank_batches
    graphs, _ = util.load_data("PTC", False)
    store = GraphStore(graphs)
    V = int(store.node_start[-1])
    np.random.seed(123)
    mine = rank_batches(BatchLoader(store, 4, 4, with_input_y=True), world, rank, steps)
    sampler = LogUniformSampler(V)
    draws = [sampler.sample_set_order(64)[0] for _ in range(world * steps)]   # one draw per batch, in order
    my_sids = [np.asarray(draws[s * world + rank], dtype=np.int64) for s in range(steps)]
    torch.manual_seed(123)
    m = TransformerU2GNN(vocab_size=V, feature_dim_size=store.X.shape[1], ff_hidden_size=32, sampled_num=64,
                         num_self_att_layers=1, num_U2GNN_layers=1, dropout=0.5, device="cpu")
    return store, m, mine, my_sids


def _unsup_worker(rank, world, port, out_dir):
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True")
    import torch.distributed as dist
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from u2gnn_hip.core import FlatParams
    from u2gnn_hip.dp import UnSupGradSync, max_batch_nodes
    store, m, mine, my_sids = _unsup_setup(world, rank)
    flat = FlatParams(m, names=m.trainable_names())
    sd = {k: v.detach() for k, v in m.state_dict().items() if k.startswith("u2gnn_layers.")}
    b, sids = mine[1], my_sids[1]                       # second global step
    g_enc, g_w = _unsup_grads(b, sids, sd, m.ss.weight.detach().clone())
    for k, v in g_enc.items():
        flat.grads[k].copy_(v)
    # compact rows: label rows, then the sample rows not already counted among the labels
    lab = torch.from_numpy(b.input_y)
    smp = torch.from_numpy(sids)
    rows_lab = g_w.index_select(0, lab)
    rows_smp = g_w.index_select(0, smp) * (~torch.isin(smp, lab)).float()[:, None]
    sync = UnSupGradSync(flat, max_batch_nodes(store.node_start, 4))
    gW = flat.grads["ss.weight"]
    assert float(gW.abs().sum()) == 0.0            # zero between steps
    touched = sync.rows(lab, rows_lab, smp, rows_smp, gW)
    sync(flat)
    np.savez(os.path.join(out_dir, f"u{rank}.npz"), g=flat.gflat.numpy().copy())
    for ids in touched:                               # what UnSupTrainer.clear_row_grads does
        keep = ids >= 0
        gW[ids[keep]] = 0.0
    assert float(gW.abs().sum()) == 0.0
    dist.destroy_process_group()


def test_gloo_world2_unsup_sparse_row_exchange(tmp_path, rdzv_port):
    """Row e2: 2 ranks, each one UnSup batch + its own sample draw; after the encoder
    all-reduce and the ss.weight row all-gather, both ranks hold the same gradient, equal to the mean
    of the dense oracle gradients of the same 2 consecutive batches of the single stream."""
    world = 2
    mp.spawn(_unsup_worker, args=(world, rdzv_port, str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(os.path.join(tmp_path, f"u{i}.npz"))) for i in range(world)]
    assert np.array_equal(r[0]["g"], r[1]["g"])
    sys.path[:0] = [os.path.join(REPO, "graph-transformer_amd"), REPO]
    from u2gnn_hip.batching import BatchLoader  # noqa: F401  (path check)
    enc_sum, w_sum = None, None
    for rank in range(world):
        store, m, mine, my_sids = _unsup_setup(world, rank)
        sd = {k: v.detach() for k, v in m.state_dict().items() if k.startswith("u2gnn_layers.")}
        g_enc, g_w = _unsup_grads(mine[1], my_sids[1], sd, m.ss.weight.detach())
        enc_sum = g_enc if enc_sum is None else {k: enc_sum[k] + g_enc[k] for k in g_enc}
        w_sum = g_w if w_sum is None else w_sum + g_w
    names = m.trainable_names()
    off, got, ref = 0, [], []
    params = dict(m.named_parameters())
    for n in names:
        k = params[n].numel()
        got.append(r[0]["g"][off:off + k])
        ref.append(((w_sum if n == "ss.weight" else enc_sum[n]) / world).reshape(-1).numpy())
        off += (k + 3) // 4 * 4
    got, ref = np.concatenate(got), np.concatenate(ref)
    assert np.abs(ref).max() > 0
    assert np.allclose(got, ref, rtol=1e-5, atol=1e-6)
