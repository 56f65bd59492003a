"""HIP-graph replay of training steps (u2gnn_hip.train.StepGraphs, ABI v6 device step state).

* the seed epoch: every dropout-drawing kernel mixes the device epoch into its seed (mask ==
  the plain mask of seed ^ epoch * golden; epoch 0 == no change);
* Adam with the device schedule (u2gnn_adam_dev) == the host-schedule Adam;
* replayed steps == eager steps (eval mode: no dropout, so every step is deterministic), for the
  supervised C4-shaped model and the UnSup sampled-softmax model;
* in train mode successive replays of one captured graph draw different masks."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

GOLD = 0x9E3779B97F4A7C15


def test_seed_epoch_mixes_into_every_mask():
    from u2gnn_hip import kernels as K
    seed = 0x1234567890ABCDEF
    m0 = K.dropout_mask(seed, 300, 70, 0.5)
    ep = torch.zeros(1, device="cuda", dtype=torch.int64)
    K.set_seed_epoch(ep)
    try:
        assert torch.equal(K.dropout_mask(seed, 300, 70, 0.5), m0)          # epoch 0: unchanged
        K.step_advance(ep, None)
        K.step_advance(ep, None)
        assert int(ep.item()) == 2
        m2 = K.dropout_mask(seed, 300, 70, 0.5)
    finally:
        K.set_seed_epoch(None)
    mixed = (seed ^ ((2 * GOLD) & 0xFFFFFFFFFFFFFFFF)) & 0xFFFFFFFFFFFFFFFF
    assert torch.equal(m2, K.dropout_mask(mixed, 300, 70, 0.5))
    assert not torch.equal(m2, m0)


def test_adam_device_schedule_matches_host_schedule():
    from u2gnn_hip import kernels as K
    g = torch.Generator(device="cuda").manual_seed(2)
    n = 10000
    p0 = torch.randn(n, device="cuda", generator=g)
    grads = [torch.randn(n, device="cuda", generator=g) for _ in range(5)]
    outs = []
    for dev_sched in (False, True):
        p, m, v = p0.clone(), torch.zeros(n, device="cuda"), torch.zeros(n, device="cuda")
        sq = torch.empty(1, device="cuda")
        ws = torch.empty(1024, device="cuda")
        t = torch.zeros(1, device="cuda", dtype=torch.int64)
        lr = torch.full((1,), 5e-4, device="cuda", dtype=torch.float64)
        for s, gr in enumerate(grads, 1):
            K.sqnorm(gr, n, ws, sq)
            if dev_sched:
                K.step_advance(None, t)
                K.adam_dev(p, gr, m, v, n, sq, 0.5, 0.9, 0.999, 1e-8, lr, t)
            else:
                K.adam(p, gr, m, v, n, sq, 0.5, 0.9, 0.999, 1e-8, 5e-4 / (1 - 0.9 ** s), (1 - 0.999 ** s) ** 0.5)
        outs.append(p)
    assert ((outs[0] - outs[1]).abs().max() / outs[0].abs().max()).item() <= 1e-6


def _sup(N_graphs=16, T=2):
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.synthetic import collab_like
    np.random.seed(123)
    loader = BatchLoader(collab_like(), N_graphs, 16)
    batches = [loader() for _ in range(2)]
    bs = [DeviceBatch.from_offsets(h.input_x, h.offsets, h.X_concat, h.labels, device="cuda") for h in batches]
    torch.manual_seed(123)
    return TransformerU2GNN(367, 1024, 3, T, 0.5, 1, precision="bf16x3"), bs


def test_sup_graph_replay_equals_eager_steps():
    from u2gnn_hip.train import StepGraphs, SupTrainer
    base, bs = _sup()
    sd = {k: v.clone() for k, v in base.state_dict().items()}
    finals = []
    for graphed in (False, True):
        base.load_state_dict(sd)
        m = base.to("cuda").eval()
        tr = SupTrainer(m, lr=5e-4)
        runner = StepGraphs(tr) if graphed else None
        losses = []
        for i in range(5):
            b = bs[i % 2]
            loss = runner.step(b, False) if graphed else tr.step(b, False)
            losses.append(float(loss.item()))
        if runner is not None:
            runner.close()
            assert tr.opt.step_count == 5
        torch.cuda.synchronize()
        finals.append((np.array(losses), tr.flat.flat.detach().cpu().clone()))
    (l0, p0), (l1, p1) = finals
    assert np.allclose(l0, l1, rtol=1e-6, atol=0)
    assert ((p0 - p1).abs().max() / p0.abs().max()).item() <= 1e-6


def test_graph_replays_draw_fresh_dropout_masks():
    from u2gnn_hip.train import StepGraphs, SupTrainer
    m, bs = _sup(8, 1)
    m = m.to("cuda").train()
    tr = SupTrainer(m, lr=0.0)   # lr 0: the parameters never move, only the masks can change the loss
    runner = StepGraphs(tr)
    try:
        losses = [float(runner.step(bs[0]).item()) for _ in range(4)]
        assert int(runner.epoch.item()) == 4
    finally:
        runner.close()
    assert len(set(losses)) == 4, losses


def test_unsup_graph_replay_equals_eager_steps():
    import util
    from pytorch_U2GNN_UnSup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader, GraphStore
    from u2gnn_hip.core import DeviceBatch
    from u2gnn_hip.train import StepGraphs
    from u2gnn_hip.unsup import UnSupTrainer
    graphs, _ = util.load_data("PTC", False)
    store = GraphStore(graphs)
    V = int(store.node_start[-1])
    np.random.seed(123)
    loader = BatchLoader(store, 4, 4, with_input_y=True)
    hbs = [loader() for _ in range(2)]
    torch.manual_seed(123)
    model = TransformerU2GNN(feature_dim_size=store.X.shape[1], ff_hidden_size=256, dropout=0.5, num_self_att_layers=2,
                             vocab_size=V, sampled_num=512, num_U2GNN_layers=1, device="cuda", precision="bf16x3")
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    bs = [DeviceBatch.from_offsets(h.input_x, h.offsets, h.X_concat, None, device="cuda", input_y=h.input_y)
          for h in hbs]
    sids = [torch.from_numpy(model.ss.draw_samples()).cuda() for _ in hbs]
    finals = []
    for graphed in (False, True):
        model.load_state_dict(sd)
        model = model.to("cuda").eval()
        tr = UnSupTrainer(model, lr=5e-3, max_norm=0.5)
        runner = StepGraphs(tr) if graphed else None
        losses = []
        for i in range(4):
            args = (bs[i % 2], sids[i % 2], False)
            losses.append(float((runner.step(*args) if graphed else tr.step(*args)).item()))
        if runner is not None:
            runner.close()
        torch.cuda.synchronize()
        finals.append((np.array(losses), tr.flat.flat.detach().cpu().clone()))
    (l0, p0), (l1, p1) = finals
    assert np.allclose(l0, l1, rtol=1e-6, atol=0)
    assert ((p0 - p1).abs().max() / p0.abs().max()).item() <= 1e-6


def test_eager_steps_while_graphs_are_live_advance_adam():
    """once StepGraphs switches Adam to the device schedule, an eager trainer.step must
    still advance the device step count (a fresh t of 0 gave lr / (1 - b1^0) = inf).  Eager and
    replayed steps interleaved == five eager steps; the context manager releases the epoch."""
    from u2gnn_hip.train import StepGraphs, SupTrainer
    base, bs = _sup(8, 1)
    sd = {k: v.clone() for k, v in base.state_dict().items()}
    finals = []
    for mixed in (False, True):
        base.load_state_dict(sd)
        m = base.to("cuda").eval()
        tr = SupTrainer(m, lr=5e-4)
        losses = []
        if mixed:
            with StepGraphs(tr) as runner:
                for i in range(5):
                    b = bs[i % 2]
                    loss = tr.step(b, False) if i in (0, 1, 4) else runner.step(b, False)
                    losses.append(float(loss.item()))
                assert int(tr.opt.t_dev.item()) == 5
            assert tr.opt.t_dev is None and tr.opt.step_count == 5
        else:
            losses = [float(tr.step(bs[i % 2], False).item()) for i in range(5)]
        torch.cuda.synchronize()
        finals.append((np.array(losses), tr.flat.flat.detach().cpu().clone()))
    (l0, p0), (l1, p1) = finals
    assert np.isfinite(p1.numpy()).all()
    assert np.allclose(l0, l1, rtol=1e-6, atol=0)
    assert ((p0 - p1).abs().max() / p0.abs().max()).item() <= 1e-6
