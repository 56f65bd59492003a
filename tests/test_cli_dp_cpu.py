"""Data parallelism of the drop-in CLIs (u2gnn_hip.cli, used by train_pytorch_U2GNN_{Sup,UnSup}.py
--world_size) on CPU with gloo, world 2.  The CLIs themselves need the GPU (no CPU fallback), so the
training step here is the oracle's (train_pytorch_U2GNN_Sup.py:149-161 restated, eval-mode dropout so
both sides are deterministic) driven by the CLI's own loop pieces: Run.next_batch (rank r takes batch r of
each global step and replays the others), Run.average_grads (the gradient mean before the clip),
Run.sum (the epoch loss over the ranks), step_seed (per-batch seeds by stream position).

Check: after three global steps both ranks hold the same parameters, equal to ONE process taking the
same six consecutive batches of the reference stream in pairs with the mean gradient; the epoch loss is
the sum of the six batch losses; the launcher (self_launch) reaches every rank."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import torch
import torch.multiprocessing as mp

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "graph-transformer_amd")
STEPS = 3



def _oracle_loss(params, hb, C):
    from oracle import u2gnn_oracle as O
    s = O.sup_forward(params, torch.from_numpy(hb.input_x), hb.offsets, torch.from_numpy(hb.X_concat), 1, 1,
                      train=False, slots=1)
    return O.soft_cross_entropy(s, O.label_smoothing(torch.from_numpy(hb.labels), C))


def _setup():
    import util
    from pytorch_U2GNN_Sup import TransformerU2GNN
    from u2gnn_hip.batching import BatchLoader, GraphStore
    graphs, C = util.load_data("MUTAG", False)
    np.random.seed(123)
    torch.manual_seed(123)
    m = TransformerU2GNN(7, 32, C, 1, 0.5, 1)
    params = {k: v.detach().clone().requires_grad_(True) for k, v in m.state_dict().items()}
    return BatchLoader(GraphStore(graphs), 4, 4), params, C


def _worker(rank, world, port, out_dir):
    sys.path[:0] = [PKG, REPO]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), TORCHELASTIC_USE_AGENT_STORE="True", WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    torch.set_num_threads(1)
    from oracle import u2gnn_oracle as O
    from u2gnn_hip.cli import Run, step_seed
    run = Run.init("gloo", device_type="cpu")
    assert (run.world, run.rank) == (world, rank)
    loader, params, C = _setup()
    names = list(params)
    state = {}
    acc = torch.zeros(1)
    idx = []
    for _ in range(STEPS):
        hb, i = run.next_batch(loader)
        idx.append(i)
        for p in params.values():
            p.grad = None
        loss = _oracle_loss(params, hb, C)
        loss.backward()
        run.average_grads(params.values())
        with torch.no_grad():
            O.clip_and_adam([params[n] for n in names], [params[n].grad for n in names], state, 5e-4)
        acc += loss.detach()
    total = run.sum(acc)
    np.savez(os.path.join(out_dir, f"r{rank}.npz"), total=total, idx=np.array(idx),
             seeds=np.array([step_seed(123, i) for i in idx], dtype=np.uint64),
             **{"p." + n: params[n].detach().numpy() for n in names})
    run.close()


def test_cli_dp_world2_equals_one_process_over_the_same_batches(tmp_path, rdzv_port):
    world = 2
    mp.spawn(_worker, args=(world, rdzv_port, str(tmp_path)), nprocs=world, join=True)
    r = [dict(np.load(os.path.join(tmp_path, f"r{i}.npz"))) for i in range(world)]
    assert list(r[0]["idx"]) == [0, 2, 4] and list(r[1]["idx"]) == [1, 3, 5]
    assert len(set(r[0]["seeds"].tolist() + r[1]["seeds"].tolist())) == 2 * STEPS
    sys.path[:0] = [PKG, REPO]
    from oracle import u2gnn_oracle as O
    loader, params, C = _setup()
    names = list(params)
    seq = [loader() for _ in range(world * STEPS)]     # the single stream, consecutive batches
    state, total = {}, 0.0
    for s in range(STEPS):
        grads = []
        for hb in seq[world * s: world * (s + 1)]:
            for p in params.values():
                p.grad = None
            loss = _oracle_loss(params, hb, C)
            loss.backward()
            total += float(loss)
            grads.append({n: params[n].grad.clone() for n in names})
        mean = [sum(g[n] for g in grads) / world for n in names]
        with torch.no_grad():
            O.clip_and_adam([params[n] for n in names], mean, state, 5e-4)
    for n in names:
        assert np.array_equal(r[0]["p." + n], r[1]["p." + n]), n
        assert np.allclose(r[0]["p." + n], params[n].detach().numpy(), rtol=1e-6, atol=1e-7), n
    assert abs(float(r[0]["total"]) - total) <= 1e-5 * abs(total)
    assert float(r[0]["total"]) == float(r[1]["total"])


def test_self_launch_starts_every_rank(tmp_path):
    """--world_size N without a launcher: the CLI runs torch.distributed.run on itself as a child."""
    script = tmp_path / "probe.py"
    script.write_text(textwrap.dedent(f"""
        import os, sys
        sys.path[:0] = [{PKG!r}, {REPO!r}]
        from u2gnn_hip.cli import self_launch
        rc = self_launch(2, __file__, sys.argv[1:])
        if rc is not None:
            sys.exit(rc)
        print("rank", os.environ["RANK"], "of", os.environ["WORLD_SIZE"], sys.argv[1:], flush=True)
    """))
    r = subprocess.run([sys.executable, str(script), "--x", "1"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = sorted(x for x in r.stdout.splitlines() if x.startswith("rank "))
    assert lines == ["rank 0 of 2 ['--x', '1']", "rank 1 of 2 ['--x', '1']"]
