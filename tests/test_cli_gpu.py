"""Integration: the drop-in CLIs run end-to-end on the GPU (1 epoch, capped steps) and write the
reference's stdout line and acc file."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "graph-transformer_amd")


def _run(script, extra, tmp_path, env=None, stderr=False):
    run = tmp_path / "run" / "x"
    run.mkdir(parents=True)
    cmd = [sys.executable, os.path.join(PKG, script), "--run_folder", str(run), "--num_epochs", "1"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600, env=dict(os.environ, **(env or {})))
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return (r.stdout, run, r.stderr) if stderr else (r.stdout, run)


@pytest.mark.parametrize("autograd", [False, True])
def test_sup_cli_mutag(tmp_path, autograd):
    out, run = _run("train_pytorch_U2GNN_Sup.py", ["--dataset", "MUTAG", "--model_name", "MUTAG", "--batch_size", "4",
                                                   "--num_neighbors", "4", "--ff_hidden_size", "128",
                                                   "--num_timesteps", "1"] + (["--autograd"] if autograd else []),
                    tmp_path)
    assert "| epoch   1 |" in out and "test acc" in out
    acc = run.parent / "runs_pytorch_U2GNN_Sup" / "MUTAG" / "checkpoints" / "model_acc.txt"
    assert acc.read_text().startswith("epoch 1 fold 1 acc ")


def test_unsup_cli_ptc(tmp_path):
    out, run = _run("train_pytorch_U2GNN_UnSup.py", ["--dataset", "PTC", "--model_name", "PTC", "--num_timesteps", "2",
                                                     "--max_steps", "20"], tmp_path)
    assert "| epoch   1 |" in out and "mean" in out
    acc = run.parent / "runs_pytorch_U2GNN_UnSup" / "PTC" / "checkpoints" / "model_acc.txt"
    assert acc.read_text().startswith("epoch 1 mean: ")


def _checksums(err):
    lines = sorted(x.split()[2:] for x in err.splitlines() if x.startswith("param_checksum rank "))
    return {int(x[0]): (x[1], x[2]) for x in lines}


@pytest.mark.parametrize("script,extra,head", [
    ("train_pytorch_U2GNN_Sup.py", ["--dataset", "MUTAG", "--model_name", "MUTAG", "--num_neighbors", "4",
                                    "--ff_hidden_size", "128", "--max_steps", "6"], "epoch 1 fold 1 acc "),
    ("train_pytorch_U2GNN_UnSup.py", ["--dataset", "PTC", "--model_name", "PTC", "--num_timesteps", "2",
                                      "--max_steps", "6"], "epoch 1 mean: ")])
def test_cli_world2_gloo_on_one_gpu(tmp_path, script, extra, head):
    """--world_size 2: the CLI launches two ranks itself (torch.distributed.run as a child); gloo lets both
    share this box's one GPU.  Rank 0 alone prints the epoch line and writes the acc file, and after the
    data-parallel steps both ranks hold the same parameters (clip + Adam run identically on
    every rank after the gradient average)."""
    out, run, err = _run(script, extra + ["--world_size", "2", "--dist_backend", "gloo"], tmp_path,
                         env={"U2GNN_PARAM_CHECKSUM": "1"}, stderr=True)
    assert out.count("| epoch   1 |") == 1, out[-2000:]
    sums = _checksums(err)
    assert set(sums) == {0, 1}, err[-2000:]
    assert sums[0] == sums[1]
    kind = "Sup" if "UnSup" not in script else "UnSup"
    acc = run.parent / f"runs_pytorch_U2GNN_{kind}" / extra[3] / "checkpoints" / "model_acc.txt"
    assert acc.read_text().startswith(head)
