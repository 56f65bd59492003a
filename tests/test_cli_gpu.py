"""Integration: the drop-in CLIs run end-to-end on the GPU (1 epoch, capped steps) and write the
reference's stdout line and acc file."""
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "graph-transformer_amd")


def _run(script, extra, tmp_path):
    run = tmp_path / "run" / "x"
    run.mkdir(parents=True)
    cmd = [sys.executable, os.path.join(PKG, script), "--run_folder", str(run), "--num_epochs", "1"] + extra
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]
    return r.stdout, run


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
