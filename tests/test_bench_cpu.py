"""bench.py's launcher contract on CPU (no GPU is touched): `--gpus N` without a launcher starts
torch.distributed.run with N ranks as a child process and relays their lines; inside a launcher,
WORLD_SIZE must equal --gpus."""
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _env(**kw):
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR",
                                                             "MASTER_PORT")}
    env.update(kw)
    return env


def test_gpus_2_spawns_two_ranks():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "2", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=_env(), cwd=REPO)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [json.loads(x) for x in p.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["launch_check"] for x in lines)


def test_world_size_must_match_gpus():
    p = subprocess.run([sys.executable, os.path.join(REPO, "bench.py"), "--gpus", "1", "--launch-check"],
                       capture_output=True, text=True, timeout=300, env=_env(WORLD_SIZE="2", RANK="0"), cwd=REPO)
    assert p.returncode != 0
    assert "WORLD_SIZE=2 but --gpus 1" in p.stderr
