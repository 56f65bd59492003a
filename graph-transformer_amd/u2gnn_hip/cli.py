"""Data parallelism for the drop-in CLIs (train_pytorch_U2GNN_{Sup,UnSup}.py; SURVEY.md §5 "Config /
flags": --world_size, §8(e)).  The reference trains on one device (train_pytorch_U2GNN_Sup.py:17); here a
CLI run with ``--world_size N`` trains one process per GPU:

* ``self_launch``: without a launcher around it the CLI starts ``torch.distributed.run --nproc-per-node N``
  on itself as a CHILD process before anything touches the GPU (no exec), and exits with its code.
  Under the launcher (WORLD_SIZE set) ``Run.init`` joins the process group: backend ``nccl`` (RCCL over
  xGMI) by default, ``gloo`` for several ranks on one GPU (tests).
* A global step is ``world`` consecutive batches of the reference's single numpy stream: rank r assembles
  batch r and replays the others (``Run.next_batch``; dp.rank_batches), so the ranks together train on
  exactly the batches one process would take in ``world`` steps, with the averaged gradient.
* EPOCHS ROUND UP TO A MULTIPLE OF ``world`` BATCHES: an epoch is ceil(num_batches_per_epoch / world)
  global steps.  When ``world`` does not divide the batch count, each epoch trains world - (nb % world)
  extra batches of the stream (MUTAG, nb = 43, world 2: 44), the epoch's summed loss (the plateau rule's
  input) covers those batches too, and from the second epoch on the stream positions differ from a
  one-process run with the same --num_epochs.  A one-process run is reproduced exactly when ``world``
  divides the batch count, or with --max_steps inside the first epoch (tests/test_cli_dp_cpu.py).
* Fused trainer: each batch's dropout seed is a function of its index in the stream (``step_seed``),
  whichever rank trains it.  --autograd: the module draws its dropout from torch's generator, seeded
  123 + rank per rank, so a data-parallel --autograd run is NOT reproducible by one process.
* Every rank runs the evaluation (it consumes the same numpy draws, so the streams stay aligned; the
  parameters are identical on every rank); rank 0 alone prints and writes the acc file.
"""
from __future__ import annotations

import os
import subprocess
import sys
from typing import List, Optional

import torch

from .dp import rank_batches  # noqa: F401  (the same partition rule; re-exported for the CLIs)


def self_launch(world_size: int, script: str, argv: List[str]) -> Optional[int]:
    """world_size > 1 and no launcher: run the launcher on ``script argv`` as a child process and return
    its exit code (the caller exits with it).  None when the caller should train itself.  The launcher runs
    --standalone (its own rendezvous on a port it binds itself: no probe-then-close port race)."""
    if world_size <= 1 or "WORLD_SIZE" in os.environ:
        return None
    cmd = [sys.executable, "-m", "torch.distributed.run", "--standalone", "--local-addr=127.0.0.1",
           f"--nproc-per-node={world_size}", os.path.abspath(script)] + list(argv)
    return subprocess.call(cmd)


def check_world(run_world: int, flag: int) -> None:
    """--world_size against the launcher's WORLD_SIZE: the flag left at its default (1) takes the launcher's
    value; an explicit flag must match it."""
    if flag != 1 and flag != run_world:
        raise SystemExit(f"WORLD_SIZE={run_world} but --world_size {flag}")


_MASK = (1 << 64) - 1


def step_seed(base: int, index: int) -> int:
    """Dropout seed of the batch at position ``index`` of the stream (splitmix64 of base and index)."""
    z = (int(base) * 0x9E3779B97F4A7C15 + (int(index) + 1) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _MASK
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _MASK
    return (z ^ (z >> 31)) & ((1 << 62) - 1)


class Run:
    """This process's place in the job (world, rank, device) and the few collectives the CLI loop uses."""

    def __init__(self, world: int = 1, rank: int = 0, local_rank: int = 0, dist=None):
        self.world, self.rank, self.local_rank, self.dist = world, rank, local_rank, dist
        self.index = 0   # position of the next global step's first batch in the stream

    @staticmethod
    def init(backend: str = "nccl", device_type: str = "cuda") -> "Run":
        world = int(os.environ.get("WORLD_SIZE", "1"))
        rank = int(os.environ.get("RANK", "0"))
        local_rank = int(os.environ.get("LOCAL_RANK", "0"))
        if world == 1:
            return Run()
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if device_type == "cuda" and backend == "nccl":
            dev = torch.device("cuda", local_rank)
            torch.cuda.set_device(dev)
            from .engine import side_stream
            side_stream(dev)   # before RCCL creates its streams (its own hardware queue; bench.py does the same)
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        return Run(world, rank, local_rank, dist)

    @property
    def main(self) -> bool:
        return self.rank == 0

    def device(self) -> torch.device:
        """One GPU per rank; several ranks share the visible GPUs round-robin only under gloo (tests)."""
        n = torch.cuda.device_count()
        if self.world > 1 and self.local_rank >= n and (self.dist is None or self.dist.get_backend() != "gloo"):
            raise SystemExit(f"rank {self.rank}: local rank {self.local_rank} but {n} GPU(s); one rank per GPU")
        return torch.device("cuda", self.local_rank % max(1, n))

    def next_batch(self, loader):
        """This rank's batch of the next global step (rank r of each group of ``world`` consecutive batches;
        the others' draws are consumed without building them) and its index in the stream."""
        hb = None
        for g in range(self.world):
            if g == self.rank:
                hb = loader()
            else:
                loader.replay()
        i = self.index + self.rank
        self.index += self.world
        return hb, i

    def sum(self, t: torch.Tensor) -> float:
        """Sum of a 1-element tensor over the ranks (the epoch's loss)."""
        if self.dist is not None:
            t = t.clone()
            self.dist.all_reduce(t)
        return float(t.item())

    def average_grads(self, params) -> None:
        """Mean of p.grad over the ranks (the autograd loop: after loss.backward(), before the clip)."""
        if self.dist is None:
            return
        for p in params:
            if p.grad is not None:
                self.dist.all_reduce(p.grad)
                p.grad.mul_(1.0 / self.world)

    def broadcast(self, t: torch.Tensor, src: int = 0) -> None:
        if self.dist is not None:
            self.dist.broadcast(t, src)

    def close(self) -> None:
        if self.dist is not None:
            self.dist.barrier()
            self.dist.destroy_process_group()
            self.dist = None
