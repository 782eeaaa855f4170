"""Multi-GPU driver helpers: one process per GPU, blocks dealt round-robin, no data-path
collective (blocks are independent — SURVEY.md §8e). torch.distributed carries only the
control plane: the barriers around the timed region and scalar max / sum reductions of its
duration and byte counts. Those are a few host scalars per run, so the process group is gloo
on every host — the same code the CPU tests (world size 2) and the GPU test (2 ranks on one
device) run; no RCCL communicator is created, because nothing on the data path exchanges."""
from __future__ import annotations

import os
import time
from dataclasses import dataclass
from typing import Callable

BACKEND = "gloo"


@dataclass
class Rank:
    rank: int = 0
    world: int = 1
    local_rank: int = 0
    dist: object = None  # torch.distributed when world > 1


def init() -> Rank:
    """Read RANK/WORLD_SIZE/LOCAL_RANK (torch.distributed.run); init the gloo control-plane group
    if > 1 rank."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    r = Rank(rank, world, local, None)
    if world > 1:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group(BACKEND)
        r.dist = dist
    return r


def rank_blocks(total_blocks: int, rank: int, world: int) -> list[int]:
    """Round-robin deal: global block b -> rank b mod world."""
    return list(range(rank, total_blocks, world))


def barrier(r: Rank) -> None:
    if r.dist is not None:
        r.dist.barrier()


def max_over_ranks(r: Rank, value: float) -> float:
    if r.dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    r.dist.all_reduce(t, op=r.dist.ReduceOp.MAX)
    return float(t.item())


def sum_over_ranks(r: Rank, value: float) -> float:
    if r.dist is None:
        return value
    import torch
    t = torch.tensor([value], dtype=torch.float64)
    r.dist.all_reduce(t, op=r.dist.ReduceOp.SUM)
    return float(t.item())


def timed_steps(r: Rank, step: Callable[[], None], steps: int, warmup: int,
                sync: Callable[[], None]) -> float:
    """W untimed steps, then K timed steps bracketed by barrier + device sync on both sides;
    returns the MAX over ranks of the timed duration (seconds)."""
    for _ in range(warmup):
        step()
    sync()
    barrier(r)
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    sync()
    barrier(r)
    dt = time.perf_counter() - t0
    return max_over_ranks(r, dt)


def finalize(r: Rank) -> None:
    if r.dist is not None:
        r.dist.destroy_process_group()
