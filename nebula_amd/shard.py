"""Multi-GPU plumbing: one process per GPU, packets sharded by contiguous range, no data-path
collective (packets are independent — SURVEY.md §8e). torch.distributed is used only for the
control plane: a start barrier and the max-over-ranks of the measured time.
"""
from __future__ import annotations

import os
import time
from typing import Optional, Tuple


def dist_env() -> Tuple[int, int, int]:
    """(rank, world_size, local_rank) from the torch.distributed.run environment."""
    return int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")), int(os.environ.get("LOCAL_RANK", "0"))


def shard_range(n: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous [lo, hi) packet range of `rank`; the ranges tile [0, n) exactly."""
    return n * rank // world, n * (rank + 1) // world


class Control:
    """Barrier + max-reduce over ranks on a gloo (CPU) process group; no-ops for world_size 1."""

    def __init__(self, world: int, init: bool = True):
        self.world = world
        self.dist = None
        if world > 1:
            import torch.distributed as dist

            if init and not dist.is_initialized():
                dist.init_process_group("gloo")
            self.dist = dist

    def barrier(self) -> None:
        if self.dist is not None:
            self.dist.barrier()

    def max(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t[0])

    def sum(self, x: float) -> float:
        if self.dist is None:
            return x
        import torch

        t = torch.tensor([x], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.SUM)
        return float(t[0])


def timed(ctrl: Control, fn, sync=None) -> float:
    """Run fn() between barrier+sync brackets; return the max wall time over ranks."""
    ctrl.barrier()
    if sync:
        sync()
    t0 = time.perf_counter()
    fn()
    if sync:
        sync()
    ctrl.barrier()
    return ctrl.max(time.perf_counter() - t0)


def aggregate_gibs(total_bytes_all_ranks: float, seconds: float) -> float:
    return total_bytes_all_ranks / seconds / float(1 << 30)
