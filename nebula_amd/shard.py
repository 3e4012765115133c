"""Multi-GPU plumbing, packets sharded by contiguous range with no data-path collective (packets
are independent — SURVEY.md §8e), in two forms:
  * one process per GPU (bench.py under torch.distributed.run): torch.distributed carries only the
    control plane, a start barrier and the max-over-ranks of the measured time;
  * several engines in one process (Nebula is one process): `host_batch_multi` (one host thread
    per engine over a host arena) and `ShardedDevice` (per-engine device-resident shards enqueued
    together), over the C ABI's neb_*_batch_host_multi / neb_*_batch_sharded.
"""
from __future__ import annotations

import os
import time
from typing import Optional, Tuple

import numpy as np


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


def host_batch_multi(engines, alg: int, open_: bool, desc, arena, key_hint: int = 0xFFFFFFFF):
    """neb_seal/open_batch_host_multi: contiguous shards of a host batch, one thread per engine.
    Every engine must hold the batch's keys at the same key_ids."""
    import ctypes as C


    from . import _lib as L

    status = np.full(len(desc), -1, np.int32)
    hs = (C.c_void_p * len(engines))(*[e.handle.value for e in engines])
    fn = L.lib().neb_open_batch_host_multi if open_ else L.lib().neb_seal_batch_host_multi
    rc = fn(hs, len(engines), alg, desc.ctypes.data_as(C.c_void_p), len(desc), arena.ctypes.data_as(C.c_void_p),
            arena.nbytes, status.ctypes.data_as(C.c_void_p), key_hint)
    L.check(rc, fn.__name__)
    return status


class ShardedDevice:
    """A batch split into contiguous shards, shard k resident on engine k's device (its own
    descriptors, arena and statuses as torch tensors), sealed / opened by one neb_*_batch_sharded
    call that enqueues every shard before waiting for any."""

    def __init__(self, engines, batch, ciphers_per_engine):
        import torch

        from .batch import slot_desc
        from .workload import shard

        self.engines = engines
        self.alg = batch.alg
        self.parts = []
        m = len(engines)
        for k, (e, ciphers) in enumerate(zip(engines, ciphers_per_engine)):
            part = shard(batch, k, m)
            dev = torch.device("cuda", e.device)
            d = slot_desc(part, ciphers)
            self.parts.append(dict(
                batch=part, desc=torch.from_numpy(d.view(np.uint8).copy()).to(dev),
                arena=torch.from_numpy(part.arena).to(dev),
                status=torch.full((part.n,), -1, dtype=torch.int32, device=dev),
                stream=torch.cuda.Stream(device=dev)))
        self.key_hint = ciphers_per_engine[0][0].key_id if batch.nkeys == 1 else 0xFFFFFFFF

    def _shards(self):
        from . import _lib as L

        arr = (L.Shard * len(self.parts))()
        for k, (e, p) in enumerate(zip(self.engines, self.parts)):
            arr[k] = L.Shard(e.handle.value, p["desc"].data_ptr(), p["batch"].n, p["arena"].data_ptr(),
                             p["status"].data_ptr(), p["stream"].cuda_stream)
        return arr

    def run(self, open_: bool) -> None:
        from . import _lib as L

        fn = L.lib().neb_open_batch_sharded if open_ else L.lib().neb_seal_batch_sharded
        L.check(fn(self.alg, self._shards(), len(self.parts), self.key_hint), fn.__name__)

    def arenas(self):
        return [p["arena"].cpu().numpy() for p in self.parts]

    def statuses(self):
        return [p["status"].cpu().numpy() for p in self.parts]
