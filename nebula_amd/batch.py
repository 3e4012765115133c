"""Batched data plane: the SendBatch / recvmmsg flush points (interface.go:465-469, :395-400)
driven through neb_seal_batch / neb_open_batch on device-resident arenas, and through the pinned
host pipeline (neb_*_batch_host) for the TUN/UDP-side rate.

torch is used only as plumbing: device allocations and the current HIP stream.
"""
from __future__ import annotations

import ctypes as C
from typing import List, Optional

import numpy as np

from . import _lib as L
from .noiseutil import CipherAESGCM, CipherChaChaPoly, CipherState, Engine
from .workload import Batch


def install_keys(engine: Engine, b: Batch) -> List[CipherState]:
    """Install every key of the batch (noise CipherFunc.Cipher for each, in one device launch:
    neb_cipher_create_batch) and return the CipherStates."""
    cf = CipherAESGCM if b.alg == L.ALG_AESGCM else CipherChaChaPoly
    return cf.CipherBatch(engine, [bytes(b.keys[32 * i:32 * i + 32]) for i in range(b.nkeys)])


def install_keys_multi(engines: List[Engine], b: Batch) -> List[List[CipherState]]:
    """Every key of the batch on every engine of a set, each tunnel key one install shared by all
    of them (neb_cipher_create_multi); result[k] = engine k's CipherStates, same key_ids on all."""
    cf = CipherAESGCM if b.alg == L.ALG_AESGCM else CipherChaChaPoly
    per_key = [cf.CipherMulti(engines, bytes(b.keys[32 * i:32 * i + 32])) for i in range(b.nkeys)]
    return [[cs[k] for cs in per_key] for k in range(len(engines))]


def slot_desc(b: Batch, ciphers: List[CipherState]) -> np.ndarray:
    """Descriptors with batch key indices replaced by the engine's key-table slots."""
    slots = np.array([c.key_id for c in ciphers], np.uint32)
    d = b.desc.copy()
    d["key_id"] = slots[b.desc["key_id"]]
    return d


class DeviceBatch:
    """A batch resident in HBM: arena, descriptors and status as torch CUDA tensors."""

    def __init__(self, engine: Engine, b: Batch, ciphers: List[CipherState], device: Optional[int] = None):
        import torch

        self.torch = torch
        self.engine = engine
        self.batch = b
        self.dev = torch.device("cuda", engine.device if device is None else device)
        d = slot_desc(b, ciphers)
        self.desc_host = d
        self.arena = torch.from_numpy(b.arena).to(self.dev)
        self.desc = torch.from_numpy(d.view(np.uint8)).to(self.dev)
        self.status = torch.full((b.n,), -1, dtype=torch.int32, device=self.dev)
        self.key_hint = int(d["key_id"][0]) if len(ciphers) == 1 else L.KEYS_MIXED
        self.n = b.n

    def _call(self, fn, stream) -> None:
        torch = self.torch
        s = torch.cuda.current_stream(self.dev).cuda_stream if stream is None else stream
        rc = fn(self.engine.handle, self.batch.alg, C.c_void_p(self.desc.data_ptr()), self.n,
                C.c_void_p(self.arena.data_ptr()), C.c_void_p(self.status.data_ptr()), self.key_hint,
                C.c_void_p(s))
        L.check(rc, fn.__name__)

    def seal(self, stream=None) -> None:
        self._call(L.lib().neb_seal_batch, stream)

    def open(self, stream=None) -> None:
        self._call(L.lib().neb_open_batch, stream)

    def arena_host(self) -> np.ndarray:
        return self.arena.cpu().numpy()

    def status_host(self) -> np.ndarray:
        return self.status.cpu().numpy()


class PinnedBuffer:
    """hipHostMalloc'd bytes (backs batch.Arena, overlay/batch/coalesce_core.go:142-169)."""

    def __init__(self, nbytes: int):
        p = C.c_void_p()
        L.check(L.lib().neb_host_alloc(nbytes, C.byref(p)), "neb_host_alloc")
        self.ptr = p.value
        self.nbytes = nbytes
        self.array = np.ctypeslib.as_array((C.c_uint8 * nbytes).from_address(self.ptr))

    def free(self) -> None:
        if self.ptr:
            L.lib().neb_host_free(C.c_void_p(self.ptr))
            self.ptr = None

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def host_batch(engine: Engine, alg: int, open_: bool, desc: np.ndarray, arena: np.ndarray,
               key_hint: int = L.KEYS_MIXED) -> np.ndarray:
    """Seal/open a host-resident batch in place (pinned H2D -> kernel -> D2H pipeline)."""
    assert desc.dtype == L.DESC_DTYPE and arena.dtype == np.uint8 and arena.flags["C_CONTIGUOUS"]
    status = np.full(len(desc), -1, np.int32)
    fn = L.lib().neb_open_batch_host if open_ else L.lib().neb_seal_batch_host
    rc = fn(engine.handle, alg, desc.ctypes.data_as(C.c_void_p), len(desc), arena.ctypes.data_as(C.c_void_p),
            arena.nbytes, status.ctypes.data_as(C.c_void_p), key_hint)
    L.check(rc, fn.__name__)
    return status


class SubmitQueue:
    """neb_queue_*: one algorithm and direction's submission queue. Many threads call submit() with
    their own small flushes (Nebula's 64-128 packet TX / RX flushes, interface.go:381-487); the
    queue joins them into device batches and returns each caller its own results."""

    def __init__(self, engine: Engine, alg: int, open_: bool, max_packets: int = 0, max_delay_us: int = 0,
                 arena_bytes: int = 0, depth: int = 0):
        cfg = L.QueueConfig(max_packets, max_delay_us, arena_bytes, depth, 0)
        h = C.c_void_p()
        L.check(L.lib().neb_queue_create(engine.handle, alg, 1 if open_ else 0, C.byref(cfg), C.byref(h)),
                "neb_queue_create")
        self.h = h
        self.alg = alg
        self.open = open_

    def submit(self, desc: np.ndarray, arena: np.ndarray, status: Optional[np.ndarray] = None) -> np.ndarray:
        """Seal/open desc over arena (host memory, in place per descriptor), blocking until done."""
        assert desc.dtype == L.DESC_DTYPE and arena.dtype == np.uint8 and arena.flags["C_CONTIGUOUS"]
        if status is None:
            status = np.full(len(desc), -1, np.int32)
        rc = L.lib().neb_queue_submit(self.h, desc.ctypes.data_as(C.c_void_p), len(desc),
                                      arena.ctypes.data_as(C.c_void_p), arena.nbytes,
                                      status.ctypes.data_as(C.c_void_p))
        L.check(rc, "neb_queue_submit")
        return status

    def flush(self) -> None:
        L.check(L.lib().neb_queue_flush(self.h), "neb_queue_flush")

    def stats(self) -> dict:
        v = (C.c_uint64 * 4)()
        L.check(L.lib().neb_queue_stats(self.h, v), "neb_queue_stats")
        return {"batches": v[0], "packets": v[1], "submissions": v[2], "bytes": v[3]}

    def close(self) -> None:
        if self.h:
            L.lib().neb_queue_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
