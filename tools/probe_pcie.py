"""PCIe probe for the host-resident path (C2 batch, 1 GPU): pinned copy rates H2D, D2H and both
directions at once on two streams, then seal+open run by the kernels directly on pinned host
memory (zero-copy: descriptors, arena and status stay in hipHostMalloc'd buffers, the kernels'
loads and stores cross PCIe), checked by an open(seal(x)) = x round trip.
usage: python tools/probe_pcie.py [steps]"""
import ctypes as C
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np
import torch

from nebula_amd import _lib as L
from nebula_amd import workload as W
from nebula_amd.batch import PinnedBuffer, install_keys, slot_desc
from nebula_amd.noiseutil import Engine

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
b = W.config(1)
eng = Engine(0, 4096)
ciphers = install_keys(eng, b)
d = slot_desc(b, ciphers)
nb = b.arena.nbytes

# --- pinned copies -------------------------------------------------------------------------
h1 = torch.empty(nb, dtype=torch.uint8).pin_memory()
h2 = torch.empty(nb, dtype=torch.uint8).pin_memory()
g1 = torch.empty(nb, dtype=torch.uint8, device="cuda")
g2 = torch.empty(nb, dtype=torch.uint8, device="cuda")
s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()


def timed(fn, n=steps):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n


def h2d():
    with torch.cuda.stream(s1):
        g1.copy_(h1, non_blocking=True)


def d2h():
    with torch.cuda.stream(s2):
        h2.copy_(g2, non_blocking=True)


def both():
    h2d()
    d2h()


t = timed(h2d)
print(f"H2D alone      {nb / t / 1e9:6.1f} GB/s", flush=True)
t = timed(d2h)
print(f"D2H alone      {nb / t / 1e9:6.1f} GB/s", flush=True)
t = timed(both)
print(f"H2D + D2H      {2 * nb / t / 1e9:6.1f} GB/s total ({nb / t / 1e9:.1f} each way)", flush=True)

# --- zero-copy seal+open -------------------------------------------------------------------
arena = PinnedBuffer(nb)
arena.array[:] = b.arena
dbuf = PinnedBuffer(d.nbytes)
dbuf.array[:] = d.view(np.uint8)
sbuf = PinnedBuffer(4 * b.n)
status = sbuf.array.view(np.int32)
hint = int(d["key_id"][0])
lib = L.lib()
stream = torch.cuda.current_stream().cuda_stream


def call(fn):
    rc = fn(eng.handle, b.alg, C.c_void_p(dbuf.ptr), b.n, C.c_void_p(arena.ptr), C.c_void_p(sbuf.ptr), hint,
            C.c_void_p(stream))
    L.check(rc, "zero-copy batch")


def step():
    call(lib.neb_seal_batch)
    call(lib.neb_open_batch)


status[:] = -1
step()
torch.cuda.synchronize()
# statuses, and the payload of a sample of packets restored (the tag bytes now hold the tags)
smp = np.arange(0, b.n, 97)
idx = (d["src_off"][smp].astype(np.int64)[:, None] + np.arange(int(d["len"][0]))).ravel()
ok = bool((status == 0).all()) and np.array_equal(arena.array[idx], b.arena[idx])
t = timed(step)
print(f"zero-copy seal+open: {2 * b.payload_bytes / t / 2**30:6.2f} GiB/s payload, {t * 1e3:.3f} ms/step, "
      f"round trip {'ok' if ok else 'FAILED'}", flush=True)
