"""Per-call latency and throughput of one AES-256-GCM batch against its size (one tunnel key,
1300-B packets), from Nebula's own flush sizes (RX: one recvmmsg batch of 64, TX: SendBatchCap
128, interface.go:381-413, 478-487) up to the 64 Ki headline batch. Each call is synchronous, as
a flush would use it: device-resident (neb_seal_batch / neb_open_batch + stream sync) and
host-resident (neb_*_batch_host on a pinned arena: zero-copy). Prints one JSON line per size.
usage (GPU box): python tools/batch_sweep.py [sizes...]
"""
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch

    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import DeviceBatch, PinnedBuffer, host_batch, install_keys, slot_desc
    from nebula_amd.noiseutil import Engine

    sizes = [int(x) for x in sys.argv[1:]] or [64, 128, 512, 2048, 8192, 65536]
    eng = Engine(0, max_keys=16)
    for n in sizes:
        b = W.make_batch(L.ALG_AESGCM, n, 1, seed=W.SEED ^ n)
        ciphers = install_keys(eng, b)
        db = DeviceBatch(eng, b, ciphers)
        reps = max(20, min(2000, 2_000_000 // n))
        out = {"packets": n, "payload_bytes": int(b.payload_bytes), "reps": reps}
        # a repeated seal is well defined (same keystream: it toggles the payload, the tag follows
        # the output); an open must follow its seal, so the pair is timed and the seal taken off
        def pair():
            db.seal()
            db.open()

        for name, fn in (("device_seal", db.seal), ("device_pair", pair)):
            for _ in range(5):
                fn()
            torch.cuda.synchronize()
            ts = []
            for _ in range(reps):
                t0 = time.perf_counter()
                fn()
                torch.cuda.synchronize()
                ts.append(time.perf_counter() - t0)
            out[name + "_us"] = round(float(np.median(ts)) * 1e6, 1)
        assert (db.status_host() == 0).all()
        out["device_seal_open_gibs"] = round(2 * b.payload_bytes / (out["device_pair_us"] * 1e-6) / 2**30, 2)
        d = slot_desc(b, ciphers)
        buf = PinnedBuffer(b.arena.nbytes)
        buf.array[:] = b.arena
        hint = int(d["key_id"][0])
        ts = []
        for k in range(3 + max(10, reps // 4)):
            t0 = time.perf_counter()
            s1 = host_batch(eng, b.alg, False, d, buf.array, hint)
            s2 = host_batch(eng, b.alg, True, d, buf.array, hint)
            if k >= 3:
                ts.append(time.perf_counter() - t0)
        assert (s1 == 0).all() and (s2 == 0).all()
        out["host_pair_us"] = round(float(np.median(ts)) * 1e6, 1)
        out["host_seal_open_gibs"] = round(2 * b.payload_bytes / (out["host_pair_us"] * 1e-6) / 2**30, 2)
        # the same with the descriptors and statuses in pinned memory too (neb_host_alloc), as a Go
        # caller would keep them beside the arena: the kernels read and write them in place
        import ctypes as C
        dbuf = PinnedBuffer(d.nbytes)
        sbuf = PinnedBuffer(4 * n)
        dbuf.array[:] = d.view(np.uint8)
        lib = L.lib()
        ts = []
        for k in range(3 + max(10, reps // 4)):
            t0 = time.perf_counter()
            for fn in (lib.neb_seal_batch_host, lib.neb_open_batch_host):
                L.check(fn(eng.handle, b.alg, C.c_void_p(dbuf.ptr), n, C.c_void_p(buf.ptr), buf.nbytes,
                           C.c_void_p(sbuf.ptr), hint), fn.__name__)
            if k >= 3:
                ts.append(time.perf_counter() - t0)
        assert (sbuf.array.view(np.int32) == 0).all()
        out["host_pinned_desc_pair_us"] = round(float(np.median(ts)) * 1e6, 1)
        out["host_pinned_desc_seal_open_gibs"] = round(2 * b.payload_bytes / (out["host_pinned_desc_pair_us"] * 1e-6) / 2**30, 2)
        dbuf.free()
        sbuf.free()
        buf.free()
        for c in ciphers:
            c.destroy()
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
