#!/usr/bin/env python3
"""A/B of the mixed-key binning forms over batch size: the atomic histogram
(sub-bins from 256 Ki packets) against the tile form, on the C5 shape (AES-256-GCM, 4096 keys,
IMIX 90/576/1300 7:4:1) at 64 Ki-1 Mi packets — the per-GPU shard sizes of C5 over 16-1 GPUs.
Times seal + open of one device-resident batch per step (HIP events on the stream), alternating
the two forms, and prints one JSON line per size. GPU box only."""
import json
import sys
import time

import torch

sys.path.insert(0, ".")
from nebula_amd import Engine, _lib as L  # noqa: E402
from nebula_amd import workload as W  # noqa: E402
from nebula_amd.batch import DeviceBatch, install_keys  # noqa: E402

NEVER = 4_000_000_000


def main():
    sizes = [int(x) for x in sys.argv[1:]] or [65536, 131072, 262144, 524288, 1 << 20]
    eng = Engine(0, max_keys=4096)
    for n in sizes:
        b = W.make_batch(L.ALG_AESGCM, n, 4096, sizes=(90, 576, 1300), ratio=(7, 4, 1), seed=W.SEED ^ n, name="tiles")
        ciphers = install_keys(eng, b)
        db = DeviceBatch(eng, b, ciphers)
        payload = float(b.desc["len"].astype("int64").sum())
        res = {}
        for rep in range(3):
            for form, tile_from in (("atomics", NEVER), ("tiles", 0)):
                with L.knob(L.KNOB_TILE_BINS_FROM, tile_from):
                    for _ in range(2):  # warm
                        db.seal()
                        db.open()
                    torch.cuda.synchronize()
                    steps = 10
                    t0 = time.perf_counter()
                    for _ in range(steps):
                        db.seal()
                        db.open()
                    torch.cuda.synchronize()
                    dt = (time.perf_counter() - t0) / steps
                assert (db.status_host() == 0).all()
                res.setdefault(form, []).append(round(2 * payload / dt / 2**30, 2))
        print(json.dumps({"packets": n, "gibs": res}), flush=True)
        for c in ciphers:
            c.destroy()
        del db
    eng.close()


if __name__ == "__main__":
    main()
