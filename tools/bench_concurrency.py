#!/usr/bin/env python3
"""Concurrency measurements of the host-facing surfaces ("Concurrency"):

  percall  EncryptDanger / DecryptDanger (neb_encrypt_danger / neb_decrypt_danger, the per-packet
           CipherState surface, noiseutil/cipher_state.go:23-38) from T threads at once, 1300-B
           packets: calls/s, GiB/s of payload, per-call latency p50 / p99.
  queue    the submission queue (neb_queue_*): T threads each sealing (then opening) Nebula-sized
           flushes of F packets (128 = SendBatchCap, tx_batch.go:5; 64 = listen.batch, main.go:181)
           with deadline D us: seal+open GiB/s of payload, per-submission latency p50 / p99, device
           batches per second and mean batch size.

usage: python tools/bench_concurrency.py [percall|queue|all] [--seconds S]
Every result is one JSON line on stdout.
"""
import argparse
import ctypes as C
import json
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

GIB = float(1 << 30)


def percall(eng, threads, seconds, size=1300, alg=1):
    from nebula_amd import _lib as L
    from nebula_amd.noiseutil import CipherAESGCM, CipherChaChaPoly

    lib = L.lib()
    cf = CipherAESGCM if alg == L.ALG_AESGCM else CipherChaChaPoly
    cs = cf.Cipher(eng, bytes(range(32)))
    stop = threading.Event()
    lat = [[] for _ in range(threads)]
    calls = [0] * threads

    def worker(t):
        out = (C.c_uint8 * (size + 64))()
        back = (C.c_uint8 * (size + 64))()
        ad = (C.c_uint8 * 16)()
        pt = (C.c_uint8 * size)(*([t & 0xFF] * size))
        ret = C.c_size_t()
        n = t << 40
        mine = lat[t]
        while not stop.is_set():
            t0 = time.perf_counter()
            rc = lib.neb_encrypt_danger(cs.handle, out, 0, size + 64, ad, 16, pt, size, C.c_uint64(n), None,
                                        C.byref(ret))
            rc |= lib.neb_decrypt_danger(cs.handle, back, 0, size + 64, ad, 16, out, size + 16, C.c_uint64(n), None,
                                         C.byref(ret))
            mine.append(time.perf_counter() - t0)
            if rc:
                raise RuntimeError(rc)
            n += 1
            calls[t] += 2

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    time.sleep(0.3)  # warm-up: slots and streams created
    for i in range(threads):
        calls[i] = 0
        lat[i].clear()
    t0 = time.perf_counter()
    time.sleep(seconds)
    dt = time.perf_counter() - t0
    tot = sum(calls)
    stop.set()
    for th in ths:
        th.join()
    cs.destroy()
    lats = np.array([x for v in lat for x in v]) * 1e6 / 2  # per call (a pair is seal + open)
    return {"bench": "percall", "threads": threads, "calls_per_s": round(tot / dt, 1),
            "gibs": round(tot * size / dt / GIB, 4), "latency_us_p50": round(float(np.percentile(lats, 50)), 1),
            "latency_us_p99": round(float(np.percentile(lats, 99)), 1), "packet_bytes": size,
            "cipher": "AES-256-GCM" if alg == 1 else "ChaCha20-Poly1305"}


def queue(eng, threads, flush, deadline_us, seconds, nkeys=64):
    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import SubmitQueue, install_keys, slot_desc

    b = W.make_batch(L.ALG_AESGCM, threads * flush, nkeys, name="queue")
    ciphers = install_keys(eng, b)
    d = slot_desc(b, ciphers)
    mp = max(4096, threads * flush)
    sq = SubmitQueue(eng, L.ALG_AESGCM, False, max_packets=mp, max_delay_us=deadline_us)
    oq = SubmitQueue(eng, L.ALG_AESGCM, True, max_packets=mp, max_delay_us=deadline_us)
    stop = threading.Event()
    lat = [[] for _ in range(threads)]
    pk = [0] * threads

    def worker(t):
        dd = d[t * flush:(t + 1) * flush].copy()
        lo = int(dd["aad_off"].min())
        for k in ("src_off", "dst_off", "aad_off"):
            dd[k] -= np.uint64(lo)
        arena = b.arena[lo:lo + flush * b.stride].copy()
        st = np.zeros(flush, np.int32)
        while not stop.is_set():
            t0 = time.perf_counter()
            sq.submit(dd, arena, st)
            t1 = time.perf_counter()
            oq.submit(dd, arena, st)
            t2 = time.perf_counter()
            lat[t] += [t1 - t0, t2 - t1]
            pk[t] += flush
            if (st != 0).any():
                raise RuntimeError("status")

    ths = [threading.Thread(target=worker, args=(t,)) for t in range(threads)]
    for th in ths:
        th.start()
    time.sleep(0.5)
    for i in range(threads):
        pk[i] = 0
        lat[i].clear()
    s0 = sq.stats()
    t0 = time.perf_counter()
    time.sleep(seconds)
    dt = time.perf_counter() - t0
    s1 = sq.stats()
    tot = sum(pk)
    stop.set()
    for th in ths:
        th.join()
    sq.close()
    oq.close()
    for c in ciphers:
        c.destroy()
    lats = np.array([x for v in lat for x in v]) * 1e6
    nb = s1["batches"] - s0["batches"]
    return {"bench": "queue", "threads": threads, "flush_packets": flush, "deadline_us": deadline_us,
            "gibs": round(2 * tot * 1300 / dt / GIB, 3), "packets_per_s": round(tot / dt, 1),
            "submit_latency_us_p50": round(float(np.percentile(lats, 50)), 1),
            "submit_latency_us_p99": round(float(np.percentile(lats, 99)), 1),
            "seal_batches_per_s": round(nb / dt, 1),
            "mean_seal_batch_packets": round((s1["packets"] - s0["packets"]) / max(nb, 1), 1),
            "workload": f"1300-B packets over {nkeys} tunnels, each thread seal then open of its own flush"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("what", nargs="?", default="all")
    ap.add_argument("--seconds", type=float, default=1.5)
    a = ap.parse_args()
    import torch  # noqa: F401  (one HIP runtime for the process)

    from nebula_amd.noiseutil import Engine

    eng = Engine(0, 4096)
    if a.what in ("percall", "all"):
        for t in (1, 8, 32):
            print(json.dumps(percall(eng, t, a.seconds)), flush=True)
    if a.what in ("queue", "all"):
        for t, f in ((1, 128), (8, 128), (16, 128), (32, 128), (32, 64)):
            for dl in (50, 200):
                print(json.dumps(queue(eng, t, f, dl, a.seconds)), flush=True)
    eng.close()


if __name__ == "__main__":
    main()
