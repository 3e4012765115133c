#!/usr/bin/env python3
"""bench.py — device-resident AES-256-GCM seal+open throughput (BASELINE.json metric).

  python bench.py [--gpus N] [--steps K] [--warmup W] [--settle-ms MS] [--config 1..4] [--mode device|host]

One step = seal every packet of the batch, then open every packet of it (in place, on device),
i.e. one pass of the hot path (inside.go seal + outside.go open) over one 64 Ki x 1300 B batch.
N > 1: one process per GPU, each rank owns its own batch of the same shape (packets are
independent: no collective on the data path — SURVEY.md §8e; C5 is one batch split over the ranks).
Launched by torch.distributed.run, or, when no launcher set WORLD_SIZE, by this script itself: it
starts the N rank processes with the same environment torchrun gives them and relays rank 0's line,
so `python bench.py --gpus 8` and the torchrun form measure the same thing (spawn_ranks).
Timing is bracketed by a barrier + device sync on both sides and the max over ranks is taken.
Before the W warmup steps the device modes settle (--settle-ms, default 300): untimed steps of the
same work until that much wall time has passed, so the GPU runs at the clocks a sustained load
holds (an idle MI355X needs a few hundred ms of load; the line's `settle` reports it, and
--settle-ms 0 measures from a cold start).

Printed (rank 0, one JSON line): value = (payload sealed + payload opened, all ranks) / time.
roofline: the seal kernel's algorithmic bytes (2p+32 per packet) / its mean launch time, from HIP
events bound to that kernel's own dispatch inside the timed region (neb_time_next_kernel: start and
stop of the dominant kernel, no marker packets); traffic = PMC-measured HBM bytes
per launch of this config's seal kernel from profiles/pmc_configs.json, else null.
cpu_baseline: rank 0, N = 1 only, the OpenSSL-EVP port of the per-packet loop (oracle/) on a
bounded sample of the same batch: the best of a thread sweep up to every CPU of this process's
affinity, and one thread.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s HBM3E peak
GIB = float(1 << 30)
EV_EVERY = 4  # kernel-timing events bracket every 4th step (see the timed loop)


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def settle(args, step) -> dict:
    """An idle MI355X takes a few hundred ms of load to reach the clocks a sustained load holds:
    after the 5 default warmup steps of C2 (1.2 ms) the seal kernel ran 115-122 µs, against 95-98
    µs at steady state (profiles/r5/settle). Before the W warmup steps, untimed,
    `step` (the mode's own work) repeats until --settle-ms of wall time has passed, synchronised
    every 16 steps so the host does not run ahead of the device. The line reports it."""
    import torch

    n = 0
    if args.settle_ms > 0:
        t0 = time.perf_counter()
        while (time.perf_counter() - t0) * 1e3 < args.settle_ms:
            step()
            n += 1
            if n % 16 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
    return {"ms": args.settle_ms, "steps": n}


class TimingEvent:
    """A HIP timing event recorded without the system-scope fence (hipEventDisableSystemFence, the
    flag HIP documents for timing-only events): a default event writes back and invalidates the
    caches when it is recorded, which put 6-13 µs of marker cost into every kernel bracket here
    (in-bench 123-128 µs against rocprof's 115 µs for the same seal kernel). Falls back to
    torch.cuda.Event when the HIP runtime cannot be reached through ctypes."""

    _hip = None
    FLAGS = 0x20000000  # hipEventDisableSystemFence (hip_runtime_api.h)

    @classmethod
    def hip(cls):
        if cls._hip is None:
            import ctypes

            path = None
            for line in open("/proc/self/maps"):
                if "libamdhip64" in line:
                    path = line.split()[-1]
                    break
            cls._hip = ctypes.CDLL(path) if path else False
        return cls._hip

    def __init__(self):
        import ctypes

        import torch

        self.torch_ev = None
        hip = self.hip()
        self.h = ctypes.c_void_p()
        if not hip or hip.hipEventCreateWithFlags(ctypes.byref(self.h), ctypes.c_uint(self.FLAGS)) != 0:
            self.torch_ev = torch.cuda.Event(enable_timing=True)

    def record(self, stream) -> None:
        import ctypes

        if self.torch_ev is not None:
            self.torch_ev.record(stream)
        elif self.hip().hipEventRecord(self.h, ctypes.c_void_p(stream.cuda_stream)) != 0:
            raise RuntimeError("hipEventRecord failed")

    def elapsed_time(self, end: "TimingEvent") -> float:
        import ctypes

        if self.torch_ev is not None:
            return self.torch_ev.elapsed_time(end.torch_ev)
        ms = ctypes.c_float()
        if self.hip().hipEventElapsedTime(ctypes.byref(ms), self.h, end.h) != 0:
            raise RuntimeError("hipEventElapsedTime failed")
        return float(ms.value)


def cgroup_cpus():
    """The CPU bandwidth quota of this process's cgroup, in CPUs (cgroup v2 cpu.max, else v1
    cfs_quota/cfs_period), or None when unlimited. A box may show every CPU of the machine in the
    affinity mask while the quota grants a share of them."""
    import math

    try:
        rel = ""
        for line in open("/proc/self/cgroup"):
            parts = line.strip().split(":", 2)
            if len(parts) == 3 and parts[0] == "0":
                rel = parts[2]
        for base in (os.path.join("/sys/fs/cgroup", rel.lstrip("/")), "/sys/fs/cgroup"):
            f = os.path.join(base, "cpu.max")
            if os.path.exists(f):
                q, per = open(f).read().split()[:2]
                return None if q == "max" else max(1, math.ceil(int(q) / int(per)))
        q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
        per = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
        return None if q <= 0 else max(1, math.ceil(q / per))
    except (OSError, ValueError):
        return None


def cpu_cores() -> int:
    """The CPUs this process may run on: the affinity mask (sched_getaffinity), capped by the
    cgroup's CPU quota when it has one. NEB_CPU_THREADS overrides."""
    if os.environ.get("NEB_CPU_THREADS"):
        return max(1, int(os.environ["NEB_CPU_THREADS"]))
    try:
        n = max(1, len(os.sched_getaffinity(0)))
    except Exception:
        n = os.cpu_count() or 1
    q = cgroup_cpus()
    return min(n, q) if q else n


def cpu_thread_counts(n: int):
    """Thread counts the CPU baseline sweeps up to n (every CPU of the affinity mask): on the GPU box
    the mask lists the whole machine (256) while the box's share of it is smaller, and 256 threads
    ran at 1.9 GiB/s against 3.4 on one, so the best of the sweep is the baseline."""
    return sorted({c for c in (8, 16, 32, 64, n) if c <= n} or {n})


def cpu_baseline(b, target_s: float = 4.0):
    """OpenSSL-EVP port (oracle/evp_baseline.c) on a bounded sample of the same batch: seal then
    open, each timed for about target_s seconds, on every core this process may use (one pinned
    thread per core), and again on one thread (1 and nproc threads)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle

    threads = cpu_cores()
    n = min(b.n, 16384)
    desc = b.desc[:n].copy()
    lo = int(desc["aad_off"].min())
    hi = int((desc["src_off"] + desc["len"].astype(np.uint64) + np.uint64(16)).max())
    for f in ("src_off", "dst_off", "aad_off"):
        desc[f] -= np.uint64(lo)
    arena = b.arena[lo:hi].copy()
    keys = b.keys
    sealed = arena.copy()
    _, st = oracle.evp_batch(b.alg, 0, keys, desc, sealed, threads=threads, iters=1)
    assert (st == 0).all()
    # open out of place into a scratch copy, so the ciphertext stays intact across passes
    od = desc.copy()
    od["dst_off"] = od["src_off"] + np.uint64(len(sealed))
    big = np.concatenate([sealed, np.zeros_like(sealed)])
    payload = float(desc["len"].astype(np.int64).sum())

    def rate(nthreads, secs):
        oracle.evp_batch(b.alg, 0, keys, desc, arena.copy(), threads=nthreads, iters=1)  # warm the pool
        t1, _ = oracle.evp_batch(b.alg, 0, keys, desc, arena.copy(), threads=nthreads, iters=2)
        iters = max(1, int(secs / max(t1 / 2, 1e-5)))
        t_seal, _ = oracle.evp_batch(b.alg, 0, keys, desc, arena.copy(), threads=nthreads, iters=iters)
        t_open, st2 = oracle.evp_batch(b.alg, 1, keys, od, big, threads=nthreads, iters=iters)
        assert (st2 == 0).all()
        return 2 * payload * iters / (t_seal + t_open) / GIB, iters, t_seal + t_open

    sweep = {}
    for c in cpu_thread_counts(threads):
        sweep[c] = rate(c, target_s / 2)
    best = max(sweep, key=lambda c: sweep[c][0])
    gibs, iters, tt = sweep[best]
    gibs1, iters1, tt1 = rate(1, target_s / 3)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except Exception:
        pass
    return {
        "value": round(gibs, 3), "unit": "GiB/s", "cores": best, "kind": "port",
        "value_1thread": round(gibs1, 3),
        "sweep": {str(c): round(v[0], 3) for c, v in sweep.items()},
        "affinity_cpus": threads,
        "sample": f"{n} packets of the same batch ({payload / 1e6:.1f} MB payload), seal x{iters} + open x{iters} "
                  f"({tt:.1f} s) on {best} pinned threads, the best of a sweep up to all {threads} CPUs of this "
                  f"process's affinity ('sweep'), and x{iters1} on 1 thread ({tt1:.1f} s); OpenSSL EVP "
                  + ("AES-256-GCM (AES-NI/VAES + PCLMUL class, as Go's crypto/cipher)" if b.alg == 1 else
                     "ChaCha20-Poly1305 (AVX2 / AVX-512 SIMD class, as golang.org/x/crypto/chacha20poly1305)")
                  + f", {model}",
    }


def pmc_config(cfg_name: str):
    """The committed counter pass of this config's dominant kernel (profiles/pmc_configs.json,
    written by tools/pmc_config.py): HBM bytes per launch (2*FETCH_SIZE + WRITE_SIZE, the gfx950
    correction), LDS / VALU busy fractions, rocprof mean duration, and the pass it came from.
    Keyed by config, so C3 and C5 (same kernel, different traffic) each report their own."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "pmc_configs.json")))[cfg_name]
    except Exception:
        return None


def _free_port() -> int:
    import socket

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_ranks(nranks: int, argv) -> int:
    """`--gpus N` with no launcher around this process (WORLD_SIZE unset): start the N rank
    processes here, each a fresh interpreter running this script with the torch.distributed.run
    environment (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_ADDR=127.0.0.1 / MASTER_PORT), so a bare
    `python bench.py --gpus 8` measures 8 GPUs exactly as the torchrun form does. This process
    touches no GPU (children are started, never exec'd into). The ranks run the barrier, the timing
    and the max / sum over ranks themselves; rank 0's one JSON line is relayed with `launcher` added.
    If any rank fails the others are stopped and the exit status is non-zero: never a one-GPU line
    for an N-GPU request."""
    import subprocess
    import threading

    port = _free_port()
    procs = []
    for r in range(nranks):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(nranks), LOCAL_WORLD_SIZE=str(nranks),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL, text=True))
    out = []
    reader = threading.Thread(target=lambda: out.extend(procs[0].stdout), daemon=True)
    reader.start()
    rc = 0
    while None in [p.poll() for p in procs]:  # (a list: every process polled each time)
        bad = [p.returncode for p in procs if p.returncode not in (None, 0)]
        if bad:
            rc = bad[0]
            for p in procs:
                if p.poll() is None:
                    p.kill()
            break
        time.sleep(0.1)
    for p in procs:
        p.wait()
    reader.join(timeout=10)
    rc = rc or next((p.returncode for p in procs if p.returncode != 0), 0)
    lines = [ln for ln in out if ln.lstrip().startswith("{")]
    if rc != 0 or not lines:
        log(f"bench: {nranks} rank processes, exit statuses {[p.returncode for p in procs]}; no result")
        return rc or 1
    for ln in out:
        if not ln.lstrip().startswith("{"):
            sys.stdout.write(ln)
    res = json.loads(lines[-1])
    if res.get("n_gpus") != nranks:
        log(f"bench: rank 0 reported n_gpus {res.get('n_gpus')} for {nranks} ranks")
        return 1
    res["launcher"] = f"bench.py: {nranks} rank processes (RANK/WORLD_SIZE env, gloo control plane)"
    print(json.dumps(res), flush=True)
    return 0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=1, help="BASELINE.json configs index (1 = headline)")
    ap.add_argument("--mode", choices=["device", "host", "host-staged", "tx", "rx", "rx-device", "relay"],
                    default="device",
                    help="device: the headline; host: host-resident batch (pinned arena: zero-copy); "
                         "host-staged: the same through hipMemcpyAsync staging; tx: the device TX batch "
                         "(TSO superpackets -> sealed wire packets); rx: batched receive with replay windows; "
                         "rx-device: the same with the batch and the windows in device memory; relay: GMAC-only "
                         "seal+verify of 1348-B relayed packets (VerifyRelay), device-resident")
    ap.add_argument("--settle-ms", type=float, default=300.0,
                    help="device mode: before the W warmup steps, untimed seal+open steps until this much wall "
                         "time has passed, so the GPU runs at the clocks a sustained load holds (0: none; "
                         "reported as `settle` in the line)")
    ap.add_argument("--sustain-ms", type=float, default=1000.0,
                    help="device mode: after the timed K steps, the same step repeated for about this long "
                         "(a fixed step count from the timed rate, barrier + sync around it, max over ranks): "
                         "the rate a long load holds, reported as `sustained` beside `value` (0: skip)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--inproc", action="store_true",
                    help="device mode, --gpus N engines in ONE process (Nebula is one process): each engine its "
                         "own batch of the config's shape on its GPU (round-robin over the visible devices), "
                         "all enqueued by one neb_*_batch_sharded call per step (SURVEY.md §8e)")
    ap.add_argument("--tx-superpackets", type=int, default=1457,
                    help="tx mode: 64 KiB TSO superpackets per batch (45 segments each; 1457 -> 65 565 wires, "
                         "1456 -> 65 520: within one pass of the 4096 waves of 16 packets)")
    ap.add_argument("--shard-of", type=int, default=0,
                    help="--config 4 on one rank: run only shard --shard-rank of the 1 Mi C5 batch split N ways "
                         "(the packets one GPU of an N-GPU run gets), so the per-GPU shape is measured on one GPU")
    ap.add_argument("--shard-rank", type=int, default=0)
    ap.add_argument("--shard-by", choices=["key", "range"], default="key",
                    help="--config 4 over N GPUs: each rank takes the tunnels with key_id mod N = rank (key: a "
                         "tunnel's packets and state on one device), or a contiguous packet range (range)")
    ap.add_argument("--stub", action="store_true", help=argparse.SUPPRESS)  # tests: launch + aggregation, no GPU
    args = ap.parse_args()

    from nebula_amd.shard import Control, dist_env

    if args.inproc:
        return bench_inproc(args)
    if args.gpus > 1 and int(os.environ.get("WORLD_SIZE", "1")) == 1:
        # no launcher: this process starts the ranks itself (before anything here touches the GPU)
        sys.exit(spawn_ranks(args.gpus, sys.argv[1:]))
    rank, world, local = dist_env()
    if world != args.gpus:
        log(f"note: --gpus {args.gpus} but the launcher started WORLD_SIZE={world} ranks; using WORLD_SIZE")
    if args.stub:
        return bench_stub(args, rank, world)
    import torch

    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import DeviceBatch, host_batch, install_keys, slot_desc
    from nebula_amd.noiseutil import Engine

    # one process per GPU; more ranks than devices (a rehearsal on a smaller box) share them round-robin
    ndev = torch.cuda.device_count()
    device = local % ndev if ndev else local
    torch.cuda.set_device(device)
    # control plane only (barrier / max of timings) over gloo; no data-path collective
    ctrl = Control(world)
    barrier = ctrl.barrier

    cfg = args.config
    t0 = time.time()
    if args.mode == "relay":
        return bench_relay(args, ctrl, rank, world, device)
    b = W.make_batch(*{
        0: (L.ALG_AESGCM, 1024, 1),
        1: (L.ALG_AESGCM, 65536, 1),
        2: (L.ALG_AESGCM, 65536, 4096),
        3: (L.ALG_CHACHAPOLY, 65536, 4096),
    }[cfg], seed=W.SEED ^ rank, name=f"C{cfg + 1}") if cfg in (0, 1, 2, 3) else \
        (W.shard_by_key if args.shard_by == "key" else W.shard)(
            W.config(4), *((args.shard_rank, args.shard_of) if args.shard_of else (rank, world)))
    workload_name = {0: "C1 AES-256-GCM, 1 tunnel key, 1024 x 1300 B packets, device-resident",
                     1: "C2 AES-256-GCM, 1 tunnel key, 65536 x 1300 B packets, device-resident",
                     2: "C3 AES-256-GCM, 4096 tunnel keys, 65536 x 1300 B packets, device-resident",
                     3: "C4 ChaCha20-Poly1305, 4096 tunnel keys, 65536 x 1300 B packets, device-resident",
                     4: "C5 AES-256-GCM, 4096 tunnel keys, IMIX 90/576/1300 (7:4:1), 1 Mi packets sharded"}[cfg]
    if cfg == 4 and args.shard_of:
        if world != 1:
            raise SystemExit("--shard-of runs one shard on one rank")
        workload_name += (f": shard {args.shard_rank} of {args.shard_of} alone ({b.n} packets, one GPU's part; "
                          + ("tunnels with key_id mod N = r)" if args.shard_by == "key" else "contiguous packet range)"))
    log(f"[rank {rank}] batch {b.name}: {b.n} pkts, {b.payload_bytes / 1e6:.1f} MB payload "
        f"({time.time() - t0:.1f}s to build)")

    eng = Engine(device, max_keys=max(4096, b.nkeys))
    ciphers = install_keys(eng, b)
    payload = float(b.payload_bytes)
    alg_bytes = float(b.algorithmic_bytes)

    if args.mode == "host-staged":
        L.check(L.lib().neb_set_knob(L.KNOB_HOST_MODE, 1), "neb_set_knob")  # DMA staging
    if args.mode in ("host", "host-staged"):
        from nebula_amd.batch import PinnedBuffer

        d = slot_desc(b, ciphers)
        buf = PinnedBuffer(b.arena.nbytes)
        buf.array[:] = b.arena
        hint = int(d["key_id"][0]) if b.nkeys == 1 else L.KEYS_MIXED
        for _ in range(args.warmup):
            host_batch(eng, b.alg, False, d, buf.array, hint)
            host_batch(eng, b.alg, True, d, buf.array, hint)
        barrier()
        ts = time.perf_counter()
        for _ in range(args.steps):
            st = host_batch(eng, b.alg, False, d, buf.array, hint)
            st2 = host_batch(eng, b.alg, True, d, buf.array, hint)
        te = time.perf_counter()
        assert (st == 0).all() and (st2 == 0).all()
        dt = ctrl.max(te - ts)
        if rank == 0:
            print(json.dumps({
                "metric": {"host": "GiB/s host-resident (pinned arena, zero-copy: kernels load/store it over PCIe) ",
                           "host-staged": "GiB/s host-resident (pinned hipMemcpyAsync H2D + kernel + D2H, 3 streams) ",
                           }[args.mode]
                + ("AES-256-GCM seal+open, 1300 B pkts, 64 Ki batch" if cfg == 1 else
                   f"{'AES-256-GCM' if b.alg == L.ALG_AESGCM else 'ChaCha20-Poly1305'} seal+open ({workload_name})"),
                "value": round(2 * payload * args.steps * world / dt / GIB, 3), "unit": "GiB/s", "n_gpus": world,
                "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 4),
                "higher_is_better": True, "scaling": "weak", "data": "synthetic",
                "config": {"workload": workload_name.replace("device-resident", "host-resident pinned")},
            }), flush=True)
        return

    if args.mode == "tx":
        return bench_tx(args, eng, ctrl, rank, world)
    if args.mode == "rx":
        return bench_rx(args, eng, b, ciphers, ctrl, rank, world)
    if args.mode == "rx-device":
        return bench_rx_device(args, eng, b, ciphers, ctrl, rank, world)

    db = DeviceBatch(eng, b, ciphers)
    stream = torch.cuda.current_stream()
    # correctness gate before timing: one seal+open round trip must restore the plaintext
    db.seal()
    db.open()
    torch.cuda.synchronize()
    assert (db.status_host() == 0).all(), "round trip failed before timing"

    settled = settle(args, lambda: (db.seal(), db.open()))
    for _ in range(args.warmup):
        db.seal()
        db.open()
    torch.cuda.synchronize()
    # Kernel durations come from HIP events inside the timed region, on the launch stream. On every
    # EV_EVERY-th step the seal's and the open's dominant kernel (the single-key kernel, the mixed-key
    # chunk kernel, the ChaCha kernel) carry a start and a stop event bound to their own dispatch
    # (neb_time_next_kernel -> hipExtLaunchKernel): the kernel's own duration, with no marker packet
    # in the stream. Without a HIP handle (torch's events as the fallback) the events bracket the
    # calls as markers instead, and kernel_ms is then an upper bound.
    timed = [i for i in range(args.steps) if i % EV_EVERY == 0]
    ev = {i: tuple(TimingEvent() for _ in range(4)) for i in timed}
    bound = all(x.torch_ev is None for e in ev.values() for x in e)
    arm = L.lib().neb_time_next_kernel
    barrier()
    torch.cuda.synchronize()
    ts = time.perf_counter()
    for i in range(args.steps):
        e = ev.get(i)
        if e and bound:
            arm(e[0].h, e[1].h)
        elif e:
            e[0].record(stream)
        db.seal()
        if e and bound:
            arm(e[2].h, e[3].h)
        elif e:
            e[1].record(stream)
            e[2].record(stream)
        db.open()
        if e and not bound:
            e[3].record(stream)
    torch.cuda.synchronize()
    barrier()
    te = time.perf_counter()
    dt = te - ts
    seal_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in ev.values()]))
    open_ms = float(np.mean([e[2].elapsed_time(e[3]) for e in ev.values()]))
    call_ms = whole_seal_ms(db, stream)
    seal_kernel = ""
    if bound:  # the kernel the seal's events were bound to: one more armed (untimed) seal
        e0 = ev[timed[0]]
        arm(e0[0].h, e0[1].h)
        db.seal()
        seal_kernel = L.lib().neb_time_last_kernel().decode()
        db.open()
        torch.cuda.synchronize()
    st = db.status_host()
    assert (st == 0).all(), "open failed inside the timed region"
    dt = ctrl.max(dt)
    total_payload = ctrl.sum(2 * payload * args.steps)
    sus = sustained(args, ctrl, lambda: (db.seal(), db.open()), total_payload / args.steps, dt / args.steps * 1e3)
    assert (db.status_host() == 0).all(), "open failed in the sustained run"
    multi = hbm_over_ranks(ctrl, world, alg_bytes, seal_ms, ndev)

    if rank != 0:
        return
    value = total_payload / dt / GIB
    achieved = multi["per_gpu"]["achieved_mean"]  # GB/s, seal kernel (rank 0's alone at N = 1)
    alg_name = "AES-256-GCM" if b.alg == L.ALG_AESGCM else "ChaCha20-Poly1305"
    # the kernel the dispatch-bound events were bound to, as the library names it
    kern_tag = seal_kernel if bound else "event brackets around the whole seal call"
    # (shards: "C5/8" by tunnel, "C5/8r" by packet range)
    pmc = pmc_config(f"C{cfg + 1}" + (f"/{args.shard_of}{'r' if args.shard_by == 'range' else ''}"
                                      if cfg == 4 and args.shard_of else ""))
    lens = b.desc["len"].astype(np.int64)
    out = {
        "metric": "GiB/s device-resident AES-256-GCM seal+open, 1300 B pkts, 64 Ki batch"
        if cfg == 1 else f"GiB/s device-resident {alg_name} seal+open ({workload_name})",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "settle": settled,  # untimed, before the warmup (settle())
        "sustained": sus,  # after the timed steps: the rate over ~--sustain-ms of the same step (sustained())
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True,
        # C5 is one 1 Mi-packet batch split over the GPUs (BASELINE.json "sharded over 8xMI355X"):
        # the total is fixed; every other config gives each GPU a batch of its own
        "scaling": "strong" if cfg == 4 else "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic",
        "config": {"workload": workload_name, "packets_per_gpu": b.n,
                   "payload_bytes_per_pkt": int(lens[0]) if (lens == lens[0]).all() else
                   {"mean": round(float(lens.mean()), 1), "sizes": sorted(set(lens.tolist()))},
                   "keys": b.nkeys, "cipher": alg_name,
                   "parallelism": f"{world} GPU(s), independent packet shards, no collective"},
        "roofline": {
            "bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": round(achieved / HBM_PEAK_GBS, 4),
            "traffic": pmc["hbm_bytes_per_launch"] if pmc else None,
            "binding": {k: pmc[k] for k in ("lds_busy", "valu_busy", "mean_ns", "source") if k in pmc} if pmc else None,
            "kernel": kern_tag,
            # the seal's dominant kernel between start / stop events bound to its dispatch
            "kernel_ms": round(seal_ms, 4), "open_kernel_ms": round(open_ms, 4),
            # the whole seal call (mixed keys: with its binning passes) between marker events,
            # after the timed loop: a bound on the call, comparable across kernels and rounds
            "seal_call_ms": round(call_ms, 4),
            "seal_call_achieved": round(alg_bytes / (call_ms * 1e-3) / 1e9, 2),
            "kernel_timing": "dispatch-bound events" if bound else "marker events around the call",
            "algorithmic_bytes_per_launch": int(alg_bytes),
            # every rank's own seal kernel: per GPU (min / mean / max over ranks) and the whole job
            # against N x the HBM peak; devices = distinct GPUs the ranks ran on
            "per_gpu": multi["per_gpu"], "aggregate": multi["aggregate"],
        },
    }
    if world == 1 and not args.no_cpu_baseline:
        try:
            out["cpu_baseline"] = cpu_baseline(b)
        except Exception as e:  # the baseline is reported, never the product path
            log(f"cpu_baseline failed: {e!r}")
            out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def sustained(args, ctrl, step, payload_all_ranks: float, ms_per_step: float):
    """The rate over a long run of the same step after the timed region: ceil(--sustain-ms / the timed
    step time) more steps between a barrier and a device sync, the max time over ranks. `value` is
    the driver's K-step figure right after the settle; this one shows what a sustained load holds
    (the clocks of a long load sit a few % below the first second's)."""
    import math

    import torch

    if args.sustain_ms <= 0:
        return None
    n = max(1, math.ceil(args.sustain_ms / max(ms_per_step, 1e-3)))
    ctrl.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(n):
        step()
        if i % 64 == 63:
            torch.cuda.synchronize()  # (the host stays within 64 steps of the device)
    torch.cuda.synchronize()
    dt = ctrl.max(time.perf_counter() - t0)
    return {"steps": n, "ms": round(dt * 1e3, 1), "ms_per_step": round(dt / n * 1e3, 4),
            "value": round(payload_all_ranks * n / dt / GIB, 3)}


def whole_seal_ms(db, stream, reps: int = 4) -> float:
    """Mean time of the whole seal call (every kernel it launches) between marker events, each
    sealed batch opened back untimed so the arena stays valid; run after the timed loop."""
    import torch

    ts = []
    for _ in range(reps):
        a, z = TimingEvent(), TimingEvent()
        a.record(stream)
        db.seal()
        z.record(stream)
        db.open()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(z))
    return float(np.mean(ts))


def hbm_over_ranks(ctrl, world: int, alg_bytes: float, seal_ms: float, ndev: int) -> dict:
    """Every rank's seal-kernel bandwidth (algorithmic bytes / its own kernel time) over the ranks:
    per GPU min / mean / max and fraction of one GPU's HBM peak, and the whole job's sum against
    the peak of the distinct GPUs the ranks ran on (`devices`: N on a node, fewer only in a
    rehearsal that shares a device, whose ranks then split one GPU's HBM)."""
    ach = alg_bytes / (seal_ms * 1e-3) / 1e9
    tot = ctrl.sum(ach)
    lo, hi = -ctrl.max(-ach), ctrl.max(ach)
    mean = tot / world
    dev = min(world, max(ndev, 1))
    return {
        "per_gpu": {"achieved_min": round(lo, 2), "achieved_mean": round(mean, 2), "achieved_max": round(hi, 2),
                    "frac_mean": round(mean / HBM_PEAK_GBS, 4), "ranks": world},
        "aggregate": {"achieved": round(tot, 2), "peak": HBM_PEAK_GBS * dev, "unit": "GB/s",
                      "frac": round(tot / (HBM_PEAK_GBS * dev), 4), "devices": dev},
    }


def bench_stub(args, rank: int, world: int):
    """--stub (tests only): the launch and aggregation path without a GPU. Every rank reports a
    made-up kernel time of 0.1 x (rank + 1) ms over gloo, and rank 0 prints the JSON line."""
    from nebula_amd.shard import Control

    if os.environ.get("NEB_BENCH_STUB_FAIL") == str(rank):
        sys.exit(3)  # a rank that dies before the control plane is up
    ctrl = Control(world)
    ctrl.barrier()
    dt = ctrl.max(0.001 * (rank + 1))
    total = ctrl.sum(1.0 * GIB)
    multi = hbm_over_ranks(ctrl, world, 1e8, 0.1 * (rank + 1), world)  # (as if one GPU each)
    if rank == 0:
        print(json.dumps({"metric": "stub", "value": total / dt / GIB, "unit": "GiB/s", "n_gpus": world,
                          "steps": args.steps, "warmup": args.warmup, "ms_per_step": dt * 1e3,
                          "roofline": {"per_gpu": multi["per_gpu"], "aggregate": multi["aggregate"]}}), flush=True)
    if ctrl.dist is not None:
        ctrl.dist.destroy_process_group()


def bench_inproc(args):
    """--inproc: args.gpus engines in this one process, one per visible GPU (round-robin), each with
    its own batch of the config's shape (weak scaling, as the one-process-per-GPU mode); each step
    seals then opens every engine's batch through one neb_seal_batch_sharded / neb_open_batch_sharded
    call (every shard enqueued on its engine's stream before any is waited for)."""
    import ctypes as C

    import torch

    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import DeviceBatch, install_keys_multi
    from nebula_amd.noiseutil import Engine

    cfg, m = args.config, args.gpus
    ndev = max(1, torch.cuda.device_count())
    spec = {1: (L.ALG_AESGCM, 65536, 1), 2: (L.ALG_AESGCM, 65536, 4096), 3: (L.ALG_CHACHAPOLY, 65536, 4096)}
    engines, batches, dbs = [], [], []
    for k in range(m):
        dev = k % ndev
        torch.cuda.set_device(dev)
        b = W.make_batch(*spec[cfg], seed=W.SEED ^ k, name=f"C{cfg + 1}") if cfg in spec else W.config(4)
        if batches:
            b.keys = batches[0].keys  # one tunnel table over every engine (each its own packets)
        engines.append(Engine(dev, max_keys=4096))
        batches.append(b)
    # each tunnel key is one install on every engine (neb_cipher_create_multi): the sharded calls
    # refuse a shard whose engine holds another install in a slot its packets use
    ciphers = install_keys_multi(engines, batches[0])
    for e, b, cs in zip(engines, batches, ciphers):
        torch.cuda.set_device(e.device)
        dbs.append(DeviceBatch(e, b, cs))
    streams = [torch.cuda.Stream(device=db.dev) for db in dbs]
    arr = (L.Shard * m)()
    for k, (e, db) in enumerate(zip(engines, dbs)):
        arr[k] = L.Shard(e.handle.value, db.desc.data_ptr(), db.n, db.arena.data_ptr(), db.status.data_ptr(),
                         streams[k].cuda_stream)
    hint = dbs[0].key_hint
    if any(db.key_hint != hint for db in dbs):
        hint = L.KEYS_MIXED
    alg = batches[0].alg

    def step():
        L.check(L.lib().neb_seal_batch_sharded(alg, arr, m, hint), "seal_sharded")
        L.check(L.lib().neb_open_batch_sharded(alg, arr, m, hint), "open_sharded")

    step()
    assert all((db.status_host() == 0).all() for db in dbs)
    settled = settle(args, step)
    for _ in range(args.warmup):
        step()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step()
    dt = time.perf_counter() - t0
    assert all((db.status_host() == 0).all() for db in dbs), "open failed inside the timed region"
    payload = sum(float(b.payload_bytes) for b in batches)
    print(json.dumps({
        "metric": f"GiB/s device-resident seal+open, {m} engine(s) in one process (config {cfg + 1})",
        "value": round(2 * payload * args.steps / dt / GIB, 3), "unit": "GiB/s", "n_gpus": min(m, ndev),
        "engines": m, "steps": args.steps, "warmup": args.warmup, "settle": settled,
        "ms_per_step": round(dt / args.steps * 1e3, 4),
        "higher_is_better": True, "scaling": "weak", "dtype": "u8", "data": "synthetic",
        "config": {"workload": f"C{cfg + 1} per engine, {m} engine(s) over {ndev} visible device(s), one process, "
                               "neb_*_batch_sharded (no collective)"},
    }), flush=True)
    for cs in ciphers:
        for c in cs:
            c.destroy()
    for e in engines:
        e.close()


def bench_relay(args, ctrl, rank, world, device):
    """GMAC-only relay path: the relay seal (inside.go:491, empty plaintext) and
    VerifyRelay (connection_state.go:121-148) of 64 Ki relayed packets, AD = 1348 B each, one key
    (--config 1) or 4096 (--config 2; --config 3: ChaCha20-Poly1305, 4096 keys). Every round of these waves is AAD-only, so the kernels skip
    the AES except for E_K(J0). value = AD bytes sealed + verified per second."""
    import torch

    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import DeviceBatch, install_keys
    from nebula_amd.noiseutil import Engine

    nkeys = 4096 if args.config in (2, 3) else 1
    alg = L.ALG_CHACHAPOLY if args.config == 3 else L.ALG_AESGCM
    b = W.relay_batch(alg, 65536, nkeys, seed=W.SEED ^ rank)
    eng = Engine(device, max_keys=4096)
    db = DeviceBatch(eng, b, install_keys(eng, b))
    db.seal()
    db.open()
    torch.cuda.synchronize()
    assert (db.status_host() == 0).all(), "relay round trip failed before timing"
    settled = settle(args, lambda: (db.seal(), db.open()))
    for _ in range(args.warmup):
        db.seal()
        db.open()
    torch.cuda.synchronize()
    ctrl.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        db.seal()
        db.open()
    torch.cuda.synchronize()
    dt = ctrl.max(time.perf_counter() - t0)
    assert (db.status_host() == 0).all(), "relay verify failed inside the timed region"
    if rank == 0:
        ad = float(b.desc["aad_len"].astype(np.int64).sum())
        print(json.dumps({
            "metric": "GiB/s relay AD (" + ("Poly1305-only ChaCha20-Poly1305" if alg == L.ALG_CHACHAPOLY else
                                           "GMAC-only AES-256-GCM") + " seal + VerifyRelay), device-resident",
            "value": round(2 * ad * args.steps * world / dt / GIB, 3), "unit": "GiB/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "settle": settled,
            "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "dtype": "u8", "data": "synthetic",
            "config": {"workload": f"65536 relayed packets, AD 1348 B, empty plaintext, {nkeys} key(s)"},
        }), flush=True)


def tso_superpackets(nseg_total: int, mss: int = 1448, seed: int = 7):
    """IPv4/TCP TSO superpackets of 45 x 1448 B (64 KiB class) carrying nseg_total segments."""
    import struct

    rng = np.random.default_rng(seed)
    per = 45  # 40 + 45 x 1448 = 65200 B <= 64 KiB
    nsp = (nseg_total + per - 1) // per
    size = 40 + per * mss
    stride = (size + 15) & ~15
    arena = np.zeros(nsp * stride + 64, np.uint8)
    hdr = bytearray(40)
    hdr[0] = 0x45
    struct.pack_into(">H", hdr, 2, size)
    hdr[8], hdr[9] = 64, 6
    hdr[12:16], hdr[16:20] = bytes([10, 0, 0, 1]), bytes([10, 0, 0, 2])
    struct.pack_into(">HHII", hdr, 20, 40000, 443, 1, 1)
    hdr[32], hdr[33] = 0x50, 0x18
    for i in range(nsp):
        o = i * stride
        arena[o:o + 40] = np.frombuffer(bytes(hdr), np.uint8)
        arena[o + 40:o + size] = rng.integers(0, 256, size - 40, dtype=np.uint8)
    return arena, nsp, size, stride, per


def bench_tx(args, eng, ctrl, rank, world):
    import torch

    from nebula_amd import _lib as L
    from nebula_amd.inside import TX_PACKET_DTYPE, TX_TUNNEL_DTYPE, DeviceTxBatch, slot_bytes
    from nebula_amd.noiseutil import CipherAESGCM

    mss = 1448
    arena, nsp, size, stride, per = tso_superpackets(45 * args.tx_superpackets, mss)
    key = CipherAESGCM.Cipher(eng, bytes(range(32)))
    tun = np.zeros(1, TX_TUNNEL_DTYPE)
    tun[0] = (2, key.key_id, 0xBEEF)
    pk = np.zeros(nsp, TX_PACKET_DTYPE)
    for i in range(nsp):
        pk[i] = (i * stride, size, 0, 1, 1, 40, mss, 20, 16, 0)
    nwire = nsp * per
    db = DeviceTxBatch(eng, L.ALG_AESGCM, tun, pk, arena, nwire * slot_bytes(40 + mss), nwire, key.key_id)
    db.seal()
    torch.cuda.synchronize()
    r = db.result()
    assert len(r.wires) == nwire and (r.wire_status == 0).all() and (r.packet_status == 0).all()
    settled = settle(args, db.seal)
    for _ in range(args.warmup):
        db.seal()
    torch.cuda.synchronize()
    ctrl.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        db.seal()
    torch.cuda.synchronize()
    dt = ctrl.max(time.perf_counter() - t0)
    if rank == 0:
        tun_bytes = float(nsp * size) * args.steps * world
        print(json.dumps({
            "metric": "GiB/s TUN bytes in, device TX batch (TSO 64 KiB superpackets -> segment + checksum + "
                      "header + AES-256-GCM seal)",
            "value": round(tun_bytes / dt / GIB, 3), "unit": "GiB/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "settle": settled, "ms_per_step": round(dt / args.steps * 1e3, 4),
            "higher_is_better": True, "scaling": "weak", "dtype": "u8", "data": "synthetic",
            "wire_packets_per_s": round(nwire * args.steps * world / dt, 1),
            "config": {"workload": f"{nsp} IPv4/TCP TSO superpackets x {per} segments of {mss} B "
                                   f"({nwire} wire packets), 1 tunnel, device-resident"},
        }), flush=True)


def bench_rx(args, eng, b, ciphers, ctrl, rank, world):
    """Batched receive (host arena, replay windows) vs the plain host-resident open of the same batch."""
    from nebula_amd import _lib as L
    from nebula_amd.batch import PinnedBuffer, host_batch, slot_desc
    from nebula_amd.connection_state import Bits, ReplayWindow, rx_open_batch

    d = slot_desc(b, ciphers)
    buf = PinnedBuffer(b.arena.nbytes)
    buf.array[:] = b.arena
    hint = int(d["key_id"][0]) if b.nkeys == 1 else L.KEYS_MIXED
    st = host_batch(eng, b.alg, False, d, buf.array, hint)
    assert (st == 0).all()
    sealed = buf.array.copy()
    nkeys = eng.max_keys
    times = {"rx": 0.0, "open": 0.0}
    for it in range(args.warmup + args.steps):
        for mode in ("rx", "open"):
            buf.array[:] = sealed
            wins = [None] * nkeys
            if mode == "rx":
                for c in ciphers:
                    wins[c.key_id] = Bits(ReplayWindow)
            t0 = time.perf_counter()
            if mode == "rx":
                st = rx_open_batch(eng, b.alg, wins, d, buf.array, hint)
            else:
                st = host_batch(eng, b.alg, True, d, buf.array, hint)
            el = time.perf_counter() - t0
            assert (st == 0).all(), mode
            if it >= args.warmup:
                times[mode] += el
    if rank == 0:
        payload = float(b.payload_bytes) * args.steps
        print(json.dumps({
            "metric": "GiB/s host-resident batched receive (replay window Check -> GPU open -> Update)",
            "value": round(payload / times["rx"] / GIB, 3), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "higher_is_better": True, "dtype": "u8", "data": "synthetic",
            "open_only_gibs": round(payload / times["open"] / GIB, 3),
            "config": {"workload": f"{b.name}: {b.n} packets, {b.nkeys} tunnel(s), host pinned arena"},
        }), flush=True)


def bench_rx_device(args, eng, b, ciphers, ctrl, rank, world):
    """Batched receive with the batch and the replay windows in device memory (neb_rx_open_batch)
    against the plain device open of the same batch. Every step receives the next batch of the
    same tunnels (counters advanced by n, re-sealed untimed), so every packet passes its window."""
    import torch

    from nebula_amd import _lib as L
    from nebula_amd.batch import DeviceBatch
    from nebula_amd.connection_state import Bits, DeviceWindows, ReplayWindow, rx_open_batch_device

    db = DeviceBatch(eng, b, ciphers)
    pt = db.arena.clone()
    base = db.desc_host.copy()
    dw = DeviceWindows(eng, eng.max_keys, ReplayWindow)
    for c in ciphers:
        w = Bits(ReplayWindow)
        w.Update(1)
        w.Update(2)
        dw.load(c.key_id, w)
    settled = settle(args, lambda: (db.seal(), db.open()))
    times = {"rx": 0.0, "open": 0.0}
    for it in range(args.warmup + args.steps):
        d = base.copy()
        d["counter"] = d["counter"] + np.uint64(it * b.n)
        db.desc.copy_(torch.from_numpy(d.view(np.uint8)))
        for mode in ("open", "rx"):
            db.arena.copy_(pt)
            db.seal()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            if mode == "rx":
                rx_open_batch_device(eng, b.alg, dw, db.desc, db.arena, db.status, db.key_hint,
                                     torch.cuda.current_stream().cuda_stream)
            else:
                db.open()
            torch.cuda.synchronize()
            el = time.perf_counter() - t0
            st = db.status_host()
            assert (st == 0).all(), (mode, np.unique(st))
            if it >= args.warmup:
                times[mode] += el
    dw.destroy()
    if rank == 0:
        payload = float(b.payload_bytes) * args.steps
        print(json.dumps({
            "metric": "GiB/s device-resident batched receive (replay windows in HBM: Check -> open -> Update)",
            "value": round(payload / times["rx"] / GIB, 3), "unit": "GiB/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "settle": settled, "higher_is_better": True, "dtype": "u8", "data": "synthetic",
            "ms_per_step": round(times["rx"] / args.steps * 1e3, 4),
            "open_only_gibs": round(payload / times["open"] / GIB, 3),
            "open_only_ms": round(times["open"] / args.steps * 1e3, 4),
            "config": {"workload": f"{b.name}: {b.n} packets, {b.nkeys} tunnel(s), device-resident, "
                                   f"windows of {ReplayWindow}"},
        }), flush=True)


if __name__ == "__main__":
    main()
