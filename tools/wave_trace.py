"""Wave timeline of the AES-GCM kernels (gcm_chunk_kernel; gcm_single_kernel for --config 1) on one batch.

Needs the trace build (tools/build_variant.sh wtrace -DNEB_WAVE_TRACE=1) selected with
NEB_LIB_PATH=build_abl/wtrace/libnebula_aead.so. Seals (and opens) a BASELINE config once after a
warmup, fetches the per-chunk records (neb_debug_wave_trace) and reports where the kernel's time
goes: the span, when each workgroup (one per CU) finishes, how many waves hold a chunk over time,
and chunk durations by kind.

  python tools/wave_trace.py --config 2 --out gpurun_out/wave_trace_c3.json
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

TICK_NS = 10.0  # s_memrealtime: 100 MHz


def fetch(lib):
    cap = 64 * 8192  # kWaveTraceSlots x kWaveTraceWaves
    buf = np.zeros((cap, 4), dtype=np.uint32)
    n = lib.neb_debug_wave_trace(buf.ctypes.data_as(ctypes.c_void_p), ctypes.c_uint32(cap))
    if n < 0:
        raise RuntimeError("neb_debug_wave_trace failed")
    buf = buf[:n]
    buf = buf[(buf[:, 0] >> 31) == 1]
    buf[:, 0] &= 0x7FFFFFFF
    return buf.copy()


def analyse(tr, waves_per_wg=16):
    a, c, t0, t1 = (tr[:, i].astype(np.int64) for i in range(4))
    # phase records (trace build, round 6): per chunk {descriptor in | round keys in << 16, tables
    # staged} and the groups' sums {desc | rounds << 16, final | finish << 16}, in 10-ns ticks
    pa, pb = c == 0xFFFFFFFE, c == 0xFFFFFFFD
    phases = None
    if pa.any() and pb.any():
        lo, hi = lambda x: (x & 0xFFFF) * TICK_NS / 1e3, lambda x: (x >> 16) * TICK_NS / 1e3
        phases = {"chunk_desc": lo(t0[pa]), "round_keys": hi(t0[pa]), "stage": t1[pa] * TICK_NS / 1e3,
                  "pkt_desc": lo(t0[pb]), "rounds": hi(t0[pb]), "final": lo(t1[pb]), "finish": hi(t1[pb])}
    keep = ~(pa | pb)
    a, c, t0, t1 = a[keep], c[keep], t0[keep], t1[keep]
    t1 = np.where(t1 < t0, t1 + (1 << 32), t1)
    wg, wave = a >> 20, (a >> 16) & 15
    start = c == 0xFFFFFFFF
    ch = ~start
    k0 = t0[start].min()
    span = (t1[ch].max() - k0) * TICK_NS / 1e3
    prologue = (t1[start] - t0[start]) * TICK_NS / 1e3
    count, lg, full = (a >> 8) & 255, (a >> 4) & 15, a & 1
    dur = (t1 - t0) * TICK_NS / 1e3
    out = {"span_us": round(float(span), 2), "chunks": int(ch.sum()), "workgroups": int(len(np.unique(wg))),
           "prologue_us_mean": round(float(prologue.mean()), 2), "prologue_us_max": round(float(prologue.max()), 2)}
    # when each workgroup's last chunk ends, relative to the kernel's first wave start
    wg_end = {}
    for g, e in zip(wg[ch], t1[ch]):
        wg_end[g] = max(wg_end.get(g, 0), e)
    ends = (np.array(list(wg_end.values())) - k0) * TICK_NS / 1e3
    out["wg_end_us"] = {p: round(float(np.percentile(ends, p)), 2) for p in (0, 10, 50, 90, 99, 100)}
    # per wave: busy time (inside chunks) over the span
    busy = dur[ch].sum()
    nw = len(np.unique(a[start] >> 16))
    out["wave_busy_frac"] = round(float(busy / (nw * span)), 4)
    # waves holding a chunk over time (1 us bins)
    nb = int(np.ceil(span)) + 1
    act = np.zeros(nb)
    for s_, e_ in zip((t0[ch] - k0) * TICK_NS / 1e3, (t1[ch] - k0) * TICK_NS / 1e3):
        i0, i1 = int(s_), int(np.ceil(e_))
        act[i0:i1] += 1
    step = max(1, nb // 40)
    out["active_waves_per_us"] = [int(x) for x in act[::step]]
    out["active_waves_step_us"] = step
    if phases is not None:
        out["phase_us_mean"] = {k: round(float(v.mean()), 2) for k, v in phases.items()}
        out["phase_us_total_per_wave"] = {k: round(float(v.sum()) / max(1, len(np.unique(a[start] >> 16))), 2)
                                          for k, v in phases.items()}
    # chunk durations by kind
    kinds = {}
    for f, l, n_, d in zip(full[ch], lg[ch], count[ch], dur[ch]):
        key = f"{'front' if f else 'back'} lg{l} " + ("16" if n_ >= 16 else ("9-15" if n_ >= 9 else "1-8"))
        kinds.setdefault(key, []).append(d)
    out["chunk_us"] = {k: {"n": len(v), "mean": round(float(np.mean(v)), 2), "max": round(float(np.max(v)), 2)}
                       for k, v in sorted(kinds.items())}
    # mean chunk duration by wave index in the workgroup (index // 4 is the wave's age rank on its
    # SIMD: a workgroup's waves go to the SIMDs in turn) and the order the waves finish in
    out["chunk_us_by_wave"] = [round(float(dur[ch & (wave == w)].mean()), 2) for w in range(waves_per_wg)
                               if (ch & (wave == w)).any()]
    # chunks per wave
    per_wave = np.bincount((wg[ch] * waves_per_wg + wave[ch]).astype(np.int64))
    out["chunks_per_wave"] = {int(k): int(v) for k, v in zip(*np.unique(per_wave, return_counts=True))}
    # per workgroup, on its own clock (s_memrealtime may be offset between XCDs): its span from its
    # first wave's start, and how many of its waves hold a chunk over that span (mean over workgroups)
    spans, prof = [], np.zeros(64)
    for g in np.unique(wg):
        m = wg == g
        g0 = t0[m & start].min()
        gs = (t1[m & ch].max() - g0) * TICK_NS / 1e3
        spans.append(gs)
        for s_, e_ in zip(t0[m & ch], t1[m & ch]):  # 64 bins over the workgroup's span
            i0 = int((s_ - g0) * TICK_NS / 1e3 / gs * 64)
            i1 = int(np.ceil((e_ - g0) * TICK_NS / 1e3 / gs * 64))
            prof[i0:min(i1, 64)] += 1
    spans = np.array(spans)
    out["wg_span_us"] = {p: round(float(np.percentile(spans, p)), 2) for p in (0, 10, 50, 90, 100)}
    out["wg_active_waves_profile"] = [round(float(x), 1) for x in prof / len(spans)]
    # workgroup start offsets by blockIdx mod 8 (the XCD a workgroup usually lands on)
    st = {}
    for g, t in zip(wg[start], t0[start]):
        st[g] = min(st.get(g, t), t)
    out["wg_start_us_by_mod8"] = {int(x): round(float((np.median([v for g, v in st.items() if g % 8 == x]) - k0) *
                                                     TICK_NS / 1e3), 2) for x in range(8)}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--config", type=int, default=2)
    ap.add_argument("--out", default=None)
    ap.add_argument("--shard-of", type=int, default=0, help="--config 4: shard 0 of the 1 Mi batch split N ways")
    ap.add_argument("--shard-by", choices=["key", "range"], default="key")
    args = ap.parse_args()
    if args.out:
        os.makedirs(os.path.dirname(args.out), exist_ok=True)
    import torch

    from nebula_amd import _lib as L
    from nebula_amd import workload as W
    from nebula_amd.batch import DeviceBatch, install_keys
    from nebula_amd.noiseutil import Engine

    assert os.environ.get("NEB_LIB_PATH"), "set NEB_LIB_PATH to the trace build"
    lib = L.lib()
    lib.neb_debug_wave_trace.restype = ctypes.c_int
    lib.neb_debug_wave_trace.argtypes = [ctypes.c_void_p, ctypes.c_uint32]
    b = {1: lambda: W.make_batch(L.ALG_AESGCM, 65536, 1, name="C2"),
         2: lambda: W.make_batch(L.ALG_AESGCM, 65536, 4096, name="C3"),
         4: lambda: (W.shard_by_key if args.shard_by == "key" else W.shard)(W.config(4), 0, args.shard_of)
         if args.shard_of else W.config(4)}[args.config]()
    eng = Engine(0, max_keys=max(4096, b.nkeys))
    ciphers = install_keys(eng, b)
    db = DeviceBatch(eng, b, ciphers)
    import time
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # settle the clocks (bench.py settle())
        for _ in range(8):
            db.seal()
            db.open()
        torch.cuda.synchronize()
    fetch(lib)
    res = {}
    for name, fn in (("seal", db.seal), ("open", db.open)):
        fn()
        torch.cuda.synchronize()
        tr = fetch(lib)
        res[name] = analyse(tr)
        if args.out:
            np.save(args.out.replace(".json", f"_{name}.npy"), tr)
    assert (db.status_host() == 0).all()
    s = json.dumps(res, indent=1)
    print(s)
    if args.out:
        open(args.out, "w").write(s)


if __name__ == "__main__":
    main()
