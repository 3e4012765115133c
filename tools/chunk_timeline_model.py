"""Processor-sharing model of gcm_chunk_kernel's workgroups on C3.

One workgroup per CU with 16 wave slots. The kernel deals the chunk list (fronts, then long tails,
then short tails, each kind longest first) to the workgroups as chunks w, w + G, w + 2G, ...; a
workgroup's waves draw its chunks in order as they finish. A round (one 16-B block per lane) takes
max(L, w * T16 / 16) us when w waves of the CU are running: throughput-bound at full occupancy
(T16 = 5.1 us with 16 waves, measured), latency-bound at L with few waves. Prints the kernel span
(the slowest workgroup) and the bound with every wave-round at full occupancy.

  python tools/chunk_timeline_model.py [L_us] [overhead_rounds_per_chunk]
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
sys.path.insert(0, ROOT)
import sched_model as M  # noqa: E402
from nebula_amd import workload as W  # noqa: E402

T16 = 5.1   # us per round with 16 waves on the CU (tools/wave_trace.py, round 3)
WAVES = 16
CUS = 256


def chunk_rounds(ch, nblk):
    lpp = 1 << ch.lg
    per = 64 // lpp
    return sum(int(((nblk[ch.packets[g:g + per]] + lpp - 1) // lpp).max()) for g in range(0, len(ch.packets), per))


def workgroup_span(items, lat, ov):
    queue = list(items)
    run = [queue.pop(0) + ov for _ in range(min(WAVES, len(queue)))]
    t = 0.0
    while run:
        rt = max(lat, len(run) * T16 / WAVES)
        m = min(run)
        t += m * rt
        nxt = []
        for r in run:
            r -= m
            if r <= 1e-9:
                if queue:
                    nxt.append(queue.pop(0) + ov)
            else:
                nxt.append(r)
        run = nxt
    return t


def main(lat=3.2, ov=1.0):
    n = 65536
    kid = W.key_ids(n, 4096)
    lens = W.payload_lens(n, (1300,), (1,))
    aad = np.full(n, 16, np.uint32)
    plan = M.plan(kid, aad, lens, 4096)
    nblk = M.blocks(aad, lens)
    order = sorted(plan, key=lambda c: c.bucket)  # the kernel's order: cost buckets, longest first
    rounds = [chunk_rounds(c, nblk) for c in order]
    spans = [workgroup_span(rounds[w::CUS], lat, ov) for w in range(CUS)]
    bound = (sum(rounds) + ov * len(rounds)) / CUS * T16 / WAVES
    return max(spans), float(np.median(spans)), bound


if __name__ == "__main__":
    lat = float(sys.argv[1]) if len(sys.argv) > 1 else 3.2
    ov = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    mx, med, bound = main(lat, ov)
    print(f"span {mx:.1f} us (median workgroup {med:.1f}), all rounds at full occupancy {bound:.1f} us")
