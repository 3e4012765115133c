"""Memory-side byte floors of a bench config's seal launch, for reading the PMC traffic
(profiles/pmc_configs.json) against: the algorithmic bytes (what bench.py's roofline counts), the
bytes of the distinct 64-B / 128-B lines the batch touches (every packet's AAD + payload read, its
payload + tag written; neighbours share boundary lines), and the same with every packet's lines
counted on their own plus one 128-B line per descriptor — what a kernel that visits packets in
key order (the mixed-key chunks, not slot order) fetches when a boundary line's two packets run
far apart in time.
usage: python tools/line_floor.py [config numbers, default 1 2 4]
"""
import sys

import os

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

from nebula_amd import workload as W


def distinct_lines(off, ln, g):
    lo, hi = off // g, (off + ln + g - 1) // g
    order = np.argsort(lo, kind="stable")
    lo, hi = lo[order], hi[order]
    # union of [lo, hi) intervals: running max of hi
    run = np.maximum.accumulate(hi)
    prev = np.concatenate([[lo[0]], run[:-1]])
    return int(np.sum(np.maximum(hi - np.maximum(lo, prev), 0)))


def own_lines(off, ln, g):
    return int(np.sum((off + ln + g - 1) // g - off // g))


def main():
    cfgs = [int(x) for x in sys.argv[1:]] or [1, 2, 4]
    for c in cfgs:
        b = W.config(c)
        d = b.desc
        ln = d["len"].astype(np.int64)
        so, do, ao, al = (d[k].astype(np.int64) for k in ("src_off", "dst_off", "aad_off", "aad_len"))
        algo = int((al + ln).sum() + (ln + 16).sum())
        ro, rl = np.concatenate([ao, so]), np.concatenate([al, ln])
        out = {"config": f"C{c + 1}", "packets": b.n, "algorithmic_bytes": algo}
        for g in (64, 128):
            out[f"shared_{g}B_lines_bytes"] = (distinct_lines(ro, rl, g) + distinct_lines(do, ln + 16, g)) * g
        # AAD and payload are adjacent in a slot: one read range per packet
        rd = own_lines(np.minimum(ao, so), np.maximum(ao + al, so + ln) - np.minimum(ao, so), 128) * 128
        wr = own_lines(do, ln + 16, 64) * 64
        out["own_lines_bytes"] = rd + wr + b.n * 128
        print(out)


if __name__ == "__main__":
    main()
