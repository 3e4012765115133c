#!/usr/bin/env python3
"""VALU issue accounting of a rocprofv3 counter pass.

gfx950 issues a wave64 VALU instruction in one quad-cycle (4 cycles) per SIMD, and two VOP1/VOP2
instructions of two different waves of the same SIMD in one quad-cycle (SQ_ACTIVE_INST_VALU2 counts
the second of each pair; tools/micro/valu_pair.hip: one dependent chain per lane pairs as well as 8,
one wave per SIMD never pairs, VOP3 / DPP never pair). So the SIMD's VALU-busy cycles are
4 x (SQ_INSTS_VALU - SQ_ACTIVE_INST_VALU2) / SIMDs, and the issue fraction is that over
SQ_BUSY_CU_CYCLES / CUs (valu_mix: 0.96-0.99 for every single-instruction kernel).

usage: valu_issue.py COUNTER_CSV [--kernel SUBSTR] [--units N] [--cus 256]
  --units: work units per dispatch (e.g. 16384 four-packet groups) for per-unit counts
"""
import argparse
import collections
import csv
import json


def summarize(path, kernel=None, units=None, cus=256):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"]
        if kernel and kernel not in k:
            continue
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k].add(r["Dispatch_Id"])
    out = []
    for k, v in agg.items():
        n = len(disp[k])
        m = {c: x / n for c, x in v.items()}
        vi = m.get("SQ_INSTS_VALU", 0.0)
        if vi < 1e5:
            continue
        rec = {"kernel": k, "dispatches": n, "per_dispatch": {c: round(x) for c, x in m.items()}}
        busy = m.get("SQ_BUSY_CU_CYCLES", 0.0) / cus
        if busy and "SQ_ACTIVE_INST_VALU2" in m:
            simd = 4 * cus
            rec["cu_busy_cycles"] = round(busy)
            rec["valu_cycles_per_simd"] = round(4 * (vi - m["SQ_ACTIVE_INST_VALU2"]) / simd)
            rec["valu_issue_frac"] = round(4 * (vi - m["SQ_ACTIVE_INST_VALU2"]) / simd / busy, 4)
            rec["valu_frac_no_coissue"] = round(4 * vi / simd / busy, 4)
            rec["coissued_frac"] = round(m["SQ_ACTIVE_INST_VALU2"] / vi, 4)
        if units:
            rec["per_unit"] = {c: round(x / units, 1) for c, x in m.items() if c.startswith("SQ_INSTS")}
        out.append(rec)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--kernel")
    ap.add_argument("--units", type=float)
    ap.add_argument("--cus", type=int, default=256)
    a = ap.parse_args()
    for rec in summarize(a.csv, a.kernel, a.units, a.cus):
        print(json.dumps(rec))


if __name__ == "__main__":
    main()
