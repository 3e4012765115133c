"""Idle gaps between consecutive kernels of one queue from rocprofv3 kernel_trace.csv files.

tools/trace_gaps.py DIR [NAME_SUBSTR...]: for the kernels whose name contains one of the substrings
(default: every kernel except the runtime's copy/fill helpers and key setup), prints the mean
duration per kernel and the gaps (previous end -> next start) between back-to-back launches in the
longest run of such launches — the part of a bench step that is not kernel time.
"""
import csv
import glob
import statistics
import sys

d = sys.argv[1]
subs = sys.argv[2:]
for f in sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)):
    rows = []
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        if subs and not any(s in k for s in subs):
            continue
        if not subs and ("rocclr" in k or "key_setup" in k or "at::native" in k):
            continue
        rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), k))
    rows.sort()
    if not rows:
        continue
    gaps = [(rows[i + 1][0] - rows[i][1], rows[i][2][:40], rows[i + 1][2][:40]) for i in range(len(rows) - 1)]
    # the timed region: gaps under 200 us (warmup / setup gaps are host-bound and much longer)
    g = [x for x in gaps if x[0] < 200_000]
    print("==", f, f"{len(rows)} launches")
    by = {}
    for s, e, k in rows:
        by.setdefault(k[:70], []).append(e - s)
    for k, v in by.items():
        print(f"  {k:70s} n={len(v):4d} mean={statistics.mean(v) / 1e3:8.2f} us")
    pairs = {}
    for x, a, b in g:
        pairs.setdefault((a, b), []).append(x)
    for (a, b), v in pairs.items():
        print(f"  gap {a} -> {b}: n={len(v)} median={statistics.median(v) / 1e3:.2f} us "
              f"min={min(v) / 1e3:.2f} max={max(v) / 1e3:.2f}")
