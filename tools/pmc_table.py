"""Per-kernel mean of every counter in rocprofv3 --pmc passes (counter_collection.csv files under a
directory): one row per kernel, one column per counter. Usage: pmc_table.py DIR [name filter]."""
import collections
import csv
import glob
import os
import sys


def main():
    d = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        per = collections.defaultdict(float)  # (dispatch, kernel, counter) -> summed over agents/dims
        for r in csv.DictReader(open(f)):
            per[(r["Dispatch_Id"], r["Kernel_Name"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (disp, k, c), v in per.items():
            acc[k][c].append(v)
    for k, cs in sorted(acc.items()):
        if filt not in k:
            continue
        print(k[:90])
        for c, vs in sorted(cs.items()):
            print(f"    {c:28s} {sum(vs) / len(vs):16.1f}   (n={len(vs)})")


if __name__ == "__main__":
    main()
