"""Condense a tools/profile.sh run (gpurun_out/prof_<tag>) into profiles/<tag>/: the kernel-trace
stats CSV and, per counter pass, the mean value of every counter per kernel (pmc_<pass>.json).
usage: python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>
"""
import collections
import csv
import glob
import json
import os
import shutil
import sys


def main():
    src, dst = sys.argv[1], sys.argv[2]
    os.makedirs(dst, exist_ok=True)
    for f in glob.glob(os.path.join(src, "trace", "*kernel_stats.csv")):
        shutil.copy(f, os.path.join(dst, "trace_kernel_stats.csv"))
    for d in sorted(glob.glob(os.path.join(src, "*"))):
        name = os.path.basename(d)
        files = glob.glob(os.path.join(d, "*counter_collection.csv"))
        if not files:
            continue
        vals = collections.defaultdict(lambda: collections.defaultdict(list))
        for r in csv.DictReader(open(files[0])):
            vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
        out = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()}
        json.dump(out, open(os.path.join(dst, f"pmc_{name}.json"), "w"), indent=1, sort_keys=True)
    print("wrote", dst)


if __name__ == "__main__":
    main()
