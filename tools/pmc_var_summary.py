"""Mean counter values of the seal kernels in rocprofv3 output dirs (tools/pmc_variants.sh)."""
import collections
import csv
import glob
import os
import sys

for d in sys.argv[1:]:
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    if not files:
        continue
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(files[0])):
        k = r["Kernel_Name"]
        if "kernel<false>" in k:
            vals[k.split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, cs in vals.items():
        print(os.path.basename(d), k, {c: f"{sum(v) / len(v):.4g}" for c, v in sorted(cs.items())})
