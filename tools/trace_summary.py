"""Per-kernel mean duration from rocprofv3 kernel_trace.csv files: tools/trace_summary.py DIR..."""
import csv
import glob
import sys
from collections import defaultdict

for d in sys.argv[1:]:
    for f in sorted(glob.glob(f"{d}/**/*kernel_trace.csv", recursive=True)):
        agg = defaultdict(list)
        for r in csv.DictReader(open(f)):
            agg[r["Kernel_Name"]].append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
        print("==", f)
        for k, v in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
            if "rocclr" in k or "key_setup" in k:
                continue
            print(f"  {k[:70]:70s} n={len(v):5d} mean={sum(v) / len(v) / 1e3:8.1f} us")
