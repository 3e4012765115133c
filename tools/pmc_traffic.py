"""Condense rocprofv3 FETCH_SIZE / WRITE_SIZE passes (tools/profile.sh) into
profiles/pmc_traffic.json: HBM bytes per launch for each kernel.

Per MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reports half the bytes of wide coalesced streaming
reads on gfx950 (16 B/lane global loads, which is what the AEAD kernels issue), so it is doubled;
WRITE_SIZE (KiB) is exact for 16 B/lane stores.
usage: python tools/pmc_traffic.py gpurun_out/prof_<tag> [more prof dirs...] [--out out.json]
"""
import collections
import csv
import json
import os
import re
import sys


def short(name):
    m = re.search(r"neb::(\w+<[^>]*>|\w+)\(", name)
    return m.group(1) if m else name


def main():
    args = sys.argv[1:]
    out = os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json")
    if "--out" in args:
        i = args.index("--out")
        out = args[i + 1]
        del args[i:i + 2]
    bases = args
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    for base in bases:
        for tag in ("fetch", "write"):
            for r in csv.DictReader(open(os.path.join(base, tag, f"{tag}_counter_collection.csv"))):
                vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    kernels = {}
    for k, c in vals.items():
        if "FETCH_SIZE" not in c or "WRITE_SIZE" not in c:
            continue
        f = sum(c["FETCH_SIZE"]) / len(c["FETCH_SIZE"])
        w = sum(c["WRITE_SIZE"]) / len(c["WRITE_SIZE"])
        kernels[k] = {"fetch_size_kib": round(f, 1), "write_size_kib": round(w, 1),
                      "hbm_bytes_per_launch": int(2 * f * 1024 + w * 1024), "launches": len(c["FETCH_SIZE"])}
    json.dump({"source": [os.path.relpath(b) for b in bases], "correction": "bytes = 2*FETCH_SIZE*1024 + WRITE_SIZE*1024",
               "kernels": kernels}, open(out, "w"), indent=1)
    print(json.dumps(kernels, indent=1))


if __name__ == "__main__":
    main()
