#!/bin/bash
# One counter pass per variant (the product build "base" or build_abl/<name>) over a bench config,
# condensed to gpurun_out/pmc_ab/<variant>.json (per kernel, the mean of each counter).
#   tools/pmc_ab.sh "<variants>" "<counters (one pass: <= 8 SQ, <= 4 TCC)>" "<bench args>"
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/pmc_ab; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in $1; do
    if [ "$v" = base ]; then unset NEB_LIB_PATH; else export NEB_LIB_PATH=$R/build_abl/$v/libnebula_aead.so; fi
    rm -rf $OUT/raw_$v
    timeout -s KILL 120 rocprofv3 --pmc $2 --output-format csv -d $OUT/raw_$v -o p -- python3 $R/bench.py --no-cpu-baseline $3 > $OUT/$v.log 2>&1 || { echo "$v rc=$?"; tail -5 $OUT/$v.log; exit 1; }
    python3 - "$OUT/raw_$v" "$OUT/$v.json" <<'PY'
import collections, csv, glob, json, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for r in csv.DictReader(open(f)):
    vals[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
out = {k: {c: sum(x) / len(x) for c, x in cs.items()} for k, cs in vals.items()}
json.dump(out, open(sys.argv[2], "w"), indent=1, sort_keys=True)
for k, cs in out.items():
    if "chunk_kernel<false>" in k or "single_kernel<false, false>" in k:
        print(sys.argv[2].split("/")[-1], k[:40], {c: round(v) for c, v in cs.items()})
PY
    rm -rf $OUT/raw_$v
done
