#!/bin/bash
# One LDS counter pass per build_abl variant on the C2 bench (GPU box): bank conflicts, LDS-array
# cycles, CU-busy cycles, LDS and VALU instruction counts of the single-key kernels.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for v in $(cat $R/build_abl/variants.txt); do
  OUT=$R/gpurun_out/pmcab_$v; mkdir -p $OUT
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_BUSY_CU_CYCLES SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_CMD_FIFO_FULL --output-format csv -d $OUT -o lds -- python3 $R/bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/run.log 2>&1 || exit 1
  python3 - $OUT <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if "single_kernel<false>" in r["Kernel_Name"]:
        v[r["Counter_Name"]].append(float(r["Counter_Value"]))
m = {k: sum(x) / len(x) for k, x in v.items()}
print(sys.argv[1].split("_")[-1], {k: round(x / 1e6, 2) for k, x in m.items()}, "lds_busy", round(m["SQ_LDS_IDX_ACTIVE"] / m["SQ_BUSY_CU_CYCLES"], 3))
PY
done
