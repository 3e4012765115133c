#!/bin/bash
# A/B on one box: for each variant (the product build "base" or build_abl/<name>), run the bench
# arguments and a rocprof kernel trace of the first argument set. Stops at the first abnormal exit.
#   tools/ab.sh "<variant> <variant> ..." "<bench args;bench args;...>"
mkdir -p gpurun_out/ab
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
IFS=';' read -ra BENCHES <<< "$2"
for v in $1; do
    if [ "$v" = base ]; then unset NEB_LIB_PATH; else export NEB_LIB_PATH=$PWD/build_abl/$v/libnebula_aead.so; fi
    i=0
    for b in "${BENCHES[@]}"; do
        i=$((i+1))
        timeout -k 10 300 python bench.py --no-cpu-baseline $b > gpurun_out/ab/${v}_$i.log 2>&1
        rc=$?
        echo "$v bench $i rc=$rc: $(grep -o '"value": [0-9.]*' gpurun_out/ab/${v}_$i.log) $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab/${v}_$i.log)"
        [ $rc -ne 0 ] && { tail -5 gpurun_out/ab/${v}_$i.log; exit $rc; }
    done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ab/trace_$v -o run -- python bench.py --no-cpu-baseline ${BENCHES[0]} --steps 10 > gpurun_out/ab/trace_$v.log 2>&1 || { echo "trace $v failed"; exit 1; }
    f=$(find gpurun_out/ab/trace_$v -name "*kernel_stats.csv" | head -1)
    python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows[:8]:
    print(f"   {r['Name'][:60]:60s} calls {r['Calls']:>5s} avg {float(r['AverageNs'])/1e3:9.1f} us  tot% {float(r['Percentage']):5.1f}")
PY
done
