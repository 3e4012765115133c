#!/bin/bash
# One GPU iteration: targeted tests -> benches -> kernel trace. Stops at the first step that dies
# abnormally (exit > 1); test failures (exit 1) still let later steps run.
#   tools/iter.sh "<pytest -k expr>" "<bench args;bench args;...>" [trace bench args]
mkdir -p gpurun_out/iter
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/iter/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 6 "gpurun_out/iter/$name.log"
    if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
if [ -n "$1" ]; then
    step tests 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "$1"
fi
i=0
IFS=';' read -ra BENCHES <<< "$2"
for b in "${BENCHES[@]}"; do
    [ -z "$b" ] && continue
    i=$((i+1))
    step bench_$i 300 python bench.py --no-cpu-baseline $b
done
if [ -n "$3" ]; then
    step trace 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/iter/trace -o run -- python bench.py --no-cpu-baseline $3
    find gpurun_out/iter/trace -name "*kernel_stats.csv" -exec cp {} gpurun_out/iter/kernel_stats.csv \;
    head -12 gpurun_out/iter/kernel_stats.csv | cut -c1-200
fi
