#!/bin/bash
# Round 5: device receive with windows (C2 / C3 / C4) and a kernel trace of the C3 receive.
mkdir -p gpurun_out/r5_rx
cd ${GRAFT_REPO_ROOT:-.}
for c in 1 2 3; do
  timeout -k 10 300 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline \
      > gpurun_out/r5_rx/rxd_c$c.json 2> gpurun_out/r5_rx/rxd_c$c.err || exit $?
  cat gpurun_out/r5_rx/rxd_c$c.json
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r5_rx/trace_c3 -o run -- \
    python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/r5_rx/trace.log 2>&1 || exit $?
find gpurun_out/r5_rx/trace_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} gpurun_out/r5_rx/c3_kernel_stats.csv
python - <<'PY'
import csv
for r in csv.DictReader(open("gpurun_out/r5_rx/c3_kernel_stats.csv")):
    print(f"{r['Name'][:70]:70s} {r['Calls']:>5s} {float(r['AverageNs'])/1e3:8.1f}us")
PY
