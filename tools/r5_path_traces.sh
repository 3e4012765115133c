#!/bin/bash
# Round 5: rocprofv3 kernel traces (--kernel-trace --stats) of the TX batch and the C3 device
# receive on the final code. Usage (GPU box): bash tools/r5_path_traces.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_traces; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/tx -o tx -- python3 $R/bench.py --mode tx --steps 20 --warmup 5 > $OUT/tx.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/rxd_c3 -o rxd_c3 -- python3 $R/bench.py --mode rx-device --config 2 --steps 20 --warmup 5 > $OUT/rxd_c3.log 2>&1 || exit $?
for d in tx rxd_c3; do find $OUT/$d -name "*kernel_stats.csv" -exec cp {} $OUT/${d}_kernel_stats.csv \; ; done
find $OUT -name "*kernel_trace.csv" -delete
ls $OUT
