#!/bin/bash
# The GPU suite (log kept), the device receive on C2 / C3 twice, and a kernel trace of the C3
# receive. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_rx; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for c in 1 2; do
    timeout -k 10 200 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rxd_c${c}_$r.json 2> $OUT/rxd_c${c}_$r.err || exit $?
    echo "rx-device C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/rxd_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/rxd_c${c}_$r.json) $(grep -o '"open_only_gibs": [0-9.]*' $OUT/rxd_c${c}_$r.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_rx_c3 -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_rx.log 2>&1 || exit $?
python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_rx_c3/run_kernel_stats.csv | head -16
