#!/bin/bash
# Round 5: one-atomic first-occurrence inserts — the receive tests, rx-device C2-C4, a C3 trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_rxtab; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rx.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2; do
  for c in 1 2 3; do
    timeout -k 10 300 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rx_c$((c+1))_$rep.json 2> $OUT/rx_c$((c+1))_$rep.err || exit $?
    echo "C$((c+1)) rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/rx_c$((c+1))_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d.get('open_only_gibs'))")"
  done
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- \
    python3 $R/bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
grep -E "rx_" $OUT/trace_c3/run_kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-120
