#!/bin/bash
# The sort passes' digit-count reads all at once (build_var/histall, -DNEB_RX_HIST_ALL=1) against
# the product's eight at a time: the receive tests on the variant, rx-device C3 / C2 alternating,
# and a kernel trace of each. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4c_rxhist; mkdir -p $OUT
cd $R
V="NEB_LIB_PATH=$R/build_var/histall/libnebula_aead.so"
env $V timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_rx_histall.log 2>&1
rc=$?; tail -2 $OUT/pytest_rx_histall.log; [ $rc -ne 0 ] && exit $rc
ab_env() { case $1 in prod) echo "";; *) echo "$V";; esac; }
for r in 1 2 3; do
  for v in prod histall; do
    for c in 2 1; do
      env $(ab_env $v) timeout -k 10 200 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${v}_c${c}_$r.json 2> $OUT/${v}_c${c}_$r.err || exit $?
      echo "$v rx-device C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/${v}_c${c}_$r.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in prod histall; do
  env $(ab_env $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_$v.log 2>&1 || exit $?
  echo "== $v"
  python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'rx_' in r['Name']: print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_$v/run_kernel_stats.csv
done
