#!/bin/bash
# Sort tile size A/B on C5: prod (4 packets per thread), build_var/items8, build_var/items16 (via
# NEB_LIB_PATH) and the histogram (NEB_SCHED_SORT_FROM=4000000000), alternating; the binning and
# full-size parity tests on prod first; a kernel trace of prod. Stops at the first abnormal exit.
# (Historical: the sorted binning and its NEB_SORT_ITEMS builds were removed after this A/B; the
# script records how profiles/r4b/sort/ab_items.log was made.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_sort2; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "binning or full_size" -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
ab_env() { case $1 in prod) echo "";; hist) echo "NEB_SCHED_SORT_FROM=4000000000";; *) echo "NEB_LIB_PATH=$R/build_var/$1/libnebula_aead.so";; esac; }
for r in 1 2; do
  for v in prod items8 items16 hist; do
    env $(ab_env $v) timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_$r.json 2> $OUT/ab_${v}_$r.err || exit $?
    echo "$v C5 run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_$r.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_prod_c5 -o run -- python bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_prod_c5.log 2>&1 || exit $?
python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_prod_c5/run_kernel_stats.csv | head -14
