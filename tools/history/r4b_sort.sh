#!/bin/bash
# The sorted binning of large mixed-key batches: the GPU suite (log kept), then C5 (and C3 as a
# control) with the sort (default) against the histogram (NEB_SCHED_SORT_FROM=4000000000),
# alternating, and kernel traces of both on C5. Stops at the first abnormal exit.
# (Historical: the sorted binning and NEB_SCHED_SORT_FROM were removed after this A/B; the script
# records how profiles/r4b/sort was made.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_sort; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
ab_env() { case $1 in sort) echo "";; hist) echo "NEB_SCHED_SORT_FROM=4000000000";; esac; }
for r in 1 2; do
  for v in sort hist; do
    for c in 4 2; do
      st=20; [ $c = 4 ] && st=10
      env $(ab_env $v) timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_c${c}_$r.json 2> $OUT/ab_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in sort hist; do
  env $(ab_env $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_c5 -o run -- python bench.py --config 4 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_${v}_c5.log 2>&1 || exit $?
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_${v}_c5/run_kernel_stats.csv | head -14
done
