#!/bin/bash
# Round-4 (second session) check on one box: smoke, the whole GPU suite (log kept), then the A/B of
# the mixed-key binning (new = one launch, old = NEB_SCHED_FUSED=0: three launches) on C3 / C5 and on
# the device receive (C2 / C3), kernel traces of both, and the per-packet sweep.
# Stops at the first abnormal exit.
# (Historical: the one-launch binning and NEB_SCHED_FUSED were removed after this A/B; the script
# records how profiles/r4b/binning1-2 were made.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b; mkdir -p $OUT
cd $R
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
ab_env() { case $1 in new) echo "";; old) echo "NEB_SCHED_FUSED=0";; esac; }
for r in 1 2; do
  for v in new old; do
    for c in 2 4; do
      st=20; [ $c = 4 ] && st=10
      env $(ab_env $v) timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_c${c}_$r.json 2> $OUT/ab_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json)"
    done
    for c in 1 2; do
      env $(ab_env $v) timeout -k 10 200 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rxd_${v}_c${c}_$r.json 2> $OUT/rxd_${v}_c${c}_$r.err || exit $?
      echo "$v rx-device C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/rxd_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/rxd_${v}_c${c}_$r.json) $(grep -o '"open_only_gibs": [0-9.]*' $OUT/rxd_${v}_c${c}_$r.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in new old; do
  for c in 2 4; do
    env $(ab_env $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_c$c -o run -- python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_${v}_c$c.log 2>&1 || exit $?
  done
done
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_rx_c3 -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_rx.log 2>&1 || exit $?
for d in $OUT/trace_*/; do echo "== $d"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    print('%-70s %6s %10.1f us' % (r['Name'][:70], r['Calls'], float(r['AverageNs'])/1e3))
" $d/run_kernel_stats.csv | head -14; done
cd $R/tools/native || exit 1
: > $OUT/percall.jsonl
for t in 1 4 16 64; do
  timeout -k 5 60 ./queue_bench percall $t 1.5 >> $OUT/percall.jsonl 2>> $OUT/percall.err || exit $?
done
cat $OUT/percall.jsonl
