#!/bin/bash
# Round-4 (second session) check on one box: smoke, the whole GPU suite (log kept), the device
# receive on C2 / C3 (the merged scan + admission launch) with its kernel trace, the one-launch
# binning against three launches (NEB_SCHED_FUSED=0) on C3 / C5 with kernel traces of both, and the
# stream-id probe. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b; mkdir -p $OUT
cd $R
timeout -k 10 60 python tools/streamid_probe.py > $OUT/streamid.json 2>&1 || { cat $OUT/streamid.json; exit 3; }
cat $OUT/streamid.json
timeout -k 10 300 python __graft_entry__.py smoke > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
for c in 1 2; do
  timeout -k 10 200 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rxd_c$c.json 2> $OUT/rxd_c$c.err || exit $?
  cut -c1-400 $OUT/rxd_c$c.json
done
# binning variants: new = one launch (C3) / radix sort (C5); fz = one launch, no sort; old = three launches
ab_env() { case $1 in new) echo "";; fz) echo "NEB_SCHED_SORT_FROM=4000000000";; old) echo "NEB_SCHED_FUSED=0 NEB_SCHED_SORT_FROM=4000000000";; esac; }
for r in 1 2; do
  for v in new fz old; do
    for c in 2 4; do
      [ $v = fz ] && [ $c = 2 ] && continue
      st=20; [ $c = 4 ] && st=10
      env $(ab_env $v) timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_c${c}_$r.json 2> $OUT/ab_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_rx_c3 -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
for v in new old; do
  for c in 2 4; do
    env $(ab_env $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_c$c -o run -- python bench.py --config $c --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_${v}_c$c.log 2>&1 || exit $?
  done
done
for d in $OUT/trace_*; do echo "== $d"; find $d -name '*kernel_stats.csv' | head -1 | xargs cut -c1-140 | head -12; done
