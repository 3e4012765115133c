#!/bin/bash
# Scheduler / mixed-key variants on one box: the GPU suite, C3 / C5 benches per variant (VARIANTS),
# and kernel traces of C3 and C5 per variant (TRACE_VARIANTS). Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/split; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
setv() {
  unset NEB_MIXED_SPLIT NEB_CTR_RK NEB_GH_UMAX NEB_SCHED_SDESC NEB_GH_OCC NEB_SUB_BINS_FROM NEB_SPLIT_TAILS NEB_PAIR_TAILS
  [ $1 = sub8 ] && export NEB_SUB_BINS_FROM=0
  [ $1 = pair0 ] && export NEB_PAIR_TAILS=0
  [ $1 = split ] && export NEB_MIXED_SPLIT=1
  [ $1 = sdesc ] && export NEB_SCHED_SDESC=1
  return 0
}
for v in ${VARIANTS:-fused sdesc split}; do
  setv $v
  for c in 2 4; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_c$c.json 2> $OUT/bench_${v}_c$c.err || exit $?
    echo "$v C$((c+1)): $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_c$c.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_c$c.json)"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in ${TRACE_VARIANTS:-fused}; do
  setv $v
  for c in 2 4; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_c$c -o run -- python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_${v}_c$c.log 2>&1 || exit $?
    f=$(find $OUT/trace_${v}_c$c -name "*kernel_stats.csv" | head -1); echo "== $v C$((c+1))"; cut -d, -f1-4 "$f" | head -7
  done
done
exit $rc
