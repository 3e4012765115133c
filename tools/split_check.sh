#!/bin/bash
# The mixed-key split passes on one box: the GPU suite, C3 / C5 benches (split, then the fused
# kernel for comparison), and kernel traces of the split C3 and C5 runs. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/split; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
for v in ${VARIANTS:-fused sdesc split}; do
  unset NEB_MIXED_SPLIT NEB_CTR_RK NEB_GH_UMAX NEB_SCHED_SDESC NEB_GH_OCC NEB_SUB_BINS_FROM NEB_SPLIT_TAILS
  [ $v = sub8 ] && export NEB_SUB_BINS_FROM=0
  [ $v = nosplit ] && export NEB_SPLIT_TAILS=0
  [ $v = split ] && export NEB_MIXED_SPLIT=1
  [ $v = sdesc ] && export NEB_SCHED_SDESC=1
  for c in 2 4; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_c$c.json 2> $OUT/bench_${v}_c$c.err || exit $?
    echo "$v C$((c+1)): $(grep -o '"value": [0-9.]*' $OUT/bench_${v}_c$c.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_${v}_c$c.json)"
  done
done
unset NEB_MIXED_SPLIT NEB_CTR_RK NEB_GH_UMAX NEB_SCHED_SDESC NEB_GH_OCC NEB_SPLIT_TAILS
cd /tmp && export TMPDIR=/tmp && cd $R
for c in 2 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c$c -o run -- python bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/trace_c$c.log 2>&1 || exit $?
  f=$(find $OUT/trace_c$c -name "*kernel_stats.csv" | head -1); cut -d, -f1-4 "$f" | head -9
done
exit $rc
