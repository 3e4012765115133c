#!/bin/bash
# Round-4 evidence on one box: the per-packet sweep (fixed FIFO pool), the submission queue with its
# phase timers, and every BASELINE config through bench.py with its CPU baseline. Stops at the first
# abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4e; mkdir -p $OUT
cd $R/tools/native || exit 1
: > $OUT/percall.jsonl
for t in 1 4 8 16 32 64; do
  timeout -k 5 60 ./queue_bench percall $t 1.5 >> $OUT/percall.jsonl 2>> $OUT/percall.err || exit $?
done
cat $OUT/percall.jsonl
: > $OUT/queue.jsonl
for m in queue queuezc; do
  for t in 16 32 64; do
    timeout -k 5 60 ./queue_bench $m $t 128 50 8192 1.5 >> $OUT/queue.jsonl 2>> $OUT/queue.err || exit $?
  done
done
grep -v phases $OUT/queue.jsonl | cut -c1-220
cd $R
for c in ${CONFIGS:-0 1 2 3 4}; do
  st=20; [ $c = 4 ] && st=10
  timeout -k 10 400 python bench.py --config $c --steps $st --warmup 5 > $OUT/bench_c$c.json 2> $OUT/bench_c$c.err || exit $?
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); cb=d.get('cpu_baseline') or {}; print('C%d' % (int(sys.argv[2])+1), d['value'], d['ms_per_step'], 'cpu', cb.get('value'), cb.get('cores'), cb.get('value_1thread'))" $OUT/bench_c$c.json $c
done
