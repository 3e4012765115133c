#!/bin/bash
# Round-4 host-side changes on the GPU: the whole -m gpu suite, the per-packet sweep (fixed pool),
# and the batched key install with a kernel trace. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4; mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
rc=$?; tail -5 $OUT/pytest_gpu.log; [ $rc -gt 1 ] && exit $rc
cd tools/native
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
cat $OUT/queue.jsonl
cd $R
timeout -k 10 120 python tools/key_install_bench.py 4096 --single > $OUT/keys.json 2>&1 || exit $?
cat $OUT/keys.json
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/keys_trace -o run -- python tools/key_install_bench.py 4096 > $OUT/keys_trace.log 2>&1 || exit $?
f=$(find $OUT/keys_trace -name "*kernel_stats.csv" | head -1); cat "$f"
# mixed-key AES-GCM: the split passes (default) against round 3's fused chunk kernel, same box
for v in split fused; do
  [ $v = fused ] && export NEB_MIXED_FUSED=1 || unset NEB_MIXED_FUSED
  for c in 2 4; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench_${v}_c$c.json 2> $OUT/bench_${v}_c$c.err || exit $?
    echo "$v C$((c+1)): $(cut -c1-200 $OUT/bench_${v}_c$c.json)"
  done
done
unset NEB_MIXED_FUSED
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/c3_trace -o run -- python bench.py --config 2 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/c3_trace.log 2>&1 || exit $?
f=$(find $OUT/c3_trace -name "*kernel_stats.csv" | head -1); cut -d, -f1-8 "$f" | head -12
exit $rc
