#!/bin/bash
# Native drivers of the C ABI (tools/native/queue_bench, built in this container): the submission
# queue at Nebula's flush sizes over 8-64 threads and batch deadlines, and the per-packet
# neb_encrypt_danger / neb_decrypt_danger surface over 1-64 threads. One JSON line each.
# Usage (GPU box): bash tools/bench_native.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/native; mkdir -p $OUT
cd $R/tools/native || exit 1
: > $OUT/native.jsonl
for t in 1 8 16 32 64; do
  timeout -k 5 60 ./queue_bench percall $t 1.5 >> $OUT/native.jsonl 2>> $OUT/native.err || exit $?
done
for d in 50 200; do
  for t in 8 16 32 64; do
    timeout -k 5 60 ./queue_bench queue $t 128 $d 8192 1.5 >> $OUT/native.jsonl 2>> $OUT/native.err || exit $?
  done
done
timeout -k 5 60 ./queue_bench queue 32 64 100 8192 1.5 >> $OUT/native.jsonl 2>> $OUT/native.err || exit $?
# the same flushes from pinned, mapped arenas: submitted zero-copy
for t in 8 16 32 64; do
  timeout -k 5 60 ./queue_bench queuezc $t 128 50 8192 1.5 >> $OUT/native.jsonl 2>> $OUT/native.err || exit $?
done
cat $OUT/native.jsonl
