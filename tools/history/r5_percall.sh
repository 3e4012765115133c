#!/bin/bash
# Round 5: the per-packet path (neb_encrypt_danger / neb_decrypt_danger) with the status poll, 1-64
# threads, and a 128-packet host-resident flush; plus the VALU issue-rate microbenchmark.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_percall; mkdir -p $OUT
cd $R/tools/native || exit 1
: > $OUT/percall.jsonl
for t in 1 4 16 64; do
  timeout -k 5 60 ./queue_bench percall $t 1.5 >> $OUT/percall.jsonl 2>> $OUT/percall.err || exit $?
done
cat $OUT/percall.jsonl
cd $R/tools/micro && timeout -k 5 60 ./valu_mix > $OUT/valu_mix.json 2>&1 || exit $?
cat $OUT/valu_mix.json
