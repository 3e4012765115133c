#!/bin/bash
# The §8f paths beside the headline: device TX batch, batched receive (1 and 4096 tunnels; host
# windows over a pinned arena, and windows in HBM over a device batch), and a
# kernel-trace profile of the TX batch. Usage (GPU box): bash tools/bench_paths.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/paths; mkdir -p $OUT
cd $R
timeout -k 10 300 python bench.py --mode tx --steps 20 --warmup 5 > $OUT/tx.json 2> $OUT/tx.err || exit 1
cat $OUT/tx.json
timeout -k 10 300 python bench.py --mode rx --steps 5 --warmup 2 --config 1 > $OUT/rx_c2.json 2> $OUT/rx_c2.err || exit 1
cat $OUT/rx_c2.json
timeout -k 10 300 python bench.py --mode rx --steps 5 --warmup 2 --config 2 > $OUT/rx_c3.json 2> $OUT/rx_c3.err || exit 1
cat $OUT/rx_c3.json
for c in 1 2 3; do
  timeout -k 10 300 python bench.py --mode rx-device --steps 10 --warmup 2 --config $c > $OUT/rxd_c$c.json 2> $OUT/rxd_c$c.err || exit 1
  cat $OUT/rxd_c$c.json
done
for c in 1 2; do
  timeout -k 10 300 python bench.py --mode relay --steps 20 --warmup 5 --config $c > $OUT/relay_c$c.json 2> $OUT/relay_c$c.err || exit 1
  cat $OUT/relay_c$c.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_tx -o tx -- python3 $R/bench.py --mode tx --steps 10 --warmup 2 > $OUT/prof_tx.log 2>&1 || exit 1
find $OUT/prof_tx -name "*kernel_stats.csv" -exec cat {} \;
