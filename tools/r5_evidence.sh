#!/bin/bash
# Round-5 end evidence on the final code, part 1: probe, smoke, the whole GPU suite, the default
# bench line, every config with its CPU baseline, the host-resident modes.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh || exit $?
OUT=$R/gpurun_out/r5e; mkdir -p $OUT
for c in 1 2 3 4; do
  timeout -k 10 400 python bench.py --config $c --steps 20 --warmup 5 > $OUT/bench_c$((c+1)).json 2> $OUT/bench_c$((c+1)).err || exit $?
  cut -c1-240 $OUT/bench_c$((c+1)).json
done
timeout -k 10 300 python bench.py --config 1 --mode host --steps 10 --warmup 3 > $OUT/bench_host.json 2> $OUT/bench_host.err || exit $?
timeout -k 10 300 python bench.py --config 1 --mode host-staged --steps 10 --warmup 3 > $OUT/bench_host_staged.json 2> $OUT/bench_host_staged.err || exit $?
cut -c1-200 $OUT/bench_host.json $OUT/bench_host_staged.json
echo "evidence part 1 done"
