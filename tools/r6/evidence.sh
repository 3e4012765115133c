#!/bin/bash
# Round-6 evidence on the final code, part 1: probe, smoke, the whole GPU suite, the default bench
# line, every config with its CPU baseline, C5's one-GPU shards (by tunnel, by range), the
# host-resident modes. TAG names the output directory (gpurun_out/r6e_$TAG).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh || exit $?
OUT=$R/gpurun_out/r6e_${TAG:-a}; mkdir -p $OUT
cp gpurun_out/pytest_gpu.log gpurun_out/bench.log gpurun_out/smoke.log $OUT/ 2>/dev/null
run() {  # name args...
  local name=$1; shift
  timeout -k 10 400 python bench.py "$@" > $OUT/$name.json 2> $OUT/$name.err || exit $?
  cut -c1-260 $OUT/$name.json
}
for c in 1 2 3 4; do run bench_c$((c+1)) --config $c --steps 20 --warmup 5; done
run bench_c5s8_key --config 4 --shard-of 8 --steps 20 --warmup 5
run bench_c5s8_range --config 4 --shard-of 8 --shard-by range --steps 20 --warmup 5
run bench_host --config 1 --mode host --steps 10 --warmup 3
run bench_host_staged --config 1 --mode host-staged --steps 10 --warmup 3
run bench_host_staged_c3 --config 2 --mode host-staged --steps 10 --warmup 3 --no-cpu-baseline
echo "evidence part 1 done"
