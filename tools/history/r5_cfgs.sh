#!/bin/bash
# Round 5: every device config through bench.py (C3-C5 with their CPU baselines skipped), and the
# VALU micro-benchmark.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_cfgs; mkdir -p $OUT
cd $R
for c in 2 3 4; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c$((c+1)).json 2> $OUT/c$((c+1)).err || exit $?
  cut -c1-400 $OUT/c$((c+1)).json
done
cd $R/tools/micro && timeout -k 5 120 ./valu_mix > $OUT/valu_mix.json 2>&1 || exit $?
cat $OUT/valu_mix.json
