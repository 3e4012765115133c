#!/bin/bash
# Round 5: does the default warmup leave the GPU below its steady clock? C2 and C5 at warmup 5 and
# 200 (the same 20 timed steps), alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_warm; mkdir -p $OUT
cd $R
for rep in 1 2; do
  for w in 5 200; do
    for c in 1 4; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup $w --no-cpu-baseline > $OUT/c$((c+1))_w${w}_$rep.json 2> $OUT/c$((c+1))_w${w}_$rep.err || exit $?
      echo "C$((c+1)) warmup $w rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/c$((c+1))_w${w}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'])")"
    done
  done
done
