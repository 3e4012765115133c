#!/bin/bash
# Round 5: the bench's settle phase (untimed seal+open until --settle-ms of wall time, before the W
# warmup steps) against none and against 200 warmup steps, C2 and C5, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_settle; mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in "s0:--settle-ms 0" "s300:--settle-ms 300" "s1000:--settle-ms 1000" "w200:--settle-ms 0 --warmup 200"; do
    tag=${v%%:*}; flags=${v#*:}
    for c in 1 4; do
      timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 $flags --no-cpu-baseline > $OUT/c$((c+1))_${tag}_$rep.json 2> $OUT/c$((c+1))_${tag}_$rep.err || exit $?
      echo "C$((c+1)) $tag rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/c$((c+1))_${tag}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d.get('settle'))")"
    done
  done
done
