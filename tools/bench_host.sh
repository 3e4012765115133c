#!/bin/bash
# Host-resident A/B (GPU box): every host mode of neb_*_batch_host on C2 and C3, two rounds.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/host; mkdir -p $OUT
cd $R
for round in 1 2; do for cfg in ${CFGS:-1 2}; do for m in ${MODES:-host host-split host-staged}; do
  timeout -k 10 300 python bench.py --mode $m --config $cfg --steps 10 --warmup 3 > $OUT/$m.$cfg.$round.json 2> $OUT/$m.$cfg.$round.err || exit 1
  echo "$m cfg$cfg: $(python3 -c "import json,sys; d=json.load(open('$OUT/$m.$cfg.$round.json')); print(d['value'], d['ms_per_step'])")"
done; done; done
