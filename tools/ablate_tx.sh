#!/bin/bash
# Time the device TX batch with every variant built by tools/ablate.sh (interleaved rounds).
R=${GRAFT_REPO_ROOT:-$(pwd)}
for round in 1 2; do
  for v in $(cat $R/build_abl/variants.txt); do
    echo -n "$v "
    NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 200 python3 $R/bench.py --mode tx --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
