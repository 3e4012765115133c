#!/bin/bash
# Round 5: relay GMAC (1 key and 4096 keys) and TX on two builds, alternating.
# Usage (GPU box): bash tools/r5_relay_ab.sh A B
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_relayab; mkdir -p $OUT
cd $R
for rep in 1 2; do
  for v in "$@"; do
    for m in "relay --config 1" "relay --config 2" "tx"; do
      tag=$(echo $m | tr -d ' -')
      NEB_LIB_PATH=build_var/$v/libnebula_aead.so timeout -k 10 200 python bench.py --mode $m --steps 20 --warmup 5 --no-cpu-baseline > $OUT/${tag}_${v}_$rep.json 2> $OUT/${tag}_${v}_$rep.err || exit $?
      echo "$tag $v rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/${tag}_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
    done
  done
done
