#!/bin/bash
# Round 5: the TX batch on several builds, alternating. Usage (GPU box): bash tools/r5_tx_ab.sh A B ...
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_txab; mkdir -p $OUT
cd $R
for rep in 1 2 3; do
  for v in "$@"; do
    NEB_LIB_PATH=build_var/$v/libnebula_aead.so timeout -k 10 200 python bench.py --mode tx --steps 20 --warmup 5 > $OUT/${v}_$rep.json 2> $OUT/${v}_$rep.err || exit $?
    echo "tx $v rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/${v}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  done
done
