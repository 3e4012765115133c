#!/bin/bash
# TX batch A/B over the variants built by tools/ablate.sh: bench.py --mode tx per variant
# (interleaved rounds), then one kernel trace per variant. Usage: bash tools/ab_tx.sh
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_tx; mkdir -p $OUT
for round in 1 2; do
  for v in $(cat $R/build_abl/variants.txt); do
    echo -n "tx $v "
    NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 $R/bench.py --mode tx --steps 20 --warmup 5 2>/dev/null | \
      python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in $(cat $R/build_abl/variants.txt); do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o $v -- python3 $R/bench.py --mode tx --steps 10 --warmup 2 > $OUT/$v.log 2>&1 || exit 1
  echo "== $v"; grep -h "gcm_single\|tx_" $OUT/$v/*kernel_stats.csv | cut -d, -f1,2,4 | cut -c1-120
  rm -f $OUT/$v/*kernel_trace.csv
done
