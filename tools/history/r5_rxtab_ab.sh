#!/bin/bash
# Round 5: A/B of the first-occurrence inserts on one box: build_var/rx_old (CAS + atomicMax into a
# second table) against the tree's library (one CAS), rx-device C3 alternating, then a trace each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_rxtab_ab; mkdir -p $OUT
cd $R
for rep in 1 2 3; do
  for v in old new; do
    if [ $v = old ]; then export NEB_LIB_PATH=$R/build_var/rx_old/libnebula_aead.so; else unset NEB_LIB_PATH; fi
    timeout -k 10 300 python bench.py --mode rx-device --config 2 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c3_${v}_$rep.json 2> $OUT/c3_${v}_$rep.err || exit $?
    echo "$v rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/c3_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
  done
done
cd /tmp && export TMPDIR=/tmp
for v in old new; do
  if [ $v = old ]; then export NEB_LIB_PATH=$R/build_var/rx_old/libnebula_aead.so; else unset NEB_LIB_PATH; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_$v -o run -- \
      python3 $R/bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_$v.log 2>&1 || exit $?
done
unset NEB_LIB_PATH
