#!/bin/bash
# s_setprio level during the T-table lookups (NEB_PRIO; product 3) on the mixed-key configs, with C2
# as the control: build_var/prio0, prio1 via NEB_LIB_PATH, alternating.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_prio; mkdir -p $OUT
cd $R
ab_env() { case $1 in prod) echo "";; *) echo "NEB_LIB_PATH=$R/build_var/$1/libnebula_aead.so";; esac; }
for r in 1 2; do
  for v in prod prio0 prio1; do
    for c in 2 4 1; do
      st=20; [ $c = 4 ] && st=10
      env $(ab_env $v) timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_c${c}_$r.json 2> $OUT/ab_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json) $(grep -o '"kernel_ms": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json)"
    done
  done
done
