#!/bin/bash
# ChaCha kernel occupancy A/B on C4: the product (compiler's choice, 4 waves/SIMD) against
# build_var/chwpe5 / chwpe6 (-DNEB_CH_WPE=5 / 6: 96 / 80 VGPRs, with spills), alternating.
# (Historical: the NEB_CH_WPE knob was removed after this A/B; build_var/chwpe5, chwpe6 came from a
# __launch_bounds__(kChThreads, NEB_CH_WPE) variant of chacha_batch_kernel.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_ch; mkdir -p $OUT
cd $R
ab_env() { case $1 in prod) echo "";; *) echo "NEB_LIB_PATH=$R/build_var/$1/libnebula_aead.so";; esac; }
for r in 1 2; do
  for v in prod chwpe5 chwpe6; do
    env $(ab_env $v) timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_$r.json 2> $OUT/ab_${v}_$r.err || exit $?
    echo "$v C4 run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_$r.json) $(grep -o '"kernel_ms": [0-9.]*' $OUT/ab_${v}_$r.json)"
  done
done
