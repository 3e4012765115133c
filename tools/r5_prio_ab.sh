#!/bin/bash
# Round 5: age-rank priorities in gcm_single_kernel (NEB_PRIO_SPLIT variants, tools/build_variant.sh
# ps0..ps4; later the chunk-claim variants cc0..cc2) alternating; CFGS (env) the bench configs, default 1.
# Usage (GPU box): [CFGS="2 4"] bash tools/r5_prio_ab.sh [variants]
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/${ABTAG:-r5_prio}; mkdir -p $OUT
cd $R
VARS=${@:-ps0 ps1 ps2 ps3 ps4}
for rep in 1 2; do
  for v in $VARS; do
    for c in ${CFGS:-1}; do
      NEB_LIB_PATH=build_var/$v/libnebula_aead.so timeout -k 10 200 python bench.py --config $c --steps 50 --warmup 5 --no-cpu-baseline > $OUT/c$((c+1))_${v}_$rep.json 2> $OUT/c$((c+1))_${v}_$rep.err || exit $?
      echo "C$((c+1)) $v rep $rep: $(python3 -c "import json;d=json.loads(open('$OUT/c$((c+1))_${v}_$rep.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'],d['roofline']['kernel_ms'],d['roofline'].get('open_kernel_ms'))")"
    done
  done
done
