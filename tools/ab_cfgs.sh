#!/bin/bash
# Time every variant built by tools/ablate.sh on several configs (ablate_run.py), interleaved
# rounds in separate processes, then one kernel trace per variant and config.
# Usage: tools/ab_cfgs.sh CFG... (ablate_run.py config numbers)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ab_cfgs; mkdir -p $OUT
for cfg in "$@"; do
  for round in 1 2; do
    for v in $(cat $R/build_abl/variants.txt); do
      echo -n "cfg $cfg "
      NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 $R/tools/ablate_run.py $cfg 2>/dev/null | tail -1 || exit 1
    done
  done
done
cd /tmp && export TMPDIR=/tmp
for cfg in "$@"; do
  for v in $(cat $R/build_abl/variants.txt); do
    NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/c${cfg}_$v -o $v -- python3 $R/tools/ablate_run.py $cfg > $OUT/c${cfg}_$v.log 2>&1 || exit 1
  done
done
python3 $R/tools/trace_summary.py $OUT
