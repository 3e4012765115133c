#!/bin/bash
# Kernel-trace every ablation variant (grid, LDS, scratch, VGPRs and duration per dispatch).
# Usage: tools/ablate_trace.sh [config]
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-1}
OUT=$R/gpurun_out/ablate_trace; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in $(cat $R/build_abl/variants.txt); do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$v -o $v -- python3 $R/tools/ablate_run.py $CFG > $OUT/$v.log 2>&1 || exit 1
  tail -1 $OUT/$v.log
done
