#!/bin/bash
# Time every variant built by tools/ablate.sh (interleaved rounds in separate processes), then
# collect LDS/VALU counters per variant. Usage: tools/ablate_gpu.sh [config]
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFG=${1:-1}
OUT=$R/gpurun_out/ablate; mkdir -p $OUT
for round in 1 2; do
  for v in $(cat $R/build_abl/variants.txt); do
    NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 $R/tools/ablate_run.py $CFG 2>/dev/null | tail -1 || exit 1
  done
done
cd /tmp && export TMPDIR=/tmp
for v in $(cat $R/build_abl/variants.txt); do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_LDS_IDX_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CU_CYCLES --output-format csv -d $OUT/$v -o $v -- python3 $R/tools/ablate_run.py $CFG > $OUT/$v.log 2>&1 || exit 1
done
