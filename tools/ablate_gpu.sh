#!/bin/bash
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/ablate; mkdir -p $OUT
for v in BASE HORNER FINAL AES; do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 $R/tools/ablate_run.py 2>/dev/null | tail -1 || exit 1
done
cd /tmp && export TMPDIR=/tmp
for v in BASE HORNER FINAL AES; do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 180 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d $OUT/$v -o $v -- python3 $R/tools/ablate_run.py > $OUT/$v.log 2>&1 || exit 1
done
