#!/bin/bash
# One rocprofv3 counter pass per ablation variant and config: tools/pmc_variants.sh "CFG..." "COUNTERS"
R=${GRAFT_REPO_ROOT:-$(pwd)}
CFGS=${1:-1}; PMC=${2:-SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_WAVES SQ_INSTS_SMEM}
OUT=$R/gpurun_out/pmc_var; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for c in $CFGS; do
  for v in $(cat $R/build_abl/variants.txt); do
    NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $PMC --output-format csv -d $OUT/${v}_$c -o ${v}_$c -- python3 $R/tools/ablate_run.py $c > $OUT/${v}_$c.log 2>&1 || exit 1
    python3 $R/tools/pmc_var_summary.py $OUT/${v}_$c >> $OUT/summary.txt && rm -rf $OUT/${v}_$c
  done
done
cat $OUT/summary.txt
