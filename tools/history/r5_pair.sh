#!/bin/bash
# Round 5: VALU co-issue (SQ_ACTIVE_INST_VALU2) patterns, tools/micro/valu_pair.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_pair
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 $R/tools/micro/valu_pair > $OUT/pair.json 2>&1 || exit $?
timeout -k 10 -s KILL 60 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_WAVES \
    --output-format csv -d $OUT/pmc -o pair -- $R/tools/micro/valu_pair > $OUT/pmc.log 2>&1 || exit $?
cat $OUT/pair.json
