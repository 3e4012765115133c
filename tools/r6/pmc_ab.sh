#!/bin/bash
# One counter pass (the VALU/LDS issue counters) per variant and config: VARIANTS="name=lib ...",
# CONFIGS="2 4:8". Output under gpurun_out/r6_pmc/<name>_<cfg>/.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-2 4:8}; do
  c=${cfg%%:*}; so=""; nm=c$c; [ "$cfg" != "$c" ] && so="--shard-of ${cfg#*:}" && nm=c${c}s${cfg#*:}
  for v in ${VARIANTS:-new=}; do
    name=${v%%=*}; lib=${v#*=}
    O=$R/gpurun_out/r6_pmc/${name}_$nm
    mkdir -p $O
    NEB_LIB_PATH=$lib timeout -k 10 120 rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_SALU SQ_WAVE_CYCLES --output-format csv -d $O -o lds -- python3 $R/bench.py --config $c $so --steps 6 --warmup 2 --settle-ms 100 --no-cpu-baseline > $O/run.log 2>&1 || exit $?
    echo "$name $nm"; python3 $R/tools/valu_issue.py $(find $O -name 'lds_counter_collection.csv') --kernel "gcm_chunk_kernel<false" | cut -c1-600
  done
done
