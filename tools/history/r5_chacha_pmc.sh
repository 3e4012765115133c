#!/bin/bash
# Round 5: what bounds the ChaCha20-Poly1305 kernel (C4). The counter list, then counter passes of
# the seal over the C4 bench: VALU instruction mix by type and the cycle-level busy counters that
# this rocprofv3 offers (one pass per block budget; each pass its own run, no trace domains).
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_chacha
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
have() { grep -q "\b$1\b" $OUT/counters_available.txt; }
pass() {  # name counters...
    local name=$1; shift
    local cs=""
    for c in "$@"; do have $c && cs="$cs $c"; done
    [ -z "$cs" ] && { echo "$name: none available"; return 0; }
    echo "$name:$cs"
    timeout -k 10 120 rocprofv3 --kernel-trace --pmc $cs --output-format csv -d $OUT/$name -o $name -- \
        python3 $R/bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/$name.log 2>&1 || exit $?
}
pass mix1 SQ_INSTS_VALU SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS
pass cyc1 SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VALU SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES
pass cyc2 SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC SQ_INSTS_SMEM SQ_WAIT_ANY SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM SQ_BUSY_CU_CYCLES
pass valu2 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_MFMA_I8 SQ_INSTS_MFMA SQ_INSTS_VALU_F16 GRBM_GUI_ACTIVE
echo "chacha passes done"
