#!/bin/bash
# Round 5: what one VALU instruction costs on gfx950, in counters. The same cycle-level pass over
#  - tools/micro/valu_mix (one instruction kind per kernel, 8 independent chains),
#  - tools/micro/chacha_layout (ChaCha20 blocks in the quad and the lane layouts),
#  - the C4 (ChaCha20-Poly1305) and C2 (single-key AES-GCM) bench seal kernels,
# so the busy fraction of the engine's kernels is priced by what the microbenchmarks measure.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_valu
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 $R/tools/micro/chacha_layout > $OUT/layout.json 2>&1 || exit $?
timeout -k 10 120 $R/tools/micro/valu_mix > $OUT/valu_mix.json 2>&1 || exit $?
CS="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_THREAD_CYCLES_VALU SQ_BUSY_CU_CYCLES SQ_WAVES SQ_INSTS_SALU GRBM_GUI_ACTIVE"
pass() {  # name program args...
    local name=$1; shift
    timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc $CS --output-format csv -d $OUT/$name -o $name -- "$@" \
        > $OUT/$name.log 2>&1 || exit $?
}
pass micro_mix $R/tools/micro/valu_mix
pass micro_layout $R/tools/micro/chacha_layout
pass c4 python3 $R/bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline
pass c2 python3 $R/bench.py --config 1 --steps 6 --warmup 2 --no-cpu-baseline
# durations of the same kernels without counters
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c4 -o c4 -- \
    python3 $R/bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace_c4.log 2>&1 || exit $?
echo "valu passes done"
