#!/bin/bash
# rocprofv3 passes over the bench (run on the GPU box): kernel trace + stats, then counter passes
# (each in its own run, no trace domains combined with --pmc). Usage: tools/profile.sh TAG [bench args]
# PASSES (env): the passes to run, default all of them.
R=${GRAFT_REPO_ROOT:-$(pwd)}
TAG=${1:-run}; shift
ARGS=${@:---steps 10 --warmup 2 --no-cpu-baseline}
OUT=$R/gpurun_out/prof_$TAG
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
PASSES=${PASSES:-trace fetch write req wreq sq sq2 lds}
run() {  # name timeout args...
    local name=$1 t=$2; shift 2
    case " $PASSES " in *" $name "*) ;; *) return 0 ;; esac
    timeout -k 10 $t rocprofv3 "$@" --output-format csv -d $OUT/$name -o $name -- python3 $R/bench.py $ARGS > $OUT/$name.log 2>&1
    local rc=$?
    echo "$name rc=$rc"; tail -n 3 $OUT/$name.log
    if [ $rc -ne 0 ]; then exit $rc; fi
}
rocprofv3 -L > $OUT/counters_available.txt 2>&1 || true
run trace 300 --kernel-trace --stats
run fetch 300 --kernel-trace --pmc FETCH_SIZE
run write 300 --kernel-trace --pmc WRITE_SIZE
# the memory-side requests by size: FETCH_SIZE tallies a 128-B request at 64 B on gfx950, so the
# read bytes are taken as 32*RDREQ_32B + 64*RDREQ_64B + 128*RDREQ_128B (tools/pmc_config.py)
run req 300 --kernel-trace --pmc TCC_EA0_RDREQ TCC_EA0_RDREQ_32B TCC_EA0_RDREQ_64B TCC_EA0_RDREQ_128B
run wreq 300 --kernel-trace --pmc TCC_EA0_WRREQ TCC_EA0_WRREQ_64B TCC_EA0_RDREQ_DRAM TCC_EA0_WRREQ_DRAM
run sq 300 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE
run sq2 300 --kernel-trace --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
run lds 300 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INSTS_LDS SQ_BUSY_CU_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2
