#!/bin/bash
# Round 5: ChaCha20-Poly1305 whole-block rounds — parity (every ChaCha GPU test), C4 bench, kernel
# trace of the seal/open launches.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_chfast; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_gpu_parity.py tests/test_gpu_cipher_state.py tests/test_gpu_rx.py tests/test_gpu_tx.py tests/test_gpu_queue.py \
    > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --config 3 --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c4_$k.json 2> $OUT/c4_$k.err || exit $?
  cut -c1-300 $OUT/c4_$k.json
done
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o c4 -- \
    python3 $R/bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
grep chacha_batch $OUT/trace/c4_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU2 SQ_BUSY_CU_CYCLES SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR \
    --output-format csv -d $OUT/pmc -o c4 -- python3 $R/bench.py --config 3 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/pmc.log 2>&1 || exit $?
echo "pmc done"
