#!/bin/bash
# The 64-lane packets' 3-deep final (GhShoup64) against the 7-multiply tree (build_var/tree,
# -DNEB_TAIL_TREE=1): the parity tests that reach the tail and per-packet kernels, the per-packet
# kernel's phase stamps (onetrace / onetrace_tree builds), the per-packet sweep and the TX batch
# (its partial pass runs the tail kernel), alternating. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_f64; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_cipher_state.py tests/test_gpu_tx.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for v in onetrace onetrace_tree; do
  echo "$v"; NEB_LIB_PATH=$R/build_var/$v/libnebula_aead.so timeout -k 10 120 python tools/one_trace.py > $OUT/$v.log 2>&1 || exit $?
  grep -E "one [01]" $OUT/$v.log | tail -4
done
for r in 1 2; do
  for v in prod tree; do
    if [ $v = prod ]; then E=""; else E="NEB_LIB_PATH=$R/build_var/tree/libnebula_aead.so"; fi
    env $E timeout -k 10 300 python bench.py --mode tx --steps 20 --warmup 5 > $OUT/tx_${v}_$r.json 2> $OUT/tx_${v}_$r.err || exit $?
    echo "$v tx run $r: $(grep -o '"value": [0-9.]*' $OUT/tx_${v}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/tx_${v}_$r.json)"
  done
done
cd $R/tools/native || exit 1
for r in 1 2; do
  for v in prod tree; do
    : > $OUT/pc_${v}_$r.jsonl
    for t in 1 4 16; do
      if [ $v = prod ]; then timeout -k 5 60 ./queue_bench percall $t 1.0 >> $OUT/pc_${v}_$r.jsonl 2>> $OUT/pc.err || exit $?
      else LD_LIBRARY_PATH=$R/build_var/tree timeout -k 5 60 ./queue_bench percall $t 1.0 >> $OUT/pc_${v}_$r.jsonl 2>> $OUT/pc.err || exit $?; fi
    done
    echo "$v percall run $r: $(grep -o '"threads": [0-9]*, "calls_per_s": [0-9]*, "gibs": [0-9.]*, "latency_us_p50": [0-9.]*' $OUT/pc_${v}_$r.jsonl | sed 's/"threads": //; s/"calls_per_s": //; s/"gibs": [0-9.]*, "latency_us_p50"://' | tr '\n' ' ')"
  done
done
