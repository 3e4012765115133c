#!/bin/bash
# Receive-window A/B on one box: the receive parity tests, then bench.py --mode rx-device on CONFIGS
# for this build and for NEB_LIB_PATH=$BASE (a baseline build), alternating, then a kernel trace.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/rxab; mkdir -p $OUT
cd $R
timeout -k 10 400 python -u -m pytest tests/test_gpu_rx.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/pytest_rx.log 2>&1
rc=$?; tail -3 $OUT/pytest_rx.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in new base; do
    for c in ${CONFIGS:-1 2 3}; do
      if [ $v = base ]; then export NEB_LIB_PATH=$R/${BASE:-build_var/base/libnebula_aead.so}; else unset NEB_LIB_PATH; fi
      timeout -k 10 200 python bench.py --mode rx-device --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/rx_${v}_c${c}_$r.json 2> $OUT/rx_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/rx_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/rx_${v}_c${c}_$r.json)"
    done
  done
done
unset NEB_LIB_PATH
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c3 -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1
