#!/bin/bash
# One box: the GPU suite, then bench.py on CONFIGS (default C2-C5) REPS times each, one line per run.
# Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/abq; mkdir -p $OUT
cd $R
if [ -z "$NO_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
fi
for r in $(seq ${REPS:-2}); do
  for c in ${CONFIGS:-1 2 3 4}; do
    timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline $BENCH_ARGS > $OUT/bench_c${c}_$r.json 2> $OUT/bench_c${c}_$r.err || exit $?
    echo "C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/bench_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/bench_c${c}_$r.json)"
  done
done
