R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/gpu_tests.log 2>&1 || exit $?
tail -1 gpurun_out/gpu_tests.log
for c in 2 4; do timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | cut -c1-200 || exit $?; done
OUT=$R/gpurun_out/prof_ej0; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o trace -- python3 $R/bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o fetch -- python3 $R/bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/fetch.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE --output-format csv -d $OUT/write -o write -- python3 $R/bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/write.log 2>&1 || exit $?
echo done
