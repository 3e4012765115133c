# Kernel traces of the mixed-key configs (C3 = --config 2, C5 IMIX = --config 4), after the GPU tests.
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $R/gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -2 $R/gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
cd /tmp && export TMPDIR=/tmp
for c in 2 4; do
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_c$c -o c$c -- python3 $R/bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline > $R/gpurun_out/prof_c$c.log 2>&1 || exit $?
grep '^{' $R/gpurun_out/prof_c$c.log | cut -c1-120
done
