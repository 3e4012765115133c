#!/bin/bash
# Round-end evidence in one gpurun call: full GPU test suite + smoke, every config through bench.py,
# the §8f paths, and a rocprof pass set of the mixed-key config. Usage: bash tools/round_check.sh TAG
TAG=${1:-run}
bash tools/gpu_check.sh || exit $?
bash tools/bench_all.sh || exit $?
bash tools/bench_paths.sh || exit $?
bash tools/profile.sh ${TAG}_c3 --config 2 --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit $?
bash tools/profile.sh ${TAG} > /dev/null 2>&1 || exit $?
echo "profiles done"
