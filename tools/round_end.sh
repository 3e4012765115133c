#!/bin/bash
# Round-end evidence in one gpurun call: probe, smoke, pytest -m gpu, every config, the §8f paths
# (TX, host and device receive), the 2-rank rehearsal, and rocprofv3 passes (trace + counter passes)
# of C2, C3 and C5. Usage: bash tools/round_end.sh TAG
TAG=${1:-end}
bash tools/gpu_check.sh || exit $?
bash tools/bench_all.sh || exit $?
bash tools/bench_paths.sh || exit $?
bash tools/rehearse_multi.sh || exit $?
bash tools/profile.sh ${TAG}_c3 --config 2 --steps 10 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit $?
bash tools/profile.sh ${TAG}_c5 --config 4 --steps 4 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || exit $?
bash tools/profile.sh ${TAG} > /dev/null 2>&1 || exit $?
echo "profiles done"
