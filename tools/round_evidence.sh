#!/bin/bash
# Round-end evidence, first half (one gpurun call): probe, smoke, pytest -m gpu, bench default,
# every config, the §8f paths, the 2-rank rehearsal, two engines in one process, and the native
# queue / per-packet drivers. The rocprof passes are the second half (tools/profile_configs.sh).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh || exit $?
bash tools/bench_all.sh || exit $?
bash tools/bench_paths.sh || exit $?
rm -rf gpurun_out/paths/prof_tx
bash tools/rehearse_multi.sh || exit $?
timeout -k 10 300 python bench.py --gpus 2 --inproc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/multi/inproc2_c2.json 2> gpurun_out/multi/inproc2_c2.err || exit $?
cat gpurun_out/multi/inproc2_c2.json
bash tools/bench_native.sh || exit $?
echo "evidence done"
