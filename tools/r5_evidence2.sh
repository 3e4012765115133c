#!/bin/bash
# Round-5 end evidence on the final code, part 2: the §8f paths (TX, receive, relay), the N-rank
# forms on the one GPU (bare and launcher), two engines in one process, the native queue and
# per-packet drivers.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/bench_paths.sh || exit $?
rm -rf gpurun_out/paths/prof_tx
mkdir -p gpurun_out/multi
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/multi/bare_g2_c2.json 2> gpurun_out/multi/bare_g2_c2.err || exit $?
cut -c1-200 gpurun_out/multi/bare_g2_c2.json
bash tools/rehearse_multi.sh || exit $?
timeout -k 10 300 python bench.py --gpus 2 --inproc --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/multi/inproc2_c2.json 2> gpurun_out/multi/inproc2_c2.err || exit $?
cut -c1-200 gpurun_out/multi/inproc2_c2.json
bash tools/bench_native.sh || exit $?
echo "evidence part 2 done"
