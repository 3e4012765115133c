#!/bin/bash
# End-of-round check of the final code on one box: probe, smoke, the GPU suite and the C2 bench
# (tools/gpu_check.sh), the §8f paths (TX, host and device receive, relay; TX kernel trace), the
# host-resident modes, and the 2-rank rehearsal. Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
bash tools/gpu_check.sh || exit $?
bash tools/bench_paths.sh || exit $?
for m in host host-staged; do
  timeout -k 10 300 python bench.py --config 1 --mode $m --steps 10 --warmup 3 > gpurun_out/paths/$m.json 2> gpurun_out/paths/$m.err || exit $?
  cut -c1-300 gpurun_out/paths/$m.json
done
bash tools/rehearse_multi.sh || exit $?
