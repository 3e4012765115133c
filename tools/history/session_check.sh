#!/bin/bash
# One GPU call: the full check (probe, smoke, pytest -m gpu, C2 bench), every config, the device
# receive at 1 / 4096 tunnels, and the 2-rank rehearsal. Stops at the first abnormal exit.
bash tools/gpu_check.sh || exit $?
bash tools/bench_all.sh || exit $?
mkdir -p gpurun_out/paths
for c in 1 2; do
  timeout -k 10 300 python bench.py --mode rx-device --steps 10 --warmup 2 --config $c > gpurun_out/paths/rxd_c$c.json 2> gpurun_out/paths/rxd_c$c.err || exit $?
  cut -c1-300 gpurun_out/paths/rxd_c$c.json
done
bash tools/rehearse_multi.sh
