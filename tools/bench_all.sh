#!/bin/bash
# Every BASELINE config through bench.py (device-resident) plus the host-resident rate.
mkdir -p gpurun_out
for c in 1 2 3; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/bench_c$c.json 2> gpurun_out/bench_c$c.err
  rc=$?; echo "config $c rc=$rc"; cat gpurun_out/bench_c$c.json | cut -c1-300; [ $rc -ne 0 ] && tail -5 gpurun_out/bench_c$c.err && exit $rc
done
timeout -k 10 300 python bench.py --config 4 --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err
rc=$?; echo "config 4 rc=$rc"; cut -c1-300 gpurun_out/bench_c4.json; [ $rc -ne 0 ] && tail -5 gpurun_out/bench_c4.err && exit $rc
timeout -k 10 300 python bench.py --config 1 --mode host-staged --steps 10 --warmup 3 > gpurun_out/bench_host_staged.json 2> gpurun_out/bench_host_staged.err || exit $?
cut -c1-300 gpurun_out/bench_host_staged.json
timeout -k 10 300 python bench.py --config 1 --mode host --steps 10 --warmup 3 > gpurun_out/bench_host.json 2> gpurun_out/bench_host.err
rc=$?; echo "host rc=$rc"; cut -c1-300 gpurun_out/bench_host.json; exit $rc
