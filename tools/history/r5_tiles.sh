#!/bin/bash
# Round 5: tile binning (sched.hpp) — the binning parity tests, the GPU suite with every mixed-key
# batch on the tile path, then C5 / C3 with and without it and a kernel trace of each.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_tiles; mkdir -p $OUT
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "binning" \
    > $OUT/binning.log 2>&1 || { tail -30 $OUT/binning.log; exit 1; }
tail -2 $OUT/binning.log
[ "${SUITE:-1}" = 1 ] && { NEB_TILE_BINS_FROM=0 timeout -k 10 900 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests \
    > $OUT/suite_tiles.log 2>&1 || { tail -30 $OUT/suite_tiles.log; exit 1; }
tail -2 $OUT/suite_tiles.log; }
for t in 4000000000 0; do
  for c in 4 2; do
    NEB_TILE_BINS_FROM=$t timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/c$((c+1))_t$t.json 2> $OUT/c$((c+1))_t$t.err || exit $?
    echo "tiles_from=$t C$((c+1)): $(cut -c1-220 $OUT/c$((c+1))_t$t.json)"
  done
done
cd /tmp && export TMPDIR=/tmp
for t in 4000000000 0; do
  NEB_TILE_BINS_FROM=$t timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_c5_t$t -o c5 -- \
      python3 $R/bench.py --config 4 --steps 4 --warmup 2 --no-cpu-baseline > $OUT/trace_c5_t$t.log 2>&1 || exit $?
  grep -E "sched_|gcm_chunk" $OUT/trace_c5_t$t/c5_kernel_stats.csv | cut -d, -f1-4
done
