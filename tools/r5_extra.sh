#!/bin/bash
# Round 5 extra evidence: bare bench.py --gpus 4 (four ranks sharing the one GPU: the spawner and
# aggregation at N=4, not scaling), and kernel traces of the TX batch and the relay path.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r5_extra; mkdir -p $OUT
cd $R
timeout -k 10 400 python bench.py --gpus 4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bare_g4_c2.json 2> $OUT/bare_g4_c2.err || exit $?
cut -c1-220 $OUT/bare_g4_c2.json
timeout -k 10 400 python bench.py --gpus 4 --config 4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bare_g4_c5.json 2> $OUT/bare_g4_c5.err || exit $?
cut -c1-220 $OUT/bare_g4_c5.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_tx -o tx -- \
    python3 $R/bench.py --mode tx --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace_tx.log 2>&1 || exit $?
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_relay -o relay -- \
    python3 $R/bench.py --mode relay --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace_relay.log 2>&1 || exit $?
echo "extra done"
