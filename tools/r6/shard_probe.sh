#!/bin/bash
# Round 6: C5's per-GPU shard of an 8-way split (131 072 IMIX packets, 4096 keys) on one GPU:
# bench line, kernel trace, wave timeline (trace build).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r6_shard${TAG:+_$TAG}
mkdir -p $O
[ -n "$TRACE_ONLY" ] || timeout -k 10 300 python bench.py --config 4 --shard-of 8 --no-cpu-baseline > $O/bench.json 2> $O/bench.err || exit $?
cut -c1-400 $O/bench.json
if [ -n "$FULL" ]; then
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > $O/bench_1mi.json 2> $O/bench_1mi.err || exit $?
cut -c1-300 $O/bench_1mi.json
fi
[ -n "$TRACE_ONLY" ] || (cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/trace -o trace -- python3 $R/bench.py --config 4 --shard-of 8 --steps 10 --warmup 2 --no-cpu-baseline > $O/trace.log 2>&1) || exit $?
find $O/trace -name '*kernel_stats.csv' -exec cat {} \; | cut -c1-200 | head -20
if [ -z "$NOTRACE" ]; then
NEB_LIB_PATH=$R/build_var/wtrace/libnebula_aead.so timeout -k 10 300 python tools/wave_trace.py --config 4 --shard-of 8 --out $O/wave.json > $O/wave.log 2>&1 || exit $?
python - <<'PY' $O/wave.json
import json,sys
d=json.load(open(sys.argv[1]))
for k,v in d.items():
    print(k, {x:v[x] for x in ("span_us","chunks","wave_busy_frac","wg_end_us","chunk_us","chunks_per_wave","prologue_us_mean","phase_us_mean","phase_us_total_per_wave") if x in v})
PY
fi
