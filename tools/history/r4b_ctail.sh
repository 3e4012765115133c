#!/bin/bash
# Tail chunks' own-power final (GhChunkOwn) against the pairwise tree (build_var/ctree,
# -DNEB_CHUNK_TREE=1): the parity tests, then C3 / C5 alternating, then kernel traces of both on C3.
# Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_ct; mkdir -p $OUT
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_rx.py tests/test_gpu_queue.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $OUT/pytest.log 2>&1
rc=$?; tail -2 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
ab_env() { case $1 in prod) echo "";; *) echo "NEB_LIB_PATH=$R/build_var/$1/libnebula_aead.so";; esac; }
for r in 1 2 3; do
  for v in prod ctree; do
    for c in 2 4; do
      st=20; [ $c = 4 ] && st=10
      env $(ab_env $v) timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > $OUT/ab_${v}_c${c}_$r.json 2> $OUT/ab_${v}_c${c}_$r.err || exit $?
      echo "$v C$((c+1)) run $r: $(grep -o '"value": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json) $(grep -o '"ms_per_step": [0-9.]*' $OUT/ab_${v}_c${c}_$r.json)"
    done
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R
for v in prod ctree; do
  env $(ab_env $v) timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace_${v}_c3 -o run -- python bench.py --config 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/trace_${v}.log 2>&1 || exit $?
  echo "== $v"; python3 -c "
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'chunk' in r['Name']: print('%-60s %6s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_${v}_c3/run_kernel_stats.csv
done
