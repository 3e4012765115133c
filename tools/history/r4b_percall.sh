#!/bin/bash
# Per-packet A/B: the T-table fill of gcm_one_kernel by 1 / 4 (product) / 8 waves
# (build_var/one1, one8 via LD_LIBRARY_PATH; queue_bench's RUNPATH yields to it), queue_bench percall
# at 1-64 threads, alternating, then kernel + HIP traces of the product at 4 threads.
# (build_var/one1 and one8: tools/build_variant.sh one1 -DNEB_ONE_FILL_WAVES=1, one8 ... =8.)
R=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$R/gpurun_out/r4b_pc; mkdir -p $OUT
cd $R/tools/native || exit 1
timeout -k 10 300 python -u -m pytest $R/tests/test_gpu_cipher_state.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/pytest_cs.log 2>&1
rc=$?; tail -2 $OUT/pytest_cs.log; [ $rc -ne 0 ] && exit $rc
for r in 1 2; do
  for v in ${VARIANTS:-prod one1 one8}; do
    : > $OUT/pc_${v}_$r.jsonl
    for t in 1 4 16 64; do
      if [ $v = prod ]; then
        timeout -k 5 60 ./queue_bench percall $t 1.0 >> $OUT/pc_${v}_$r.jsonl 2>> $OUT/pc.err || exit $?
      else
        LD_LIBRARY_PATH=$R/build_var/$v timeout -k 5 60 ./queue_bench percall $t 1.0 >> $OUT/pc_${v}_$r.jsonl 2>> $OUT/pc.err || exit $?
      fi
    done
    echo "$v run $r: $(grep -o '"threads": [0-9]*, "calls_per_s": [0-9]*' $OUT/pc_${v}_$r.jsonl | sed 's/"threads": //; s/"calls_per_s": //' | tr '\n' ' ')"
  done
done
cd /tmp && export TMPDIR=/tmp && cd $R/tools/native
timeout -k 10 120 rocprofv3 --kernel-trace --hip-trace --stats --output-format csv -d $OUT/trace_pc4 -o run -- ./queue_bench percall 4 1.0 > $OUT/trace_pc4.log 2>&1 || exit $?
python3 -c "
import csv,sys
for f in ('kernel','hip_api'):
    for r in list(csv.DictReader(open(sys.argv[1] + '/run_%s_stats.csv' % f)))[:6]:
        print('%-60s %8s %10.1f us' % (r['Name'][:60], r['Calls'], float(r['AverageNs'])/1e3))
" $OUT/trace_pc4
