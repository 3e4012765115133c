#!/bin/bash
# Per-packet calls (tools/native/queue_bench percall) at 1-64 threads, combiner on and off.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_percall; mkdir -p $O
cd $R/tools/native || exit 1
for rep in 1 2; do
  for comb in 1 0; do
    for t in ${THREADS:-1 4 16 64}; do
      NEB_PKT_COMBINE=$comb timeout -k 5 60 ./queue_bench percall $t 1.5 > $O/run.json 2>> $O/err.log || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['combine']=int(sys.argv[2]); print(json.dumps(d))" $O/run.json $comb | tee -a $O/percall.jsonl
    done
  done
done
