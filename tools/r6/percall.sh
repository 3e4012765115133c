#!/bin/bash
# Per-packet calls (tools/native/queue_bench percall) at 1-64 threads, A/B over ENVS
# ("name:VAR=v,VAR=v ..."; default: combiner on / off).
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_percall; mkdir -p $O
cd $R/tools/native || exit 1
ENVS=${ENVS:-"comb1:NEB_PKT_COMBINE=1 comb0:NEB_PKT_COMBINE=0"}
for rep in 1 2; do
  for ev in $ENVS; do
    name=${ev%%:*}; vars=${ev#*:}
    for t in ${THREADS:-1 4 16 64}; do
      env ${vars//,/ } timeout -k 5 60 ./queue_bench percall $t ${SECS:-1.5} > $O/run.json 2>> $O/err.log || exit $?
      python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); d['env']=sys.argv[2]; print(json.dumps(d))" $O/run.json $name | tee -a $O/percall.jsonl
    done
  done
done
