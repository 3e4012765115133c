#!/bin/bash
# Alternating A/B of environment settings on one box: ENVS="name:VAR=v,VAR2=w name2:" (empty: none),
# RUNS="4:8:key 4:8:range 2 4" (config[:shard-of[:shard-by]]), REPS rounds; one JSON line per run.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=${OUT:-$R/gpurun_out/r6_abenv.jsonl}
mkdir -p $(dirname $OUT)
for rep in $(seq 1 ${REPS:-2}); do
  for run in ${RUNS:-4:8:key}; do
    IFS=: read c so sb <<< "$run"
    args="--config $c"; [ -n "$so" ] && args="$args --shard-of $so"; [ -n "$sb" ] && args="$args --shard-by $sb"
    for e in ${ENVS:-base:}; do
      name=${e%%:*}; kv=${e#*:}
      line=$(env ${kv//,/ } timeout -k 10 300 python bench.py $args --no-cpu-baseline ${BENCH_ARGS} 2>>$OUT.err) || { echo "FAIL $name $run"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(sys.argv[1]); r=d.get('roofline',{})
o={'env':sys.argv[2],'run':sys.argv[3],'rep':int(sys.argv[4]),'value':d['value'],'ms':d['ms_per_step'],'seal_k':r.get('kernel_ms'),'open_k':r.get('open_kernel_ms'),'call':r.get('seal_call_ms'),'n':d['config'].get('packets_per_gpu')}
print(json.dumps(o)); open(sys.argv[5],'a').write(json.dumps(o)+'\n')" "$line" $name $run $rep $OUT
    done
  done
done
