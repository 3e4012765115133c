#!/bin/bash
# Alternating A/B of library variants on one box: VARIANTS="name=path ..." (path "" = the in-tree
# library), CONFIGS="4:8 4 2" (config[:shard-of]), REPS rounds. One JSON line per run into $OUT.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
OUT=${OUT:-$R/gpurun_out/r6_ab.jsonl}
mkdir -p $(dirname $OUT)
for rep in $(seq 1 ${REPS:-2}); do
  for cfg in ${CONFIGS:-4:8}; do
    c=${cfg%%:*}; so=""; [ "$cfg" != "$c" ] && so="--shard-of ${cfg#*:}"
    for v in ${VARIANTS:-new=}; do
      name=${v%%=*}; lib=${v#*=}
      line=$(NEB_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $c $so --no-cpu-baseline ${BENCH_ARGS} 2>>$OUT.err) || { echo "FAIL $name $cfg"; exit 1; }
      python3 -c "
import json,sys; d=json.loads(sys.argv[1]); r=d.get('roofline',{})
o={'variant':sys.argv[2],'cfg':sys.argv[3],'rep':int(sys.argv[4]),'value':d['value'],'ms':d['ms_per_step'],'seal_k':r.get('kernel_ms'),'open_k':r.get('open_kernel_ms'),'call':r.get('seal_call_ms')}
print(json.dumps(o)); open(sys.argv[5],'a').write(json.dumps(o)+'\n')" "$line" $name $cfg $rep $OUT
    done
  done
done
