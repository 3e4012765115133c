#!/bin/bash
# Host-staged pipeline (--mode host-staged): alternating A/B against VARIANTS, then a memory-copy +
# kernel trace of the in-tree library (the copies' intervals, tools/r6/copy_overlap.py).
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
O=$R/gpurun_out/r6_host${TAG:+_$TAG}
mkdir -p $O
for rep in 1 2; do
  for cfg in ${CONFIGS:-1 2}; do
    for v in ${VARIANTS:-new=}; do
      name=${v%%=*}; lib=${v#*=}
      line=$(NEB_LIB_PATH=$lib timeout -k 10 300 python bench.py --config $cfg --mode host-staged --steps 10 --warmup 3 2>>$O/err.log) || exit 1
      echo "$name c$cfg $(echo $line | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')" | tee -a $O/ab.txt
    done
  done
done
cd /tmp && export TMPDIR=/tmp
NEB_LIB_PATH=$TRACE_LIB timeout -k 10 300 rocprofv3 --memory-copy-trace --kernel-trace --output-format csv -d $O/trace -o staged -- python3 $R/bench.py --config 1 --mode host-staged --steps 4 --warmup 1 > $O/trace.log 2>&1 || exit $?
ls $O/trace/*/ 2>/dev/null | head
