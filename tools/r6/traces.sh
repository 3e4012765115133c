#!/bin/bash
# rocprofv3 kernel traces of bench configs (CONFIGS "4:8 2 4"), with NEB_LIB_PATH=$LIB if set.
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/r6_traces${TAG:+_$TAG}
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in ${CONFIGS:-4:8 2}; do
  c=${cfg%%:*}; so=""; nm=c$c; [ "$cfg" != "$c" ] && so="--shard-of ${cfg#*:}" && nm=c${c}s${cfg#*:}
  NEB_LIB_PATH=$LIB timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/$nm -o $nm -- python3 $R/bench.py --config $c $so --steps 10 --warmup 2 --no-cpu-baseline > $O/$nm.log 2>&1 || exit $?
  echo "== $nm"; find $O/$nm -name '*kernel_stats.csv' -exec cut -d, -f1-4 {} \; | head -8
done
