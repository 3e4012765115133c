cd ${GRAFT_REPO_ROOT:-.}
mkdir -p gpurun_out/exp
export TMPDIR=/tmp
for v in default nofuse; do
  if [ $v = nofuse ]; then export NEB_SUB_BINS_FROM=0; fi
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/exp/$v -o run -- python bench.py --mode rx-device --config 2 --steps 6 --warmup 2 --no-cpu-baseline > gpurun_out/exp/$v.log 2>&1 || exit $?
  grep -h metric gpurun_out/exp/$v.log | cut -c1-200
  python - <<PY
import csv,glob
f=glob.glob("gpurun_out/exp/$v/**/*kernel_stats.csv",recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'chunk' in r['Name'] or 'sched' in r['Name']: print("$v", r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
done
