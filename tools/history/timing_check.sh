#!/bin/bash
# The bench lines of every config with dispatch-bound kernel timing: value, step, seal / open kernel ms, roofline fraction.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
for c in 1 2 3 4 0; do
  st=20; [ $c = 4 ] && st=10
  timeout -k 10 300 python bench.py --config $c --steps $st --warmup 5 --no-cpu-baseline > gpurun_out/tb_c$c.json 2> gpurun_out/tb_c$c.err || { tail -5 gpurun_out/tb_c$c.err; exit 1; }
  python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print('C%d' % (int(sys.argv[2])+1), d['value'], d['ms_per_step'], r['kernel_ms'], r['open_kernel_ms'], r['frac'], r.get('kernel_timing'))" gpurun_out/tb_c$c.json $c
done
