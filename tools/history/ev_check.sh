timeout -k 10 200 python bench.py --steps 20 --warmup 5 > gpurun_out/b_ev.json 2> gpurun_out/b_ev.err || { tail -5 gpurun_out/b_ev.err; exit 1; }
python3 -c "import json;d=json.load(open('gpurun_out/b_ev.json'));print(d['value'],d['ms_per_step'],d['roofline'])"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_ev -o e -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_ev.log 2>&1 || exit 1
grep -h "gcm_single" $GRAFT_REPO_ROOT/gpurun_out/prof_ev/*kernel_stats.csv | cut -c1-120
grep "^{" $GRAFT_REPO_ROOT/gpurun_out/prof_ev.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print(d['roofline']['kernel_ms'],d['roofline']['open_kernel_ms'])"
