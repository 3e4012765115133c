timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_tx.py tests/test_gpu_cipher_state.py > gpurun_out/t_relay.log 2>&1; rc=$?; tail -2 gpurun_out/t_relay.log; [ $rc -eq 0 ] || exit $rc
for v in BASE NEW; do for c in 1 2; do echo -n "relay $v c$c "; NEB_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 120 python bench.py --mode relay --config $c --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1; done; done
timeout -k 10 200 python bench.py --mode relay --steps 20 --warmup 5 > gpurun_out/relay_c1.json 2>/dev/null || exit 1
timeout -k 10 200 python bench.py --mode relay --config 2 --steps 20 --warmup 5 > gpurun_out/relay_c2.json 2>/dev/null || exit 1
bash tools/ab_cfgs.sh 1 2 > gpurun_out/ab_gmac_skip.log 2>&1 || exit 1
grep -v "^  neb::sched\|at::native" gpurun_out/ab_gmac_skip.log
