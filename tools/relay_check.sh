#!/bin/bash
# Relay (GMAC / Poly1305-only) parity and rates, and an A/B of the build_abl variants on C2-C4.
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py > gpurun_out/t_relay.log 2>&1; rc=$?; tail -2 gpurun_out/t_relay.log; [ $rc -eq 0 ] || exit $rc
for v in $(cat build_abl/variants.txt); do for c in 1 2 3; do echo -n "relay $v c$c "; NEB_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 120 python bench.py --mode relay --config $c --steps 20 --warmup 5 2>/dev/null | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" || exit 1; done; done
for c in 1 2 3; do timeout -k 10 200 python bench.py --mode relay --config $c --steps 20 --warmup 5 > gpurun_out/relay_c$c.json 2>/dev/null || exit 1; done
bash tools/ab_cfgs.sh ${AB_CFGS:-1 2} > gpurun_out/ab_relay.log 2>&1 || exit 1
grep -v "^  neb::sched\|at::native" gpurun_out/ab_relay.log
