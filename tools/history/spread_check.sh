#!/bin/bash
# GPU suite, the batch-size sweep per variant, and the full-size A/B (C2, C3) of build_abl variants.
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_spread.log 2>&1; rc=$?; tail -2 gpurun_out/t_spread.log; [ $rc -eq 0 ] || exit $rc
for v in $(cat build_abl/variants.txt); do echo "== sweep $v"; NEB_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 300 python tools/batch_sweep.py 64 128 512 2048 8192 2> /dev/null || exit 1; done
bash tools/ab_cfgs.sh 1 2 > gpurun_out/ab_spread.log 2>&1 || exit 1
grep -v "^  neb::sched\|at::native" gpurun_out/ab_spread.log
