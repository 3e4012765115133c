#!/bin/bash
# GPU suite on the default library, then the batch-size sweep per build_abl variant.
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/t_small.log 2>&1; rc=$?; tail -2 gpurun_out/t_small.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python __graft_entry__.py smoke 2>&1 | tail -2 || exit 1
for v in $(cat build_abl/variants.txt); do echo "== sweep $v"; NEB_LIB_PATH=$PWD/build_abl/lib_$v.so timeout -k 10 300 python tools/batch_sweep.py 1 16 64 128 512 2048 4096 8192 2> /dev/null || exit 1; done
