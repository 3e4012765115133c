#!/bin/bash
# One GPU session: probe -> smoke -> pytest -m gpu -> bench. Stops at the first step that dies
# abnormally (exit > 1: fault, abort, timeout); test failures (exit 1) still let later steps run.
mkdir -p gpurun_out
step() {  # name timeout cmd...
    local name=$1 t=$2; shift 2
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "$name rc=$rc"
    tail -n 25 "gpurun_out/$name.log"
    if [ $rc -gt 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
    return 0
}
step probe 120 python tools/probe.py
step smoke 300 python __graft_entry__.py smoke
step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider
step bench 400 python bench.py --steps 20 --warmup 5
