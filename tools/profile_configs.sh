#!/bin/bash
# Counter passes (tools/profile.sh) for every bench config, one after another, each condensed on
# the box (tools/pmc_summary.py) into gpurun_out/profiles/<tag> and its raw passes deleted, so what
# comes back stays small. Stops at the first failure.
# Usage (GPU box): tools/profile_configs.sh TAGPREFIX [config numbers, default "1 2 3 4"]
P=${1:-r3}; shift
CFGS=${@:-1 2 3 4}
for c in $CFGS; do
    n=$((c + 1))
    echo "== C$n"
    tools/profile.sh ${P}_c$n --config $c --steps 10 --warmup 2 --no-cpu-baseline > gpurun_out/prof_${P}_c$n.log 2>&1 || { tail -20 gpurun_out/prof_${P}_c$n.log; exit 1; }
    grep -E "rc=" gpurun_out/prof_${P}_c$n.log | tr '\n' ' '; echo
    python3 tools/pmc_summary.py gpurun_out/prof_${P}_c$n gpurun_out/profiles/${P}_c$n || exit 1
    cp gpurun_out/prof_${P}_c$n/trace/trace.log gpurun_out/profiles/${P}_c$n/bench.log 2>/dev/null
    rm -rf gpurun_out/prof_${P}_c$n
done
