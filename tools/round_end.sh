#!/bin/bash
# Round-end evidence in one gpurun call: probe, smoke, pytest -m gpu, every config, the §8f paths
# (TX, host and device receive), the 2-rank rehearsal, and rocprofv3 passes (trace + counter passes)
# of C2, C3 and C5, condensed on the box (tools/pmc_summary.py, tools/pmc_traffic.py) into
# gpurun_out/sum/ so the results fit gpurun's copy-back limit. Usage: bash tools/round_end.sh TAG [skip-bench]
TAG=${1:-end}
R=${GRAFT_REPO_ROOT:-$(pwd)}
if [ "$2" != "skip-bench" ]; then
  bash tools/gpu_check.sh || exit $?
  bash tools/bench_all.sh || exit $?
  bash tools/bench_paths.sh || exit $?
  rm -rf gpurun_out/paths/prof_tx
  bash tools/rehearse_multi.sh || exit $?
fi
mkdir -p gpurun_out/sum
for spec in "${TAG}:" "${TAG}_c3:--config 2 --steps 10 --warmup 2 --no-cpu-baseline" "${TAG}_c5:--config 4 --steps 4 --warmup 2 --no-cpu-baseline"; do
  t=${spec%%:*}; a=${spec#*:}
  bash tools/profile.sh $t $a > gpurun_out/sum/profile_$t.log 2>&1 || { tail -20 gpurun_out/sum/profile_$t.log; exit 1; }
  python3 tools/pmc_summary.py gpurun_out/prof_$t gpurun_out/sum/$t > /dev/null || exit 1
  python3 tools/trace_gaps.py gpurun_out/prof_$t/trace > gpurun_out/sum/$t/trace_gaps.txt 2>&1
done
python3 tools/pmc_traffic.py gpurun_out/prof_${TAG} gpurun_out/prof_${TAG}_c3 gpurun_out/prof_${TAG}_c5 --out gpurun_out/sum/pmc_traffic.json > /dev/null || exit 1
rm -rf gpurun_out/prof_${TAG} gpurun_out/prof_${TAG}_c3 gpurun_out/prof_${TAG}_c5
du -sh gpurun_out
echo "profiles done"
