#!/bin/bash
# Round-4 final evidence, part 1 (PART=prof): rocprof kernel trace + counter passes of every device
# config (tools/profile_configs.sh r4f), condensed under gpurun_out/profiles/r4f_c*.
# Part 2 (PART=bench): every BASELINE config through bench.py with its CPU baseline, the per-packet
# sweep and the submission queue (tools/r4_evidence.sh), into gpurun_out/r4e.
# Stops at the first abnormal exit.
R=${GRAFT_REPO_ROOT:-$(pwd)}
cd $R
mkdir -p gpurun_out/profiles
case ${PART:-prof} in
  prof) bash tools/profile_configs.sh r4f ${CFGS:-1 2 3 4} ;;
  bench) bash tools/r4_evidence.sh ;;
esac
