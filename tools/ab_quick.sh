# A/B timing only (no tests): every build_abl variant on the configs in CFGS (ablate_run.py indices:
# 1 = C2 single key, 2 = C3 4096 keys, 4 = C5 IMIX share), two interleaved rounds.
mkdir -p gpurun_out
R=$(pwd)
for cfg in ${CFGS:-1}; do for round in 1 2; do for v in $(cat build_abl/variants.txt); do
  echo -n "cfg $cfg: "; NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 tools/ablate_run.py $cfg 2>/dev/null | tail -1 || exit 1
done; done; done
