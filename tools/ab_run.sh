# One gpurun call: GPU parity tests, then seal timings of every tools/ablate.sh build (CFGS="2 4 7")
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_gpu.log; [ $rc -ne 0 ] && exit $rc
R=$(pwd)
for cfg in ${CFGS:-2 4 7}; do for round in 1 2; do for v in $(cat build_abl/variants.txt); do
  echo -n "cfg $cfg: "; NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 120 python3 tools/ablate_run.py $cfg 2>/dev/null | tail -1 || exit 1
done; done; done
