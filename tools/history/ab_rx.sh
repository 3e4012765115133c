#!/bin/bash
# A/B of the host-resident batched receive (bench.py --mode rx) over build_abl variants, C2 and C3,
# two interleaved rounds on one box. Usage (GPU box): bash tools/ab_rx.sh
R=$(pwd)
for round in 1 2; do for cfg in 1 2; do for v in $(cat build_abl/variants.txt); do
  NEB_LIB_PATH=$R/build_abl/lib_$v.so timeout -k 10 200 python bench.py --mode rx --steps 4 --warmup 1 --config $cfg \
    > gpurun_out/rx_ab.json 2>/dev/null || exit 1
  echo "cfg $cfg $v $(python3 -c "import json;d=json.load(open('gpurun_out/rx_ab.json'));print('rx', d['value'], 'open', d['open_only_gibs'])")"
done; done; done
