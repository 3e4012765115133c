#!/bin/bash
# Multi-rank rehearsal on a one-GPU box: bench.py under torch.distributed.run with 2 ranks sharing
# the device (the timing is meaningless, the launch, barrier, shard and max-over-ranks path is not).
mkdir -p gpurun_out/multi
for cfg in 1 4; do
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
      --master-port 29511 bench.py --gpus 2 --steps 5 --warmup 2 --config $cfg --no-cpu-baseline \
      > gpurun_out/multi/n2_c$cfg.json 2> gpurun_out/multi/n2_c$cfg.err || exit $?
  cat gpurun_out/multi/n2_c$cfg.json
done
