#!/bin/bash
# Round 5: the multi-rank bench in both launch forms on the one-GPU box (ranks share the device):
# bare `bench.py --gpus 2` (the script starts its ranks) and torch.distributed.run.
mkdir -p gpurun_out/r5_multi
timeout -k 10 300 python bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r5_multi/bare_g2.json 2> gpurun_out/r5_multi/bare_g2.err || exit $?
cat gpurun_out/r5_multi/bare_g2.json
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 \
    bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r5_multi/torchrun_g2.json 2> gpurun_out/r5_multi/torchrun_g2.err || exit $?
cat gpurun_out/r5_multi/torchrun_g2.json
timeout -k 10 300 python bench.py --gpus 2 --config 4 --steps 5 --warmup 2 > gpurun_out/r5_multi/bare_c5_g2.json 2> gpurun_out/r5_multi/bare_c5_g2.err || exit $?
cat gpurun_out/r5_multi/bare_c5_g2.json
