#!/bin/bash
# round 3: 2-rank rehearsal of the bench's N > 1 path on the one GPU (gloo exchange; RCCL refuses two ranks per card)
set -o pipefail
mkdir -p gpurun_out
export BCMPC_DIST_BACKEND=gloo BCMPC_BENCH_DEVICE=0
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29533 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r03_rehearsal_2rank.json 2> gpurun_out/r03_rehearsal_2rank.err
