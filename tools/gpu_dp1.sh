#!/bin/bash
# World-1 data-parallel step shape through torchrun (RCCL communicator, all-reduce captured
# in the step graphs): bench.py's headline section only.  Run on the GPU box via gpurun.
set -o pipefail
INF_BENCH_DP=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 200 --warmup 20 --only none --no-cpu-baseline "$@"
