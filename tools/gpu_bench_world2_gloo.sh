#!/bin/bash
# Rehearsal of bench.py's N > 1 path on a one-GPU box: two ranks share the GPU over gloo
# (eager all-reduce between the captured steps).  The driver's real multi-GPU run uses RCCL.
set -o pipefail
INF_DP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 40 --warmup 8 "$@"
