#!/bin/bash
# Round 3: GPU suite, smoke, the default bench line, the world-1 data-parallel shapes over
# RCCL (torchrun) and the world-2 gloo rehearsal of bench.py's N > 1 path.  Logs under gpurun_out/.
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r3_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3_smoke.log 2>&1 &&
timeout -k 10 600 python bench.py > $O/r3_bench.log 2>&1 &&
INF_BENCH_DP=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
  --master-addr 127.0.0.1 --master-port 29517 bench.py --steps 200 --warmup 20 --only none --no-cpu-baseline \
  > $O/r3_bench_dp1.log 2>&1 &&
INF_DP_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29519 bench.py --gpus 2 --steps 40 --warmup 8 > $O/r3_bench_gloo2.log 2>&1
