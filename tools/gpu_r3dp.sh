#!/bin/bash
# Round 3 final: bench.py's data-parallel shapes at world 1 over RCCL (torchrun) and the
# world-2 gloo rehearsal of the N > 1 path (two ranks on the one GPU)
set -o pipefail
O=gpurun_out
mkdir -p $O
bash tools/gpu_dp1.sh > $O/dp1_rccl.log 2>&1 || exit 1
bash tools/gpu_bench_world2_gloo.sh --only none --no-cpu-baseline --extra-batches "" > $O/dp2_gloo.log 2>&1
