#!/bin/bash
# Round 3: the bf16x3 parity tests, the secondary configs (A, R, fp32 and bf16x3 modes), and a
# kernel-trace profile of the 65,536-ray step.  Logs under gpurun_out/.
set -o pipefail
O=gpurun_out
mkdir -p $O/prof_r03_65k
timeout -k 10 300 python -u -m pytest tests/test_gpu_bf16x3.py -x -q --timeout 120 --timeout-method thread -s \
  > $O/r3_bf16x3_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --only configs --no-cpu-baseline --steps 50 --warmup 5 > $O/r3_bench_configs.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03_65k -o run -- \
  python bench.py --batch 65536 --steps 16 --warmup 4 --extra-batches "" --only none --no-cpu-baseline \
  > $O/r3_prof65k.log 2>&1
