#!/bin/bash
# bf16x3 / fp32 parity-mode steps after the batched split-image copy: tests, stage timing,
# the bench's secondary lines
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chainf.py tests/test_gpu_bf16x3.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r3x_tests.log 2>&1 || exit 1
: > $O/r3x_timing.log
for m in bf16x3 fp32 bf16x3; do
  timeout -k 10 120 python tools/chainf_timing.py $m >> $O/r3x_timing.log 2>&1 || exit 1
done
timeout -k 10 400 python bench.py --only none --no-cpu-baseline > $O/r3x_bench.log 2>&1
