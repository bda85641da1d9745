#!/bin/bash
# bf16x3 dW on the split-operand register GEMM: parity tests, then stage timing of both modes
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chainf.py tests/test_gpu_bf16x3.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r3w_tests.log 2>&1 || exit 1
: > $O/r3w_timing.log
for m in bf16x3 fp32; do
  timeout -k 10 120 python tools/chainf_timing.py $m >> $O/r3w_timing.log 2>&1 || exit 1
done
INF_NO_SPLIT_LGEMM=1 timeout -k 10 120 python tools/chainf_timing.py bf16x3 >> $O/r3w_timing.log 2>&1
