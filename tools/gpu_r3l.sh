#!/bin/bash
# Round 3: chainf with the LDS-DMA chunked gather -- parity tests, stage times (fp32, bf16x3)
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chainf.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/r3l_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_edge.py tests/test_gpu_bf16x3.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rays or fused_train_step or adam20 or fp32 or out_of_range" >> $O/r3l_tests.log 2>&1 &&
timeout -k 10 120 python tools/chainf_timing.py fp32 > $O/r3l_timing.log 2>&1 &&
timeout -k 10 120 python tools/chainf_timing.py bf16x3 >> $O/r3l_timing.log 2>&1
