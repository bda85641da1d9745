#!/bin/bash
# packed hi / lo conversion in chainf's split-image copy + split-major fgemm block order:
# parity tests, stage timing, the configs line and the 65,536-ray step
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_chainf.py tests/test_gpu_bf16x3.py "tests/test_gpu_kernels.py::test_chain3_wide_tiles_match_narrow" "tests/test_gpu_kernels.py::test_bf16_chain_matches_layered_and_oracle" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r3ab_tests.log 2>&1 || exit 1
: > $O/r3ab.log
for m in bf16x3 bf16x3; do
  timeout -k 10 120 python tools/chainf_timing.py $m 2>&1 | grep -E "chain |dw|update|step" >> $O/r3ab.log || exit 1
done
timeout -k 10 500 python bench.py --only configs --no-cpu-baseline --extra-batches 65536 > $O/r3ab_bench.log 2>&1
