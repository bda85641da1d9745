#!/bin/bash
# lgemm8 (128 x 128, 8 waves) correctness under the kernel tests, then step timing vs the
# default 64 x 128 kernel at split-K 2 / 4 / 8 (alternated).
set -o pipefail
INF_LG8=1 INF_DW_SPLITS=4 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "bf16_chain_matches or dp_step_shape or train_step" > gpurun_out/lg8_t.log 2>&1; rc=$?
tail -3 gpurun_out/lg8_t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in "def:" "lg8s4:INF_LG8=1 INF_DW_SPLITS=4" "lg8s8:INF_LG8=1 INF_DW_SPLITS=8" "s4:INF_DW_SPLITS=4"; do
    n=${v%%:*}; e=${v#*:}
    echo "== $n"
    env $e timeout -k 10 100 python tools/xslot_gain.py 2>&1 | grep in-kernel || exit 1
  done
done
