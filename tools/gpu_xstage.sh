#!/bin/bash
# chunked-tile staging: config-D parity tests, then the config-D bench section
set -o pipefail
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_large.py tests/test_gpu_prefetch.py -x -v --timeout 200 --timeout-method thread > gpurun_out/xs_test.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --only configD > gpurun_out/xs_bench.log 2>&1
