#!/bin/bash
# lgemm slab epilogue with the swizzled LDS tile: kernel tests, the headline line, the step's
# kernel trace (lgemm average)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_chainf.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r3ae_tests.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --only none --no-cpu-baseline --extra-batches "" > $O/r3ae_b.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r3ae -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --only none --no-cpu-baseline --extra-batches "" > $O/r3ae_prof.log 2>&1
