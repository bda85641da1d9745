#!/bin/bash
# ZP schedule (igemm.hip ahead of chain3): kernel tests first, then the whole GPU suite,
# the headline step line and its kernel trace
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/r3r_kernels.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r3r_tests.log 2>&1
echo "pytest rc=$?" >> $O/r3r_tests.log
timeout -k 10 300 python bench.py --only none --no-cpu-baseline --extra-batches "" > $O/r3r_bench.log 2>&1 || exit 1
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r3r -o run --output-format csv -- python3 bench.py --steps 40 --warmup 10 --only none --no-cpu-baseline --extra-batches "" > $O/r3r_prof.log 2>&1
