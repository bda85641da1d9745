#!/bin/bash
# Round 3: fgemm with 32-ray stages and a 5-deep LDS ring -- the wide-tile tests (fgemm vs
# lgemm on the same images, the oracle at 16,384-32,768 rays) and the 65,536-ray bench
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chain and (wide or 20000 or 32768 or 16384)" > $O/r3i_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --batch 65536 --steps 50 --warmup 10 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none > $O/r3i_bench_65k.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3i_prof -o b65k -- python bench.py --batch 65536 --steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none --no-graph > $O/r3i_prof.log 2>&1
