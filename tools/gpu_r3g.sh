#!/bin/bash
# Round 3: first GPU run of chain3's 64-ray tiles -- the chain tests (wide vs narrow tiles,
# vs the layered kernels and the oracle, ragged and out-of-range batches), the wide chain's
# phase stamps at 65,536 rays, and bench lines at 65,536 and 4,096 rays.
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chain and (wide or 20000 or 32768 or 16384)" > $O/r3g_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_edge.py -m gpu -x -v --timeout 120 --timeout-method thread -k "out_of_range" >> $O/r3g_tests.log 2>&1 &&
timeout -k 10 200 python tools/chain3_timing.py 65536 > $O/r3g_chain3_timing_65k.log 2>&1 &&
timeout -k 10 300 python bench.py --batch 65536 --steps 50 --warmup 10 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none > $O/r3g_bench_65k.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-render --no-cpu-baseline --no-config-d --only none > $O/r3g_bench_4k.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3g_prof -o b65k -- python bench.py --batch 65536 --steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none --no-graph > $O/r3g_prof.log 2>&1
