#!/bin/bash
# Round 3: wide-tile chain tests + the out-of-range edge test, the wide chain's phase stamps
# at 65,536 rays, bench lines at 65,536 and 4,096 rays, and kernel traces of the 65,536-ray
# bf16 step and the 4,096-ray bf16x3 (split-bf16 parity) step.
set -o pipefail
O=gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -m gpu -x -v --timeout 120 --timeout-method thread -k "chain and (wide or 20000 or 32768 or 16384)" > $O/r3h_tests.log 2>&1 &&
timeout -k 10 200 python -u -m pytest tests/test_gpu_edge.py -m gpu -x -v --timeout 120 --timeout-method thread -k "out_of_range" >> $O/r3h_tests.log 2>&1 &&
timeout -k 10 200 python tools/chain3_timing.py 65536 > $O/r3h_chain3_timing_65k.log 2>&1 &&
timeout -k 10 300 python bench.py --batch 65536 --steps 50 --warmup 10 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none > $O/r3h_bench_65k.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 200 --warmup 20 --no-render --no-cpu-baseline --no-config-d --only none > $O/r3h_bench_4k.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3h_prof -o b65k -- python bench.py --batch 65536 --steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none --no-graph > $O/r3h_prof.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3h_prof -o x3 -- python bench.py --mode bf16x3 --steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none --no-graph > $O/r3h_prof_x3.log 2>&1
