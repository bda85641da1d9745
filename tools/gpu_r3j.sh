#!/bin/bash
# Round 3: first GPU run of the fused fp32 chain (chainf.hip): its parity tests, the fp32
# tests that now take it (rays vs oracle, edge cases), the configs bench (fp32_mode_B) and
# a kernel trace of the fp32-mode step
set -o pipefail
O=gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_chainf.py -m gpu -x -v --timeout 120 --timeout-method thread > $O/r3j_tests.log 2>&1 &&
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_edge.py -m gpu -x -v --timeout 120 --timeout-method thread -k "rays_matches_oracle or fused_train_step or adam20 or edge or out_of_range or ragged" >> $O/r3j_tests.log 2>&1 &&
timeout -k 10 300 python bench.py --steps 50 --warmup 10 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only configs > $O/r3j_bench_configs.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/r3j_prof -o f32 -- python bench.py --mode fp32 --steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches "" --only none --no-graph > $O/r3j_prof.log 2>&1
