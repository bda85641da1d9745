#!/bin/bash
# Round 3 checkpoint: GPU suite, smoke, the full bench line, and the LDS-ring chain's phase
# timing at 65,536 rays (tile heights 128 and 64).  Logs under gpurun_out/.
set -o pipefail
O=gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/r3f_tests.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3f_smoke.log 2>&1 &&
timeout -k 10 700 python bench.py > $O/r3f_bench.log 2>&1 &&
timeout -k 10 200 python tools/chain_timing.py 65536 > $O/r3f_chain_timing_65k_bm128.log 2>&1 &&
INF_CHAIN_BM=64 timeout -k 10 200 python tools/chain_timing.py 65536 > $O/r3f_chain_timing_65k_bm64.log 2>&1
