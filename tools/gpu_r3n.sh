#!/bin/bash
# Round 3 checkpoint after the fused fp32 chain: whole GPU suite, smoke, the full bench line
set -o pipefail
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r3n_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/r3n_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3n_smoke.log 2>&1 &&
timeout -k 10 700 python bench.py > $O/r3n_bench.log 2>&1
