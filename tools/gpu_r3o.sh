#!/bin/bash
# Round 3 session-3 checkpoint: whole GPU suite + smoke (logs under gpurun_out/)
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 1050 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/r3o_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/r3o_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r3o_smoke.log 2>&1
