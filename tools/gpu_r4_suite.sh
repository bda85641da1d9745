#!/bin/bash
# Whole GPU suite (logs under gpurun_out/), then smoke.
set -o pipefail
O=gpurun_out
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider -s > $O/r4_suite.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/r4_suite.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/r4_smoke.log 2>&1
