#!/bin/bash
# Round 3 closing run at HEAD (after the lgemm epilogue swizzle): GPU suite, smoke, full bench
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/fin3_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> $O/fin3_tests.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/fin3_smoke.log 2>&1 || exit 1
timeout -k 10 700 python bench.py > $O/fin3_bench.log 2>&1
