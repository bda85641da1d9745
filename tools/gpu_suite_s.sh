#!/bin/bash
# The GPU suite with test output kept (-s): the derived bars' measured values land in the log.
set -o pipefail
O=gpurun_out/${1:-suite}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log
grep -E "^(D |4096 |1024 )|weights rel|scalars rel|^bf16 bar|^fp32 bar|^\{'fp32'" $O/tests.log | cut -c1-600
exit $rc
