#!/bin/bash
# Round 6 (second session): full GPU suite + smoke + the driver's bench command at HEAD.
set -o pipefail
O=gpurun_out/${1:-r6s}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 1
tail -2 $O/smoke.log
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
grep '^{' $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(json.dumps(d['summary']))"
