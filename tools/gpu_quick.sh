#!/bin/bash
# GPU suite + step timing (3 reps) + world-1 DP step: one gpurun call after a kernel change.
set -o pipefail
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/q_t.log 2>&1; rc=$?
tail -3 gpurun_out/q_t.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do bash tools/gpu_step_variants.sh >> gpurun_out/q_s.log 2>&1 || exit 1; done
python tools/agg_variants.py gpurun_out/q_s.log
bash tools/gpu_dp1.sh > gpurun_out/q_dp.log 2>&1; rc=$?
grep '^{' gpurun_out/q_dp.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dp1', d['ms_per_step']*1e3, d['stages'])"
exit $rc
