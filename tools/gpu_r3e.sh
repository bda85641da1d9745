#!/bin/bash
# Round 3: bf16x3 parity with the role defaults (forward 6, backward 3), GEMM occupancy
# experiment, projection-GEMM variants.  Assertion failures (rc 1) do not stop it.
O=gpurun_out
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/r3e_steps.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -s"
step r3e_x3.log 300 $PYT tests/test_gpu_bf16x3.py
step r3e_gemm_occ.log 300 python -u tools/gemm_occupancy.py
step r3e_ptab_sweep.log 300 python -u tools/ptab_sweep.py
step r3e_render_tests.log 300 $PYT tests/test_gpu_render.py -k "project"
