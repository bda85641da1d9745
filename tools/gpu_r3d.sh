#!/bin/bash
# Round 3: bf16x3 defaults + cheaper role variants, the projection-GEMM tile sweep, kernel
# traces of the fp32 / bf16x3 parity-mode steps.  Assertion failures (rc 1) do not stop it.
O=gpurun_out
step() {
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/r3d_steps.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -s"
step r3d_x3_default.log 300 $PYT tests/test_gpu_bf16x3.py
INF_X3_DX=3 INF_X3_DW=3 step r3d_x3_f6d3w3.log 300 $PYT tests/test_gpu_bf16x3.py
INF_X3_DW=3 step r3d_x3_f6d6w3.log 300 $PYT tests/test_gpu_bf16x3.py
step r3d_ptab_sweep.log 300 python -u tools/ptab_sweep.py
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p $O/prof_r03_fp32 $O/prof_r03_x3
step r3d_prof_fp32.log 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03_fp32 -o run -- \
  python bench.py --mode fp32 --steps 20 --warmup 4 --extra-batches "" --only none --no-cpu-baseline
step r3d_prof_x3.log 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03_x3 -o run -- \
  python bench.py --mode bf16x3 --steps 20 --warmup 4 --extra-batches "" --only none --no-cpu-baseline
