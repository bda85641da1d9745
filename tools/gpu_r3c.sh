#!/bin/bash
# Round 3: split-bf16 (bf16x3 / x6) parity variants, the hand-written projection GEMM, the
# secondary configs + render bench, a kernel-trace profile of the 65,536-ray step.
# A test step that fails its assertions (rc 1) does not stop the script; anything else does.
O=gpurun_out
step() {  # step <log> <seconds> <cmd...>
  local log=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $O/$log 2>&1
  local rc=$?
  echo "$log rc=$rc" >> $O/r3c_steps.txt
  if [ $rc -gt 1 ]; then exit $rc; fi
}
PYT="python -u -m pytest -x -q --timeout 200 --timeout-method thread -s"
step r3c_x3_default.log 300 $PYT tests/test_gpu_bf16x3.py
INF_X3_FWD=6 INF_X3_DX=6 INF_X3_DW=6 step r3c_x3_all6.log 300 $PYT tests/test_gpu_bf16x3.py
INF_X3_DX=3 INF_X3_DW=3 step r3c_x3_all3.log 300 $PYT tests/test_gpu_bf16x3.py
INF_X3_DX=6 INF_X3_DW=3 step r3c_x3_dx6.log 300 $PYT tests/test_gpu_bf16x3.py
step r3c_render_tests.log 400 $PYT tests/test_gpu_render.py tests/test_gpu_host.py -k "project or projected or render"
step r3c_bench_configs.log 400 python bench.py --only configs,render --no-cpu-baseline --steps 50 --warmup 5
mkdir -p $O/prof_r03_65k
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
step r3c_prof65k.log 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03_65k -o run -- \
  python bench.py --batch 65536 --steps 16 --warmup 4 --extra-batches "" --only none --no-cpu-baseline
