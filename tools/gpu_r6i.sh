#!/bin/bash
# Round 6: the fused dW + update (lgemm GT) with two k groups (variant library
# libinf_hip_gtks2.so, -DLG_GT_KS=2) against one: parity tests of the LGF path on the
# variant, the block schedule at config D, and config D's step, alternated.
set -o pipefail
O=gpurun_out/${1:-r6i}
mkdir -p $O
VAR="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_gtks2.so INF_ALLOW_STALE_LIB=1"
env $VAR timeout -k 10 400 python -u -m pytest tests/test_gpu_config_d_adam.py tests/test_gpu_shard.py "tests/test_gpu_kernels.py::test_lgf_update_matches_slab_path" "tests/test_gpu_kernels.py::test_bf16_chunked_chain3_matches_bf16_oracle" -x -q -s --timeout 300 --timeout-method thread > $O/tests_var.log 2>&1; rc=$?
tail -2 $O/tests_var.log; [ $rc -eq 0 ] || exit $rc
grep -o "D 0\.[0-9e-]* {[^}]*}" $O/tests_var.log | cut -c1-400
for lib in def var; do
  if [ $lib = var ]; then E=$VAR; else E=""; fi
  env $E LGB_STEP=1 timeout -k 10 120 python3 tools/lgemm_blocks.py 4096 4096 > $O/blocks_$lib.log 2>&1 || exit 1
  echo "== $lib"; tail -7 $O/blocks_$lib.log
done
for r in 1 2; do
  for lib in def var; do
    if [ $lib = var ]; then E=$VAR; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --only configD --no-render --no-cpu-baseline --extra-batches= > $O/d_${lib}_$r.log 2>&1 || exit 1
    grep '^{' $O/d_${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); c=d['config_D']; print('$lib $r D', round(c['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,2) for k,v in c['stages'].items()}, 'B', d['summary']['B_us'])"
  done
done
