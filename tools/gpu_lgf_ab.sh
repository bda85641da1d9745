#!/bin/bash
# The fused dW + Adam launch (lgemm.hip GT) with two k groups per block and the items' Adam
# state loaded in the main loop's last stages (INF_LGF_KS=2): its parity tests, then the
# headline step (config B) alternated between the default slab path + update launch, the
# one-group fused launch and the two-group one; config D's step likewise; block schedules.
set -o pipefail
O=gpurun_out/${1:-lgf}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_config_d_adam.py tests/test_gpu_shard.py -x -q --timeout 200 \
  --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
H="--steps 200 --warmup 20 --no-render --no-cpu-baseline --no-config-d --extra-batches= --only configs"
AF="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_auxfirst.so INF_ALLOW_STALE_LIB=1"
for r in 1 2; do
  for v in def lgf lgf2 lgf2af; do
    case $v in def) E="INF_LGF=0";; lgf) E="INF_LGF=1 INF_LGF_KS=1";; lgf2) E="INF_LGF=1 INF_LGF_KS=2";;
      lgf2af) E="INF_LGF=1 INF_LGF_KS=2 $AF";; esac
    env $E timeout -k 10 300 python3 bench.py $H > $O/B_${v}_$r.log 2>&1 || exit 1
    grep '^{' $O/B_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['summary']; print('B $v $r', s['B_us'], s['stages_us'], 'A', s.get('A_us'), 'R', s.get('R_us'))"
  done
done
HD="--steps 20 --warmup 5 --no-render --no-cpu-baseline --extra-batches= --only configD"
for r in 1 2; do
  for v in lgf lgfaf; do
    case $v in lgf) E="INF_LGF_KS=1";; lgfaf) E="INF_LGF_KS=1 $AF";; esac
    env $E timeout -k 10 300 python3 bench.py $HD > $O/D_${v}_$r.log 2>&1 || exit 1
    grep '^{' $O/D_${v}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['summary']; print('D $v $r', s['D_us'])"
  done
done
for v in lgf lgf2; do
  case $v in lgf) E="INF_LGF=1 INF_LGF_KS=1";; lgf2) E="INF_LGF=1 INF_LGF_KS=2";; esac
  env $E timeout -k 10 120 python3 tools/lgemm_blocks.py 4096 1024 > $O/blocks_B_$v.log 2>&1 || exit 1
  env $E timeout -k 10 120 python3 tools/lgemm_blocks.py 4096 4096 > $O/blocks_D_$v.log 2>&1 || exit 1
  tail -7 $O/blocks_B_$v.log; tail -7 $O/blocks_D_$v.log
done
