#!/bin/bash
# The update's 16-byte accesses to arena rows that are not 16-byte aligned (config R's
# k = 1023): GPU suite, then config R's step (the reference's intrinsic_cat.yaml) alternated
# with the library before it (libinf_hip_base.so), and the headline once each.
set -o pipefail
O=gpurun_out/${1:-unaligned}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?
tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
BASE="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_base.so INF_ALLOW_STALE_LIB=1"
R="--k 1023 --layers 6 --hidden 128 --skip 3 --loss L1 --steps 200 --warmup 20 --no-render --no-cpu-baseline --no-config-d --extra-batches= --only none"
for r in 1 2 3; do
  for lib in new base; do
    if [ $lib = base ]; then E=$BASE; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py $R > $O/R_${lib}_$r.log 2>&1 || exit 1
    grep '^{' $O/R_${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('R $lib $r', round(d['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,2) for k,v in d['stages'].items()})"
  done
done
