#!/bin/bash
# A/B of the headline leg (the driver's --steps 20 --warmup 5) between this library and the
# round-start library (libinf_hip_base.so), alternated; also configs A and R.
set -o pipefail
O=gpurun_out/${1:-ab}
mkdir -p $O
BASE="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_base.so INF_ALLOW_STALE_LIB=1"
H="--steps 20 --warmup 5 --no-render --no-cpu-baseline --no-config-d --extra-batches= --only configs"
for r in 1 2 3; do
  for lib in new base; do
    if [ $lib = base ]; then E=$BASE; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py $H > $O/${lib}_$r.log 2>&1 || exit 1
    grep '^{' $O/${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); s=d['summary']; print('$lib $r', s['B_us'], s['stages_us'], 'A', s.get('A_us'), 'R', s.get('R_us'))"
  done
done
