#!/bin/bash
# Round 6: strong-scaling local steps (DP step shape at world 1), this library against the
# round-start library (libinf_hip_base.so), alternated.
set -o pipefail
O=gpurun_out/${1:-r6h}
mkdir -p $O
BASE="INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_base.so INF_ALLOW_STALE_LIB=1"
for r in 1 2; do
  for lib in new base; do
    if [ $lib = base ]; then E=$BASE; else E=""; fi
    env $E timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --only strong --no-render --no-cpu-baseline --no-config-d --extra-batches= > $O/strong_${lib}_$r.log 2>&1 || exit 1
    grep '^{' $O/strong_${lib}_$r.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$lib $r', d['summary']['B_us'], d['summary']['strong_local_us'])"
  done
done
