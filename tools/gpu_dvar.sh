#!/bin/bash
# config-D bench section for the default library and variants, alternating twice
set -o pipefail
for rep in 1 2; do
for l in "" "$@"; do
  if [ -n "$l" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$l.so INF_ALLOW_STALE_LIB=1; else unset INF_LIB INF_ALLOW_STALE_LIB; fi
  echo "== lib ${l:-default}"
  timeout -k 10 200 python bench.py --steps 30 --warmup 5 --only configD 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        c=json.loads(l)['config_D']; print(round(c['ms_per_step']*1e3,1), {k: round(v['ms']*1e3,1) for k,v in c['stages'].items()})
" || exit 1
done
done
