#!/bin/bash
# config-D bench section under environment variants, alternated twice:
#   bash tools/gpu_denv.sh "" "INF_LGF=0" ...
set -o pipefail
for rep in 1 2; do
for v in "$@"; do
  echo "== ${v:-default}"
  env $v timeout -k 10 200 python bench.py --steps 30 --warmup 5 --only configD 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        c=json.loads(l)['config_D']; print(round(c['ms_per_step']*1e3,1), c.get('path'), {k: round(v['ms']*1e3,1) for k,v in c['stages'].items()})
" || exit 1
done
done
