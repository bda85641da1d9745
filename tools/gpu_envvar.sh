#!/bin/bash
# headline bench line under environment variants, alternated twice:
#   bash tools/gpu_envvar.sh "" "INF_LG_BM=128 INF_DW_SPLITS=4" ...
set -o pipefail
for rep in 1 2; do
for v in "$@"; do
  echo "== ${v:-default}"
  env $v timeout -k 10 200 python bench.py --steps 200 --warmup 20 --only headline 2>/dev/null | python3 -c "
import json,sys
for l in sys.stdin:
    if l.startswith('{'):
        d=json.loads(l); print(round(d['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,1) for k,v in d['stages'].items()})
" || exit 1
done
done
