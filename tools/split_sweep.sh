#!/bin/bash
# headline-step variants (GPU box): dW split-K factor, lgemm rows per block, fused update
set -uo pipefail
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u bench.py --steps 200 --warmup 10 --no-render --no-cpu-baseline --extra-batches "" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), {k:round(v['ms']*1e3,2) for k,v in d['stages'].items()})"; }
if [ $# -gt 0 ]; then for v in "$@"; do run $v; done; exit 0; fi
for bm in 32 64; do for s in 1 2 4; do run INF_LGEMM_BM=$bm INF_DW_SPLITS=$s; done; done
