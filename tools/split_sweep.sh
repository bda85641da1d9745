#!/bin/bash
# dW split-K factor x lgemm rows-per-block sweep of the headline step (GPU box)
set -uo pipefail
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u bench.py --steps 100 --warmup 10 --no-render --no-cpu-baseline --extra-batches "" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,2), {k:round(v['ms']*1e3,2) for k,v in d['stages'].items()})"; }
for bm in 32 64; do for s in 1 2 4; do run INF_LGEMM_BM=$bm INF_DW_SPLITS=$s; done; done
