#!/bin/bash
# Ring-depth / tile sweep over prebuilt variants libinf_hip_c<chain3 depth>_l<lgemm depth>.so
set -uo pipefail
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u bench.py --steps 50 --warmup 10 --no-render --no-cpu-baseline --extra-batches "" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), {k:round(v['ms']*1e3,1) for k,v in d['stages'].items()})"; }
L=intrinsic-neural-fields_amd/inf_hip
run INF_LGEMM_BM=32
run INF_LGEMM_BM=64
for v in c8_l8 c2_l2 c8_l4; do run INF_LIB=$L/libinf_hip_$v.so INF_LGEMM_BM=32; done
run INF_LGEMM_BM=32 INF_DW_SPLITS=4
run INF_LGEMM_BM=32 INF_DW_SPLITS=16
