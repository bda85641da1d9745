#!/bin/bash
# GEMM stage-count sweep: prebuilt variants libinf_hip_s<64x64 stages>_<128x128 stages>.so
set -uo pipefail
run() { echo "== $*"; env "$@" timeout -k 10 120 python -u bench.py --steps 50 --warmup 10 --no-render --no-cpu-baseline --extra-batches "" 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print(round(d['ms_per_step']*1e3,1), {k:round(v['ms']*1e3,1) for k,v in d['stages'].items()})"; }
L=intrinsic-neural-fields_amd/inf_hip
run INF_TILE_INPUT=64x64
for v in s8_2 s8_4 s6_3 s4_4; do
  run INF_LIB=$L/libinf_hip_$v.so INF_TILE_INPUT=64x64
  run INF_LIB=$L/libinf_hip_$v.so INF_TILE_INPUT=64x64 INF_DW_SPLITS=4
done
run INF_LIB=$L/libinf_hip_s8_4.so INF_TILE_INPUT=64x64 INF_TILE_DW=64x64 INF_DW_SPLITS=4
run INF_LIB=$L/libinf_hip_s8_4.so INF_TILE_INPUT=64x64 INF_TILE_DW=64x64 INF_DW_SPLITS=2
