#!/bin/bash
# config-D chain timing (k = 4096, V = 50k table) for the default library and variants
set -o pipefail
for l in "" "$@"; do
  if [ -n "$l" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$l.so INF_ALLOW_STALE_LIB=1; else unset INF_LIB INF_ALLOW_STALE_LIB; fi
  echo "== lib ${l:-default}"
  timeout -k 10 100 python tools/chain3_timing.py 4096 4096 2>&1 | grep -v amdgpu.ids || exit 1
done
