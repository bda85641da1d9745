#!/bin/bash
# Times diagnostic builds of the training step side by side (run on the GPU box via gpurun):
#   make -C intrinsic-neural-fields_amd/csrc BUILD=build_d_X OUT=../inf_hip/libinf_hip_X.so EXTRA="-D..."
#   bash tools/gpu_step_variants.sh X Y ...      (the default library first)
set -o pipefail
for l in "" "$@"; do
  if [ -n "$l" ]; then export INF_LIB=$PWD/intrinsic-neural-fields_amd/inf_hip/libinf_hip_$l.so INF_ALLOW_STALE_LIB=1; else unset INF_LIB INF_ALLOW_STALE_LIB; fi
  echo "== lib ${l:-default}"
  timeout -k 10 100 python tools/xslot_gain.py 2>&1 | grep -v amdgpu.ids || exit 1
done
