#!/bin/bash
# chainf gather in one round (CF_GR=8, fragment prologue after it) vs two (default)
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3aa.log
for v in default gr8 default gr8; do
  if [ $v = default ]; then L=intrinsic-neural-fields_amd/inf_hip/libinf_hip.so; else L=intrinsic-neural-fields_amd/inf_hip/libinf_hip_$v.so; fi
  for m in bf16x3 fp32; do
    echo "== $v $m" >> $O/r3aa.log
    INF_LIB=$L INF_ALLOW_STALE_LIB=1 timeout -k 10 120 python tools/chainf_timing.py $m 2>&1 | grep -E "chain |step" >> $O/r3aa.log || exit 1
  done
done
