#!/bin/bash
# Round 3: where the fused fp32 chain's time goes -- stage times at config B for the
# default build (fp32 and bf16x3 modes) and diagnostic builds (no fragment loads, no
# epilogues, ring depth 2)
set -o pipefail
O=gpurun_out
L=intrinsic-neural-fields_amd/inf_hip
timeout -k 10 120 python tools/chainf_timing.py fp32 > $O/r3k_timing.log 2>&1 &&
timeout -k 10 120 python tools/chainf_timing.py bf16x3 >> $O/r3k_timing.log 2>&1 &&
for v in noepi; do
  INF_LIB=$L/libinf_hip_$v.so INF_ALLOW_STALE_LIB=1 timeout -k 10 120 python tools/chainf_timing.py fp32 >> $O/r3k_timing.log 2>&1 || exit 1
done
