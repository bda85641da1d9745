#!/bin/bash
# wide chain3 tiles: chunk-gather rounds (C3_GRX_WIDE 1 = default vs 2), phase stamps at
# 16,384 rays and the 65,536-ray step
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3v.log
for v in default g2 default g2; do
  if [ $v = default ]; then L=intrinsic-neural-fields_amd/inf_hip/libinf_hip.so; else L=intrinsic-neural-fields_amd/inf_hip/libinf_hip_$v.so; fi
  echo "== $v" >> $O/r3v.log
  INF_LIB=$L INF_ALLOW_STALE_LIB=1 timeout -k 10 120 python tools/chain3_timing.py 16384 > $O/r3v_t.log 2>&1 || exit 1
  grep -E "stage|fwd0|entry ->" $O/r3v_t.log | head -3 >> $O/r3v.log
  INF_LIB=$L INF_ALLOW_STALE_LIB=1 timeout -k 10 200 python bench.py --batch 65536 --steps 20 --warmup 5 --only none --no-cpu-baseline --extra-batches "" > $O/r3v_b.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/r3v_b.log | head -1 >> $O/r3v.log
done
