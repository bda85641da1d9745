#!/bin/bash
# bf16x3 / fp32 parity modes behind the fused fp32 chain: dW split-K factor x tile sweep
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3t_sweep.log
for m in bf16x3 fp32; do
  for sp in 2 4 8; do
    for t in 128x128 128x64 64x64; do
      echo "== $m splits $sp tile $t" >> $O/r3t_sweep.log
      INF_DW_SPLITS=$sp INF_TILE_DW=$t timeout -k 10 120 python tools/chainf_timing.py $m >> $O/r3t_sweep.log 2>&1 || exit 1
    done
  done
done
