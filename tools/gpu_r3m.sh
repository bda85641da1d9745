#!/bin/bash
# Round 3: split-K factor / tile of the parity modes' dW GEMM behind the fused fp32 chain
set -o pipefail
O=gpurun_out
: > $O/r3m_timing.log
for m in fp32 bf16x3; do
  for sp in 2 4 8; do
    echo "== $m splits $sp" >> $O/r3m_timing.log
    INF_DW_SPLITS=$sp timeout -k 10 120 python tools/chainf_timing.py $m >> $O/r3m_timing.log 2>&1 || exit 1
  done
  echo "== $m splits 4 tile 128x64" >> $O/r3m_timing.log
  INF_DW_SPLITS=4 INF_TILE_DW=128x64 timeout -k 10 120 python tools/chainf_timing.py $m >> $O/r3m_timing.log 2>&1 || exit 1
done
