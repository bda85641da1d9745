#!/bin/bash
# bf16x3 split-operand dW: split-K 2 (default) vs 4, stage timing and the graph-replayed line
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3z.log
for sp in 2 4 2 4; do
  echo "== splits $sp" >> $O/r3z.log
  INF_DW_SPLITS=$sp timeout -k 10 120 python tools/chainf_timing.py bf16x3 2>&1 | grep -E "dw|update|step" >> $O/r3z.log || exit 1
done
