#!/bin/bash
# bf16x3 split-operand dW: rows per block (64 / 32) x split-K (2 / 4), stage timing
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3ac.log
for rep in 1 2; do
for bm in 64 32; do
  for sp in 2 4; do
    echo "== bm $bm splits $sp" >> $O/r3ac.log
    INF_SPLIT_LGEMM_BM=$bm INF_DW_SPLITS=$sp timeout -k 10 120 python tools/chainf_timing.py bf16x3 2>&1 | grep -E "dw|update" >> $O/r3ac.log || exit 1
  done
done
done
