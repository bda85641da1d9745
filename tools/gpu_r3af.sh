#!/bin/bash
# steps per replayed graph (8 default vs 32): the headline line, alternated
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3af.log
for g in 8 32 8 32; do
  echo "== graph steps $g" >> $O/r3af.log
  INF_GRAPH_STEPS=$g timeout -k 10 200 python bench.py --only none --no-cpu-baseline --extra-batches "" > $O/r3af_b.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/r3af_b.log | head -1 >> $O/r3af.log
done
