#!/bin/bash
# chain3: the single-chunk accy schedule (INF_C3_ACCY=1: both input layers in phase 0) vs the
# default, alternated: phase stamps at 4096 rays and the headline step line
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3ad.log
for v in 0 1 0 1; do
  echo "== accy $v" >> $O/r3ad.log
  if [ $v = 1 ]; then export INF_C3_ACCY=1; else unset INF_C3_ACCY; fi
  timeout -k 10 120 python tools/chain3_timing.py 4096 > $O/r3ad_t.log 2>&1 || exit 1
  grep -E "stage|fwd0|fwd4|entry ->" $O/r3ad_t.log | head -4 >> $O/r3ad.log
  timeout -k 10 200 python bench.py --only none --no-cpu-baseline --extra-batches "" > $O/r3ad_b.log 2>&1 || exit 1
  grep -o '"ms_per_step": [0-9.]*' $O/r3ad_b.log | head -1 >> $O/r3ad.log
done
