#!/bin/bash
# chain3 phase stamps: wide tiles (16,384 = one 64-ray workgroup per CU; 65,536) and narrow (4096, 8192)
set -o pipefail
O=gpurun_out
mkdir -p $O
: > $O/r3q_c3t.log
for b in 16384 65536 4096 8192; do
  echo "== batch $b" >> $O/r3q_c3t.log
  timeout -k 10 120 python tools/chain3_timing.py $b >> $O/r3q_c3t.log 2>&1 || exit 1
done
