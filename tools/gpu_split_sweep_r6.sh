#!/bin/bash
# Round 6: the driver's bench line on this box, then the dW split-K count per config
# (INF_DW_SPLITS) on the headline leg of configs A, R and B (tools/ only; run via gpurun).
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $O/bench.log 2>&1 || exit 1
H="--steps 80 --warmup 8 --no-render --no-cpu-baseline --no-config-d --extra-batches= --only none"
A="--k 64 --layers 4 --hidden 128 --skip 2 --verts 20000"
R="--k 1023 --layers 6 --hidden 128 --skip 3 --loss L1"
for cfg in A R B; do
  case $cfg in A) X=$A;; R) X=$R;; B) X="";; esac
  for s in def 2 4 8 16; do
    if [ $s = def ]; then E=""; else E="INF_DW_SPLITS=$s"; fi
    env $E timeout -k 10 120 python3 bench.py $H $X > $O/split_${cfg}_$s.log 2>&1 || exit 1
    python3 -c "import json,sys; d=json.loads([l for l in open('$O/split_${cfg}_$s.log') if l.startswith('{')][-1]); print('$cfg', '$s', round(d['ms_per_step']*1e3,2), {k: round(v['ms']*1e3,2) for k,v in d['stages'].items()})"
  done
done
