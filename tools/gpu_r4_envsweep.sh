#!/bin/bash
# Headline step under environment variants, alternated: bash tools/gpu_r4_envsweep.sh "ENV=1 ENV2=2" "..."
# (the first entry "-" is the default).  One line per run: variant, ms per step, stage times.
set -o pipefail
for rep in 1 2; do
  for v in "$@"; do
    env_args=""
    [ "$v" != "-" ] && env_args="$v"
    out=$(env $env_args timeout -k 10 150 python bench.py --steps 100 --warmup 20 --only none --no-cpu-baseline --extra-batches "" 2>/dev/null | grep '^{') || { echo "FAILED $v"; exit 1; }
    echo "$out" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$v', round(d['ms_per_step']*1e3,2), {k: round(x['ms']*1e3,2) for k,x in d['stages'].items()})"
  done
done
