#!/bin/bash
# PMC passes over a short bench run (stage kernels included), one rocprofv3 run per pass.
set -uo pipefail
OUT=gpurun_out/pmc_$1; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
ARGS=(--steps 20 --warmup 5 --no-render --no-cpu-baseline --extra-batches "")
i=0
for pmc in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $pmc -d "$OUT/p$i" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/p$i.log" 2>&1 || { echo "pass $i ($pmc) failed"; exit 1; }
done
