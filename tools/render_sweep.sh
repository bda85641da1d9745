#!/bin/bash
# render slice + large-batch step under library variants (GPU box): tools/render_sweep.sh [lib ...]
set -uo pipefail
L=intrinsic-neural-fields_amd/inf_hip
for lib in "$L/libinf_hip.so" "$@"; do
  echo "== $lib"
  INF_LIB=$lib timeout -k 10 120 python -u tools/render_step.py 2>/dev/null | grep '^{' | cut -c1-100 || exit 1
  INF_LIB=$lib timeout -k 10 120 python -u bench.py --batch 65536 --steps 20 --warmup 3 --no-render --no-cpu-baseline --extra-batches "" 2>/dev/null | grep '^{' | cut -c1-160 || exit 1
done
