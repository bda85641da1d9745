#!/bin/bash
# Round-2 render profiles after the projected-table path: kernel trace + FETCH_SIZE +
# WRITE_SIZE passes of bench.py's render section (feature-gather frames, projected frames,
# the projection GEMM).  Run on the GPU box via gpurun.
set -uo pipefail
PROF_TAG=bf16_render bash tools/profile.sh r02_render_proj --steps 20 --warmup 5 --no-cpu-baseline --extra-batches "" --only render || { echo "profile failed"; exit 1; }
echo "profile done"
