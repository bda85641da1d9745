#!/bin/bash
# render slice variants (GPU box): fused LDS-ring chain vs layered GEMMs
set -uo pipefail
for v in "" "INF_NO_CHAIN=1"; do echo "== $v"; env $v timeout -k 10 120 python -u tools/render_step.py 2>/dev/null | grep '^{' | cut -c1-100 || exit 1; done
export TMPDIR=/tmp
INF_NO_CHAIN=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_render_layered -o run --output-format csv -- python3 tools/render_step.py > /dev/null 2>&1
