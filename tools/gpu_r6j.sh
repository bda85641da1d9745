#!/bin/bash
# Round 6: rocprofv3 kernel trace + PMC traffic passes of the headline leg (the driver's
# --steps 20 --warmup 5), and chain3's per-phase stamps.
set -o pipefail
O=gpurun_out/${1:-r6j}
mkdir -p $O
PROF_TAG=bf16_B4096 bash tools/profile.sh r6j_headline --steps 20 --warmup 5 --only none --no-render --no-cpu-baseline --no-config-d --extra-batches= || exit 1
mv gpurun_out/prof_r6j_headline $O/prof_headline
python3 -c "import json; d=json.load(open('$O/prof_headline/summary.json')); print(d['bench_traffic']); print({k: round(v['avg_us'],2) for k,v in d['kernels'].items() if v['calls'] > 100})"
timeout -k 10 120 python3 tools/chain3_timing.py > $O/chain3_timing.log 2>&1 || exit 1
tail -30 $O/chain3_timing.log
