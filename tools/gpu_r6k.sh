#!/bin/bash
# Round 6: the N > 1 bench path rehearsed -- world 1 over RCCL (all-reduce captured in the
# step graphs, every step shape) and world 2 over gloo (two ranks sharing the GPU).
set -o pipefail
O=gpurun_out/${1:-r6k}
mkdir -p $O
bash tools/gpu_dp1.sh --steps 40 --warmup 8 > $O/dp1.log 2>&1 || { tail -20 $O/dp1.log; exit 1; }
grep '^{' $O/dp1.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('dp1', d['summary'].get('dp_us'), d['summary']['B_us'], d['config'])"
bash tools/gpu_bench_world2_gloo.sh --no-render --no-cpu-baseline --no-config-d --extra-batches= > $O/w2.log 2>&1 || { tail -30 $O/w2.log; exit 1; }
grep '^{' $O/w2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('w2', d['summary'].get('dp_us'), d['summary']['B_us'], d['n_gpus'], d['config'])"
