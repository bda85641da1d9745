#!/bin/bash
# Round 3 session-3: the full default bench line, the step profile (kernel trace + FETCH /
# WRITE passes), stage timing of the parity modes and the 65,536-ray step.
set -o pipefail
O=gpurun_out
mkdir -p $O
timeout -k 10 700 python bench.py > $O/r3p_bench.log 2>&1 || exit 1
PROF_TAG=bf16_B4096 timeout -k 10 900 bash tools/profile.sh r03_step --steps 40 --warmup 10 --no-cpu-baseline --extra-batches "" --only none || exit 1
for m in fp32 bf16x3; do
  timeout -k 10 120 python tools/chainf_timing.py $m > $O/r3p_chainf_$m.log 2>&1 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_r03_65k -o run --output-format csv -- python3 bench.py --batch 65536 --steps 16 --warmup 4 --extra-batches "" --only none --no-cpu-baseline > $O/r3p_65k.log 2>&1
