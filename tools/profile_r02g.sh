#!/bin/bash
# Round-2 profiles after the write-through chain images of the headline step (kernel trace + FETCH_SIZE + WRITE_SIZE
# passes) and the in-graph gaps between its launches.  Run via gpurun.
set -uo pipefail
PROF_TAG=bf16_B4096 bash tools/profile.sh r02_step_sc1 --steps 40 --warmup 10 --no-cpu-baseline --extra-batches "" --only none || { echo "profile failed"; exit 1; }
python3 tools/step_gaps.py gpurun_out/prof_r02_step_sc1/trace/run_kernel_trace.csv > gpurun_out/prof_r02_step_sc1/gaps.txt 2>&1
echo "profile done"
