#!/bin/bash
# Round-2 profiles at the final HEAD: kernel trace + FETCH_SIZE + WRITE_SIZE passes (each
# alone, own limit) of the headline step, the render frame and config D.  Run via gpurun.
set -uo pipefail
for spec in "step:--only none" "render:--only render" "configD:--only configD"; do
  tag=${spec%%:*}; args=${spec#*:}
  PROF_TAG=bf16_B4096 bash tools/profile.sh r02f_$tag --steps 40 --warmup 10 --no-cpu-baseline --extra-batches "" $args || { echo "profile $tag failed"; exit 1; }
  echo "profile $tag done"
done
python3 tools/step_gaps.py gpurun_out/prof_r02f_step/trace/run_kernel_trace.csv > gpurun_out/prof_r02f_step/gaps.txt 2>&1
