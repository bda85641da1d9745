#!/bin/bash
# Round-2 profiles: kernel trace + FETCH_SIZE + WRITE_SIZE passes (each alone, own limit) of
# the headline step, the render frame and config D.  Run on the GPU box via gpurun.
set -uo pipefail
for spec in "step:--only none" "render:--only render" "configD:--only configD"; do
  tag=${spec%%:*}; args=${spec#*:}
  PROF_TAG=bf16_B4096 bash tools/profile.sh r02_$tag --steps 40 --warmup 10 --no-cpu-baseline --extra-batches "" $args || { echo "profile $tag failed"; exit 1; }
  echo "profile $tag done"
done
