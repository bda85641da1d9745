#!/bin/bash
# Late round-2 refresh of the headline step's profiles (kernel trace + FETCH_SIZE +
# WRITE_SIZE passes) after the chain3 / render epilogue changes.  Run via gpurun.
set -uo pipefail
PROF_TAG=bf16_B4096 bash tools/profile.sh r02_step_late --steps 40 --warmup 10 --no-cpu-baseline --extra-batches "" --only none || { echo "profile failed"; exit 1; }
echo "profile done"
