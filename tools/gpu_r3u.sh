#!/bin/bash
# Round 3 profiles of the render frame on its hand-written projection GEMM (ptab.hip) and of
# config D: kernel trace + FETCH_SIZE + WRITE_SIZE passes (tools/profile.sh)
set -o pipefail
PROF_TAG=bf16_render timeout -k 10 900 bash tools/profile.sh r03_render --steps 20 --warmup 5 --no-cpu-baseline --extra-batches "" --only render || exit 1
PROF_TAG=bf16_D4096 timeout -k 10 900 bash tools/profile.sh r03_configD --steps 20 --warmup 5 --no-cpu-baseline --extra-batches "" --only configD
