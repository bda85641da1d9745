#!/bin/bash
# Kernel-trace + PMC profiles of bench.py (run on the GPU box via gpurun).
#   tools/profile.sh <tag> [bench args...]
# Writes gpurun_out/prof_<tag>/{trace,fetch,write}/ and gpurun_out/prof_<tag>/summary.json
# Each rocprofv3 pass runs alone under its own time limit; PMC passes use --kernel-trace only.
set -euo pipefail
TAG=${1:?tag}; shift
ARGS=("$@")
[ ${#ARGS[@]} -eq 0 ] && ARGS=(--steps 40 --warmup 10 --no-render --no-cpu-baseline --extra-batches "")
OUT=gpurun_out/prof_$TAG
mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/trace.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/fetch.log" 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/write.log" 2>&1
python3 tools/summarize_prof.py "$OUT" "${PROF_TAG:-bf16_B4096}" > "$OUT/summary.json"
