#!/bin/bash
# Runs GPU steps in order, each under its own time limit, output to gpurun_out/<name>.log:
#   bash tools/gpu_run_steps.sh "name|seconds|command" ...
# A step that fails normally (exit 1: a failed test) does not stop the rest; a time limit,
# abort, segfault or any signal exit (>= 124) ends the script there (no GPU work after it).
mkdir -p gpurun_out
for spec in "$@"; do
  name=${spec%%|*}
  rest=${spec#*|}
  secs=${rest%%|*}
  cmd=${rest#*|}
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "[step] $name rc=$rc $(( $(date +%s) - start ))s"
  if [ $rc -ge 124 ]; then
    echo "[step] $name ended abnormally (rc=$rc): stopping"
    exit $rc
  fi
done
