# SQ counter pass + FETCH/WRITE passes of the 65,536-ray step (fgemm and the wide chain),
# one rocprofv3 run per pass, kernel trace only beside the counters.
set -euo pipefail
export TMPDIR=/tmp
OUT=gpurun_out/pmc_large
mkdir -p "$OUT"
ARGS=(--steps 10 --warmup 3 --only large --no-cpu-baseline --extra-batches 65536)
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d "$OUT/sq" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/sq.log" 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/fetch.log" 2>&1
timeout -s KILL 180 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv -- python3 bench.py "${ARGS[@]}" > "$OUT/write.log" 2>&1
