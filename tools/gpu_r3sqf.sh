#!/bin/bash
# One SQ counter pass over the bf16x3 parity mode's step (chainf / lgemm SPLIT / update)
set -o pipefail
O=gpurun_out/pmc_r3sqf
mkdir -p $O
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS -d $O/sq -o run --output-format csv -- python3 bench.py --mode bf16x3 --steps 20 --warmup 5 --only none --no-cpu-baseline --extra-batches "" > $O/sq.log 2>&1
