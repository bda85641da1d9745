#!/bin/bash
# One SQ counter pass of the projection GEMM (tools/ptab_sweep.py, the default tile only)
set -uo pipefail
OUT=gpurun_out/ptab_pmc; mkdir -p $OUT; export TMPDIR=/tmp
PTAB_VARIANTS=1 timeout -s KILL 120 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT -d $OUT/p1 -o run --output-format csv -- python3 tools/ptab_sweep.py > $OUT/p1.log 2>&1 || { echo "pass failed"; tail -5 $OUT/p1.log; exit 1; }
python3 - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/ptab_pmc/p1/**/*counter_collection.csv", recursive=True)
print(f)
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f[0])):
    if "proj_gemm" in r["Kernel_Name"]:
        acc[(r["Dispatch_Id"], r["Counter_Name"])].append(float(r["Counter_Value"]))
per = collections.defaultdict(list)
for (d, c), v in acc.items():
    per[c].append(sum(v))
for c, v in sorted(per.items()):
    print(c, f"{sum(v)/len(v):.4g}", "dispatches", len(v))
PY
