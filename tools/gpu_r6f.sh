#!/bin/bash
# Round 6: kernel trace of bench.py's render leg (every rprojw / projection launch in order:
# main frames, pixel-coherent variant, 100 % random variant), and the render ids tool warm.
set -o pipefail
O=gpurun_out/${1:-r6f}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr -o run --output-format csv -- python3 tools/render_step.py > $O/render_step.log 2>&1 || exit 1
python3 - $O <<'PY'
import csv, glob, sys
O = sys.argv[1]
f = glob.glob(f"{O}/tr/**/*kernel_trace.csv", recursive=True)[0]
rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
seq = []
for r in rows:
    n = r["Kernel_Name"]
    tag = "rprojw" if "rprojw" in n else "proj" if "proj_gemm" in n else "fill" if "FillFunctor" in n else None
    if tag:
        seq.append((tag, (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3, int(r["Start_Timestamp"])))
prev = None
for tag, us, t0 in seq:
    gap = (t0 - prev) / 1e3 if prev else 0
    print(f"{tag:7s} {us:9.1f} us   (+{gap:8.1f} us since previous start)")
    prev = t0
PY
