"""Diagnostic: per-kernel durations and the gaps between them inside graph-replayed
training steps, from a rocprofv3 kernel trace (tools/profile.sh ... trace/run_kernel_trace.csv).

    python tools/step_gaps.py gpurun_out/prof_<tag>/trace/run_kernel_trace.csv
"""
import csv
import sys
from collections import defaultdict


def short(n):
    for k in ("chain3_kernel", "lgemm_kernel", "update_kernel", "ctrl_advance_kernel", "chain_kernel", "gemm_nt_kernel",
              "gather_kernel"):
        if k in n:
            return k
    return n[:30]


rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
# training steps: chain3 -> lgemm -> update launched back to back
dur = defaultdict(list)
gaps = defaultdict(list)
steps = []
for i in range(len(ev) - 2):
    a, b, c = ev[i], ev[i + 1], ev[i + 2]
    if a[0] == "chain3_kernel" and b[0] == "lgemm_kernel" and c[0] == "update_kernel":
        steps.append(i)
        dur["chain3"].append(a[2] - a[1])
        dur["lgemm"].append(b[2] - b[1])
        dur["update"].append(c[2] - c[1])
        gaps["chain3->lgemm"].append(b[1] - a[2])
        gaps["lgemm->update"].append(c[1] - b[2])
        if i + 3 < len(ev):
            gaps["update->next"].append(ev[i + 3][1] - c[2])
            dur["next:" + ev[i + 3][0]].append(0)
med = lambda v: sorted(v)[len(v) // 2] / 1e3
print(f"{len(steps)} steps")
for k, v in dur.items():
    if not k.startswith("next:"):
        print(f"  {k:8s} median {med(v):7.2f} us  min {min(v) / 1e3:7.2f}")
for k, v in gaps.items():
    print(f"  gap {k:15s} median {med(v):6.2f} us")
nxt = {k[5:]: len(v) for k, v in dur.items() if k.startswith("next:")}
print("  kernel after update:", nxt)
