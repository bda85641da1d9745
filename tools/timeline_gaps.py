"""Diagnostic: per-kernel durations and the idle gaps between consecutive kernels of a
rocprofv3 kernel trace, grouped by (previous kernel -> next kernel).  Unlike step_gaps.py it
assumes no step shape, so it reads any path's timeline (the large-batch step's chain3 ->
fgemm -> update, config D's chunked chain -> LGF, ...).

    python tools/timeline_gaps.py <run_kernel_trace.csv> [min_count]
"""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", n)
    if m:
        return m.group(1) + ("<" + m.group(2)[1:40] + ">" if m.group(2) else "")
    return n[:40]


rows = list(csv.DictReader(open(sys.argv[1])))
min_count = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
dur = defaultdict(list)
gap = defaultdict(list)
for i, (n, s, e) in enumerate(ev):
    dur[n].append(e - s)
    if i + 1 < len(ev):
        gap[(n, ev[i + 1][0])].append(ev[i + 1][1] - e)


def med(v):
    return sorted(v)[len(v) // 2] / 1e3


print("kernel durations (count, median us):")
for n, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
    if len(v) >= min_count:
        print(f"  {len(v):5d}  {med(v):9.2f}  {n}")
print("gaps between consecutive kernels (count, median us, min us):")
for (a, b), v in sorted(gap.items(), key=lambda kv: -len(kv[1])):
    if len(v) >= min_count:
        print(f"  {len(v):5d}  {med(v):7.2f}  {min(v) / 1e3:7.2f}  {a} -> {b}")
