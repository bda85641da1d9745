"""Diagnostic: per-step timeline of one bench leg's LAST n steps in a rocprofv3 kernel trace
(the timed window; a leg is identified by its chain kernel's template name): step period
(chain start to next chain start), each kernel's duration and the idle gaps of the step.

    python tools/leg_window.py <run_kernel_trace.csv[.gz]> <chain-kernel substring> [n]
"""
import csv
import gzip
import re
import statistics as st
import sys


def short(n):
    m = re.search(r"(\w+_kernel)(<[^(]*>)?", n)
    return (m.group(1) + (m.group(2) or "")) if m else n[:50]


path, key = sys.argv[1], sys.argv[2]
n = int(sys.argv[3]) if len(sys.argv) > 3 else 20
fh = gzip.open(path, "rt") if path.endswith(".gz") else open(path)
rows = sorted(csv.DictReader(fh), key=lambda r: int(r["Start_Timestamp"]))
ev = [(short(r["Kernel_Name"]), int(r["Start_Timestamp"]), int(r["End_Timestamp"])) for r in rows]
idx = [i for i, e in enumerate(ev) if key in e[0]]
last = idx[-(n + 1):]  # n steps: n periods between n + 1 chain starts
per = {}
gaps = []
periods = []
for a, b in zip(last[:-1], last[1:]):
    periods.append((ev[b][1] - ev[a][1]) / 1e3)
    for j in range(a, b):
        per.setdefault(ev[j][0], []).append((ev[j][2] - ev[j][1]) / 1e3)
        gaps.append((ev[j][0], ev[j + 1][0], (ev[j + 1][1] - ev[j][2]) / 1e3))
print(f"{len(periods)} steps of {key}: period median {st.median(periods):.2f} us, mean {st.mean(periods):.2f}, "
      f"min {min(periods):.2f}, max {max(periods):.2f}")
print("  periods:", " ".join(f"{p:.1f}" for p in periods))
for k, v in per.items():
    print(f"  {len(v):4d} x {k[:70]:70s} median {st.median(v):7.2f}  mean {st.mean(v):7.2f}  max {max(v):7.2f}")
g = {}
for a, b, x in gaps:
    g.setdefault((a[:30], b[:30]), []).append(x)
for (a, b), v in g.items():
    print(f"  gap {a} -> {b}: {len(v)} median {st.median(v):.2f} max {max(v):.2f} sum/step {sum(v) / len(periods):.2f}")
