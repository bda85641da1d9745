"""Aggregates tools/gpu_step_variants.sh logs: mean / min step time per library."""
import collections
import re
import sys

d = collections.defaultdict(list)
cur = None
for path in sys.argv[1:]:
    for line in open(path):
        if line.startswith("=="):
            cur = line.split()[-1]
        m = re.search(r"in-kernel gather ([\d.]+).*once ([\d.]+)", line)
        if m:
            d[cur].append((float(m.group(1)), float(m.group(2))))
for k, v in d.items():
    a = [x for x, _ in v]
    b = [y for _, y in v]
    print(f"{k:8s} n={len(v)} step mean {sum(a) / len(a):.2f} min {min(a):.1f}  pre-gathered mean {sum(b) / len(b):.2f}")
