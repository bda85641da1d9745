"""Print the headline fields of a bench.py JSON line (the last '{' line of a log)."""
import json
import sys

line = [x for x in open(sys.argv[1]) if x.startswith("{")][-1]
d = json.loads(line)
print("value", round(d["value"] / 1e6, 2), "M rays/s", "ms/step", round(d["ms_per_step"] * 1e3, 1), "us")
print("stages", {k: round(v["ms"] * 1e3, 1) for k, v in d["stages"].items()})
for key in ("config_D", "render", "secondary", "large_batch", "extrinsic_rff"):
    v = d.get(key)
    if v:
        print(key, json.dumps(v)[:600])
