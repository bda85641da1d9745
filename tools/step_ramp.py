"""Diagnostic: how the graph-replayed headline step's time evolves from a cold start --
per 8-step replay, HIP events around each, over ~0.5 s of back-to-back replays, then again
after 1 s idle.  Shows how long the GPU takes to reach its sustained step time (what a short
timed window, e.g. 5 warmup + 20 timed steps, sees instead).

    python tools/step_ramp.py [batch] [replays] [nb] [-- bench args, e.g. --k 64 --layers 4 --hidden 128
                                                  --skip 2 --verts 20000 for config A]
"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

argv = sys.argv[1:]
rest = argv[argv.index("--") + 1:] if "--" in argv else []
pos = argv[:argv.index("--")] if "--" in argv else argv
B = int(pos[0]) if len(pos) > 0 else 4096
R = int(pos[1]) if len(pos) > 1 else 800
NB = int(pos[2]) if len(pos) > 2 else 32
sys.argv = [sys.argv[0]] + rest
args = bench.parse()
dev = torch.device("cuda", 0)
tr = bench.Trainer(args, dev, B, 0, 1, nb=NB)
tr.capture()
gm = tr.graphs[2]


def trajectory(n):
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(n)]
    torch.cuda.synchronize()
    for a, b in ev:
        tr._wrap()
        if tr.i % 2 or tr.i + tr.GRAPH_STEPS > tr.nb:
            tr.plan.set_batch_index(0)
            tr.i = 0
        a.record()
        gm.replay()
        b.record()
        tr.i += tr.GRAPH_STEPS
    torch.cuda.synchronize()
    return [a.elapsed_time(b) * 1e3 / tr.GRAPH_STEPS for a, b in ev]  # us per step


def show(tag, t):
    cum = 0.0
    marks = []
    for i, x in enumerate(t):
        cum += x * tr.GRAPH_STEPS
        if i in (0, 1, 2, 3, 5, 10, 20, 50, 100, 200, 400, 800, 1600, 3200, 6400, len(t) - 1):
            marks.append(f"#{i} @{cum / 1e3:.1f}ms {x:.2f}")
    tail = sorted(t[len(t) // 2:])[len(t) // 4]
    print(f"{tag}: us/step per replay: " + ", ".join(marks) + f"; median of 2nd half {tail:.2f}")
    # medians of consecutive windows of 100 replays (~50 ms at 4096 rays)
    w = [sorted(t[j:j + 100])[50] for j in range(0, len(t) - 99, 100)]
    print(f"   per-100-replay medians: " + " ".join(f"{x:.1f}" for x in w))


show("cold", trajectory(R))
time.sleep(1.0)
show("after 1 s idle", trajectory(R))
show("immediately again", trajectory(R // 4))
