"""Diagnostic: what a short timed window pays on top of the settled step -- the time from
the start event to the first kernel (host submission of the first graph replay after a
synchronize) and the idle gap at every graph-replay boundary -- for graphs of 1, 4, 8, 16
and 32 steps of the headline Trainer (bench.py), after the clock settle.

    python tools/launch_window.py [batch]
"""
import os
import statistics as st
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402

import bench  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
sys.argv = [sys.argv[0]]
args = bench.parse()
dev = torch.device("cuda", 0)
tr = bench.Trainer(args, dev, B, 0, 1, nb=64)
tr.capture()
graphs = {}
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    for n in (1, 4, 8, 16, 32):
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s):
            tr._steps(n)
        graphs[n] = g
torch.cuda.current_stream().wait_stream(s)
torch.cuda.synchronize()


def replay(n, reps):
    for _ in range(reps):
        tr.plan.set_batch_index(0)
        graphs[n].replay()


def window(fn):
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1e3


# settle the clocks
t0 = time.perf_counter()
while time.perf_counter() - t0 < 0.3:
    replay(32, 4)
torch.cuda.synchronize()
steady = st.median(window(lambda: replay(32, 8)) / 256 for _ in range(5))
print(f"steady step (32-step graphs, 8 back to back): {steady:.2f} us")
print(f"empty window: {st.median(window(lambda: None) for _ in range(20)):.2f} us")
# set_batch_index is a fill kernel: time it alone
fill = st.median(window(lambda: tr.plan.set_batch_index(0)) for _ in range(20))
print(f"window with one set_batch_index fill: {fill:.2f} us")
for n in (1, 4, 8, 16, 32):
    w1 = st.median(window(lambda: graphs[n].replay()) for _ in range(20))
    w10 = st.median(window(lambda: [graphs[n].replay() for _ in range(10)]) for _ in range(5))
    per_replay = (w10 - w1) / 9
    t_host = []
    for _ in range(20):
        torch.cuda.synchronize()
        a = time.perf_counter()
        graphs[n].replay()
        t_host.append((time.perf_counter() - a) * 1e6)
        torch.cuda.synchronize()
    print(f"{n:2d}-step graph: one replay in a window {w1:8.1f} us (start overhead {w1 - n * steady:6.1f}); "
          f"each further replay {per_replay:8.1f} us (boundary {per_replay - n * steady:5.1f}); "
          f"host replay() call {st.median(t_host):6.1f} us")
