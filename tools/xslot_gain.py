"""Diagnostic: the config-B training step (graph-replayed) with the in-kernel gather vs
its rows pre-gathered ONCE into a slot (XSLOT, no gather in the step at all): the upper
bound of moving the gather off the step's critical path.

    python tools/xslot_gain.py [batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import numpy as np
import torch

from inf_hip import runtime

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k, H, L, s = 1024, 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V, N = 50000, 400 * B
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
perm = torch.randperm(N, device="cuda")
plan.set_lr(1e-5)
b = plan.make_batch(source=src, ray_idx=perm, batch=B, offset_from_ctrl=True)
plan.set_batch_index(3)
plan.set_prefetch_index(3)
assert plan.prefetch(b, 0)
for _ in range(5):
    plan.train_step(b, None, apply_adam=True)
    plan.train_step(b, None, apply_adam=True, xslot=0)
torch.cuda.synchronize()


def timed(xs, b=b, advance=False):
    g = torch.cuda.CUDAGraph()
    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        with torch.cuda.graph(g, stream=s_):
            for _ in range(8):
                plan.train_step(b, None, apply_adam=True, xslot=xs, advance=advance)
    torch.cuda.current_stream().wait_stream(s_)
    for _ in range(3):
        g.replay()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(40):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 320 * 1e3


for rep in range(2):
    plan.set_batch_index(0)
    t_g = timed(None, b, True)
    plan.set_batch_index(3)
    t_x = timed(0)
    print(f"B={B}: in-kernel gather {t_g:.1f} us/step, pre-gathered once {t_x:.1f} us/step")
