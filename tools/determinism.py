"""Diagnostic: run the same training steps twice from the same state and compare the
parameters bitwise (any difference = a race or an order-dependent reduction)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from inf_hip import runtime

mode = sys.argv[1] if len(sys.argv) > 1 else "fp32"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
k, H, L, s = 1024, 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
p0 = (rng.standard_normal(P) * 0.03).astype(np.float32)
V, N = 3000, 8 * B
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
vids = torch.from_numpy(rng.integers(0, V, (N, 3))).cuda()
bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda()
rgb = torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda()
outs = []
for rep in range(3):
    params = torch.from_numpy(p0.copy()).cuda()
    plan = runtime.Plan(k, H, L, s, mode, "L2", B, params, grads=torch.zeros_like(params),
                        exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
    plan.set_lr(1e-4)
    src = runtime.RaySource(E, vids, bary, rgb)
    for step in range(3):
        plan.train_step(plan.make_batch(source=src, offset=step * B, batch=B), None, apply_adam=True)
    torch.cuda.synchronize()
    outs.append((params.cpu().numpy().copy(), plan.grads.cpu().numpy().copy()))
for r in range(1, len(outs)):
    dp = np.abs(outs[r][0] - outs[0][0])
    dg = np.abs(outs[r][1] - outs[0][1])
    print(f"{mode} B={B} rep {r}: params differ at {int((dp > 0).sum())} (max {dp.max():.3e}), "
          f"grads differ at {int((dg > 0).sum())} (max {dg.max():.3e})")
