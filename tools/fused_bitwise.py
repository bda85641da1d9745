"""Diagnostic: separate vs INF_FUSED_UPDATE update over 3 bf16 chain3 steps of config B;
prints which arrays differ (tests/test_gpu_kernels.py::test_fused_update_bitwise)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "intrinsic-neural-fields_amd"), os.path.join(ROOT, "tests"), ROOT]
import numpy as np
import torch

from test_gpu_kernels import CFG, make_plan, rt

rng = np.random.default_rng(5)
k, H, L, s = CFG["B"]
V, B = 3000, 4096
E = rng.standard_normal((V, k)).astype(np.float32)
E /= (E.max(0) - E.min(0))
src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                     torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                     torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
out = {}
for tag in ("separate", "fused", "separate2"):
    if tag == "fused":
        os.environ["INF_FUSED_UPDATE"] = "1"
    else:
        os.environ.pop("INF_FUSED_UPDATE", None)
    plan, params, w = make_plan("B", mode="bf16", max_batch=B, adam=True)
    plan.set_lr(1e-3)
    b = plan.make_batch(source=src, batch=B)
    for _ in range(3):
        plan.train_step(b, None, apply_adam=True)
    torch.cuda.synchronize()
    out[tag] = [t.cpu().numpy().copy() for t in (params, plan.exp_avg, plan.exp_avg_sq)]
for other in ("fused", "separate2"):
    for name, a_, b_ in zip(("params", "m", "v"), out["separate"], out[other]):
        d = a_ != b_
        print(other, name, "differs at", int(d.sum()), "of", d.size, "first", np.flatnonzero(d)[:5])
