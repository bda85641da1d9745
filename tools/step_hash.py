"""Bitwise fingerprint of one fused training step (gradients, predictions, loss sum) at a
given shape -- run it under two libraries (INF_LIB=...) to check that a schedule change
left the arithmetic untouched.

    python tools/step_hash.py [batch] [k]
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from inf_hip import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
H, L, s, V = 256, 8, 4, 20000
rng = np.random.default_rng(3)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.02).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
pred = torch.empty((B, 3), device="cuda")
plan.train_step(plan.make_batch(source=src, batch=B), pred, apply_adam=False)
torch.cuda.synchronize()
h = hashlib.sha256()
for t in (plan.grads, pred):
    h.update(t.cpu().numpy().tobytes())
print(f"B={B} k={k} path={plan.last_step_path()} loss={plan.read_ctrl()['loss_sum']!r} sha={h.hexdigest()[:20]}")
