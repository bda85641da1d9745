"""Diagnostic: stage times of the fp32 parity modes' fused step at config B (4096 rays):
the fused chain (chainf.hip), the dW GEMM and the update, HIP events around replays.

    python tools/chainf_timing.py [mode] [batch]      (mode fp32 | bf16x3)
Run it against variant builds with INF_LIB=<lib> INF_ALLOW_STALE_LIB=1."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

import bench
from inf_hip import STAGE_CHAIN, STAGE_DW_GEMM, STAGE_UPDATE, runtime

mode = sys.argv[1] if len(sys.argv) > 1 else "fp32"
B = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
k, H, L, s = 1024, 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, mode, "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V = 50000
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
plan.set_lr(1e-4)
b = plan.make_batch(source=src, batch=B)
for _ in range(3):
    plan.train_step(b, None, apply_adam=True)
torch.cuda.synchronize()
print("path", plan.last_step_path(), "lib", os.environ.get("INF_LIB", "default"))
for name, st, layer, batch in (("chain", STAGE_CHAIN, 0, b), ("dw", STAGE_DW_GEMM, 0, None), ("update", STAGE_UPDATE, 1, None)):
    ms = sorted(bench.time_stage(plan, st, reps=20, batch=batch, layer=layer)[0] for _ in range(3))[1]
    print(f"{name:8s} {ms * 1e3:8.2f} us", flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(20):
    plan.train_step(b, None, apply_adam=True)
e1.record()
torch.cuda.synchronize()
print(f"step     {e0.elapsed_time(e1) / 20 * 1e3:8.2f} us (eager)")
