"""Diagnostic: the wall-clock stamps of chain4.hip (the large-batch chain, 128-ray
workgroups of four waves) for wave 0 of the first and the last workgroup, phase by phase,
plus the stage's HIP-event time.

    python tools/chain4_timing.py [batch] [k]

chain4 is the default above 8192 rays (INF_CHAIN4=0: chain3 wide tiles).
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

os.environ.setdefault("INF_CHAIN4", "1")  # (the caller may set INF_CHAIN4=0: chain3 wide)

from inf_hip import STAGE_CHAIN, lib, runtime

B = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
k = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
H, L, s = 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
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
print("path", plan.last_step_path())
ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(10):
    plan.run_stage(STAGE_CHAIN, 0, b)
ev1.record()
torch.cuda.synchronize()
print(f"chain stage: {ev0.elapsed_time(ev1) / 10 * 1e3:.1f} us (B={B})")

NS = 256
stamps = torch.zeros(2 * NS, dtype=torch.int64, device="cuda")
lib.inf_debug_timing(plan.handle, ctypes.c_void_p(stamps.data_ptr()), 1)
for _ in range(3):
    stamps.zero_()
    plan.run_stage(STAGE_CHAIN, 0, b)
    torch.cuda.synchronize()
lib.inf_debug_timing(plan.handle, None, 0)
nchunk = (-(-k // 128) * 128) // 64
labels = ["entry", "records"]
for c in range(nchunk):
    labels += [f"chunk{c} rows in, X written", f"chunk{c} MFMAs, X^T, DMA"]
labels += ["epi0 B1", "epi0 B2", "epi0 Y^T copy"]
for l in range(1, L - 2):
    labels += [f"fwd{l} MFMAs", f"epi{l} B1", f"epi{l} B2", f"epi{l} Y^T copy"]
labels += [f"fwd{L - 2} MFMAs", "head Bh (partials)", "head B2", "head dZ^T copy"]
for l in range(L - 2, 0, -1):
    labels += [f"bwd{l} MFMAs", f"bwd{l} B1", f"bwd{l} B2", f"bwd{l} dZ^T copy"]
labels += ["end"]
st = stamps.cpu().numpy().reshape(2, NS).astype(np.float64) * 10.0 / 1e3  # 100 MHz -> us
for w, name in enumerate(("first", "last")):
    t = st[w]
    n = int((t > 0).sum())
    print(f"workgroup {name}: {n} stamps, entry -> end {t[n - 1] - t[0]:.2f} us")
    for i in range(1, min(n, len(labels))):
        print(f"   {labels[i]:24s} +{t[i] - t[i - 1]:7.2f}  @{t[i] - t[0]:8.2f}")
