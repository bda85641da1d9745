"""Diagnostic: per-step wall-clock stamps of the fused bf16 chain (inf_debug_timing) for
the first and the last workgroup, aggregated per phase, plus the chain stage's event time.

    python tools/chain_timing.py [batch] [k] [hidden] [layers] [skip]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from inf_hip import lib, runtime, STAGE_CHAIN

B, k, H, L, s = [int(x) for x in (sys.argv[1:] + ["4096", "1024", "256", "8", "4"][len(sys.argv) - 1:])][:5]
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V, N = 50000, B
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
plan.set_lr(1e-4)
b = plan.make_batch(source=src, batch=B)
for _ in range(3):
    plan.train_step(b, None, apply_adam=True)
torch.cuda.synchronize()

# phase table (mirrors run_chain in plan.hip): (name, steps)
kp = (k + 127) // 128 * 128
bk = 64 if B <= 8192 else 32
phases = []
for l in range(L - 1):
    if l == 0:
        phases.append(("fwd0 X", kp // bk))
    elif l == s:
        phases += [(f"fwd{l} h", H // bk), (f"fwd{l} X", kp // bk)]
    else:
        phases.append((f"fwd{l}", H // bk))
for l in range(L - 2, 0, -1):
    phases.append((f"bwd{l}", H // bk))
nsteps = sum(n for _, n in phases)

ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(20):
    plan.run_stage(STAGE_CHAIN, 0, b)
ev1.record()
torch.cuda.synchronize()
print(f"chain stage: {ev0.elapsed_time(ev1) / 20 * 1e3:.1f} us  (B={B}, {nsteps} k-steps)")

stamps = torch.zeros(2 * (nsteps + 1), dtype=torch.int64, device="cuda")
lib.inf_debug_timing(plan.handle, ctypes.c_void_p(stamps.data_ptr()), nsteps)
for _ in range(3):
    stamps.zero_()
    plan.run_stage(STAGE_CHAIN, 0, b)
    torch.cuda.synchronize()
lib.inf_debug_timing(plan.handle, None, 0)
st = stamps.cpu().numpy().reshape(2, nsteps + 1).astype(np.float64) * 10.0 / 1e3  # 100 MHz -> us
for w, name in enumerate(("first", "last")):
    t = st[w] - st[w][0]
    print(f"workgroup {name}: total {t[nsteps]:.1f} us (first stage landed at step 0 = t0)")
    s0 = 0
    rows = []
    for pname, n in phases:
        s1 = s0 + n
        dt = t[s1] - t[s0] if s1 <= nsteps else float("nan")
        rows.append(f"{pname}:{dt:.1f}")
        s0 = s1
    print("   per phase (us): " + "  ".join(rows))
    d = np.diff(t[:nsteps])
    print(f"   per step: median {np.median(d):.2f}  p90 {np.percentile(d, 90):.2f}  max {d.max():.2f} us")
print("start skew last-first:", (st[1][0] - st[0][0]), "us")
