"""Diagnostic: per-phase wall-clock stamps of the register-streamed chain (chain3.hip) for
wave 0 of the first and the last workgroup, plus the stage's HIP-event time.

    python tools/chain3_timing.py [batch] [k] [hidden] [layers] [skip]
    C3T_RFF=1: the input is the RFF encoding (k = 2 * k_rff + 3) of interpolated positions
    C3T_MODE=bf16x3: the split-bf16 chain (chain3.hip X3) instead of the bf16 one
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
plan = runtime.Plan(k, H, L, s, os.environ.get("C3T_MODE", "bf16"), "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V, N = 50000, B
if os.environ.get("C3T_RFF"):
    ek = (k - 3) // 2
    Bm = torch.from_numpy((rng.standard_normal((3, ek)) * 8).astype(np.float32)).cuda()
    plan.encoding = runtime.Encoding("rff", ek, Bm, True)
    E = torch.from_numpy((rng.random((V, 3)) * 2 - 1).astype(np.float32)).cuda()
else:
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
plan.set_lr(1e-4)
b = plan.make_batch(source=src, batch=B)
for _ in range(3):
    plan.train_step(b, None, apply_adam=True)
torch.cuda.synchronize()
nphase = 2 * L - 3
names = [f"fwd{l}" for l in range(0, L - 1)] + [f"bwd{l}" for l in range(L - 2, 0, -1)]

ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
ev0.record()
for _ in range(50):
    plan.run_stage(STAGE_CHAIN, 0, b)
ev1.record()
torch.cuda.synchronize()
print(f"chain3 stage: {ev0.elapsed_time(ev1) / 50 * 1e3:.1f} us  (B={B}, {nphase} phases)")

n1 = 7 * nphase + 6
stamps = torch.zeros(2 * n1, dtype=torch.int64, device="cuda")
lib.inf_debug_timing(plan.handle, ctypes.c_void_p(stamps.data_ptr()), nphase)
for _ in range(5):
    stamps.zero_()
    plan.run_stage(STAGE_CHAIN, 0, b)
    torch.cuda.synchronize()
lib.inf_debug_timing(plan.handle, None, 0)
st = stamps.cpu().numpy().reshape(2, n1).astype(np.float64) * 10.0 / 1e3  # 100 MHz -> us
for w, name in enumerate(("first", "last")):
    t = st[w] - st[w][0]
    e = 3 * nphase + 3
    print(f"workgroup {name}: entry -> end {t[e - 1]:.2f} us, startup {t[1]:.2f} us "
          f"(fragments issued {t[e]:.2f}, feature tile gathered {t[e + 1]:.2f}, barrier 0 {t[e + 2]:.2f})")
    rows = []
    for p in range(nphase):
        mm = t[2 + 3 * p] - t[1 + 3 * p]
        ep = t[3 + 3 * p] - t[2 + 3 * p]
        body = t[4 * nphase + 6 + p] - t[2 + 3 * p]
        b2 = t[3 + 3 * p] - t[4 * nphase + 6 + p]
        sw = t[5 * nphase + 6 + p] - t[4 * nphase + 6 + p]
        lw = t[6 * nphase + 6 + p] - t[4 * nphase + 6 + p]
        rows.append(f"{names[p]}: mfma {mm:.2f} epi {ep:.2f} (body {body:.2f}, B2 wait {b2:.2f}; "
                    f"at B2 vs wave 0: store wave {sw:+.2f}, last wave {lw:+.2f})")
    print("   " + "\n   ".join(rows))
print("entry skew last-first:", (st[1][0] - st[0][0]), "us")
