"""Diagnostic: per-block wall-clock stamps (100 MHz) of the forward-only register chain
(rchain.hip) for wave 0 of workgroup 0 and of the middle workgroup, on the bench's
render configuration (k=1024 8x256 bf16, V=400k random rows), plus the launch time.

    python tools/rchain_timing.py [hits] [coherent(0/1)]      (PROJ=1: projected table)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from inf_hip import lib, runtime

n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 18
coherent = len(sys.argv) > 2 and sys.argv[2] == "1"
import model as M
torch.manual_seed(0)
m = M.make_model({"k": 1024, "num_layers": 8, "mlp_hidden_dim": 256, "skip_layer_idx": 4}).cuda()
m.kernel_mode = "bf16"
V = 400_000
g = torch.Generator(device="cuda").manual_seed(0)
E = torch.randn((V, 1024), generator=g, device="cuda")
if coherent:
    base = torch.randint(0, V - 64, (n // 64,), device="cuda").repeat_interleave(64)
    vids = (base[:, None] + torch.randint(0, 64, (n, 3), device="cuda")).clamp_max(V - 1)
else:
    vids = torch.randint(0, V, (n, 3), device="cuda")
bary = torch.full((n, 3), 1 / 3, device="cuda")
src = runtime.RaySource(E, vids, bary, None)
plan = m.hip_plan(n)
hit = torch.arange(n, device="cuda")
img = torch.ones((n, 3), device="cuda")
proj = None
if os.environ.get("PROJ") == "1":
    T = src.table_for(plan)
    proj = plan.project_table(T)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        plan.project_table(T, out=proj)
    e1.record()
    torch.cuda.synchronize()
    pm = e0.elapsed_time(e1) / 10
    fl = proj.shape[0] * 2 * 1024 * 512
    print(f"project_table: {pm * 1e3:.1f} us for V={V} -> {fl / pm / 1e9:.0f} TFLOP/s, "
          f"{(V * 2048 + proj.numel() * 2) / pm / 1e6:.0f} GB/s")
b = plan.make_batch(source=src, offset=0, batch=n, projected=proj)  # (n may exceed max_batch when projected)
for _ in range(3):
    plan.render(b, hit, None, img)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(10):
    plan.render(b, hit, None, img)
e1.record()
torch.cuda.synchronize()
ms = e0.elapsed_time(e1) / 10
print(f"rchain launch: {ms * 1e3:.1f} us for {n} rays ({n / 64:.0f} workgroups) -> {n / ms / 1e3:.1f} M rays/s")
RS = 4 + 64
st = torch.zeros(2 * RS, dtype=torch.int64, device="cuda")
lib.inf_debug_timing(plan.handle, ctypes.c_void_p(st.data_ptr()), 0)
plan.render(b, hit, None, img)
torch.cuda.synchronize()
lib.inf_debug_timing(plan.handle, None, 0)
s = st.cpu().numpy().reshape(2, RS).astype(np.float64) * 10 / 1e3
for w, name in enumerate(("first", "middle")):
    t = s[w] - s[w][0]
    nz = [i for i in range(RS) if s[w][i] != 0]
    last = max(nz)
    print(f"workgroup {name}: records {t[1]:.2f} us, chunk-0 gather {t[2] - t[1]:.2f} us, total {t[last]:.2f} us")
    print("   block starts:", " ".join(f"{t[i]:.2f}" for i in range(3, last + 1)))
