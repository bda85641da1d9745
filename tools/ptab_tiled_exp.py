"""Experiment: the projection GEMM (ptab.hip, default tile 256 x 256 x 64) reading the table
row-major (the product) or k-tiled [tiles_m][K / 64][256][64] (a variant library built with
-DPTAB_TILED_EXP, every stage's A slice one contiguous 32 KB run).  Same arithmetic in the
same order: the outputs must be bitwise equal (checksums printed).

    python tools/ptab_tiled_exp.py rowmajor|tiled
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import model as M  # noqa: E402
from inf_hip import runtime  # noqa: E402

mode = sys.argv[1] if len(sys.argv) > 1 else "rowmajor"
V, k, H = 400_000, 1024, 256
torch.manual_seed(0)
m = M.make_model({"k": k, "num_layers": 8, "mlp_hidden_dim": H, "skip_layer_idx": 4}).cuda()
m.kernel_mode = "bf16"
plan = m.hip_plan(4096)
g = torch.Generator(device="cuda").manual_seed(1)
E = torch.randn((V, k), generator=g, device="cuda")
E /= E.max(0, keepdim=True).values - E.min(0, keepdim=True).values
T = runtime.pack_table(E, plan.in_pad, torch.bfloat16)
del E
BM, BK = 256, 64
Vp = -(-V // BM) * BM
if mode == "tiled":
    Tp = torch.zeros((Vp, plan.in_pad), dtype=torch.bfloat16, device="cuda")
    Tp[:V] = T
    T = Tp.view(Vp // BM, BM, plan.in_pad // BK, BK).permute(0, 2, 1, 3).contiguous().view(Vp, plan.in_pad)
    del Tp
nrows = V if mode == "rowmajor" else Vp
P = plan.project_table(T[:nrows] if mode == "rowmajor" else T)
torch.cuda.synchronize()
times = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(7):
    e0.record()
    for _ in range(10):
        plan.project_table(T, out=P)
    e1.record()
    torch.cuda.synchronize()
    times.append(e0.elapsed_time(e1) / 10)
x = P[:V].float()
flops = 2 * Vp * 2 * H * plan.in_pad
t = sorted(times)[len(times) // 2]
print(f"{mode}: median {t:.4f} ms (min {min(times):.4f})  {flops / (t * 1e-3) / 1e12:.0f} TFLOP/s  "
      f"checksum {float(x.sum()):.6f} {float((x * torch.arange(V, device='cuda')[:, None] % 7).sum()):.6f}", flush=True)
