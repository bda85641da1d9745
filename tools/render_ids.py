"""The render slice's persistent launch (rprojw.hip via Plan.render over a projected table)
on one hit distribution only, for kernel traces / PMC passes that compare distributions:

    python tools/render_ids.py random|coherent [frames]

random: 2M hits on uniformly random vertex triples, random pixels (bench.py's frame);
coherent: bench.py's variant -- 64 consecutive hits around one random base vertex (each
vertex base + U[0, 64)), hits in pixel order.  V = 400k, k = 1024, 8 x 256 skip 4.  The
projection GEMM runs once, outside the frames."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import model as M  # noqa: E402
from inf_hip import runtime  # noqa: E402

kind = sys.argv[1] if len(sys.argv) > 1 else "random"
frames = int(sys.argv[2]) if len(sys.argv) > 2 else 10
H = W = 2048
V, k, Hd = 400_000, 1024, 256
n = H * W // 2
torch.manual_seed(0)
m = M.make_model({"k": k, "num_layers": 8, "mlp_hidden_dim": Hd, "skip_layer_idx": 4}).cuda()
m.kernel_mode = "bf16"
plan = m.hip_plan(4096)
g = torch.Generator(device="cpu").manual_seed(7)
E = torch.randn((V, k), generator=g)
E = (E / (E.max(0, keepdim=True).values - E.min(0, keepdim=True).values)).cuda()
gv = torch.Generator(device="cpu").manual_seed(11)
if kind == "coherent":
    base = torch.randint(0, V - 64, (n // 64 + 1,), generator=gv).repeat_interleave(64)[:n]
    vv = (base[:, None] + torch.randint(0, 64, (n, 3), generator=gv)).clamp_max(V - 1)
    hv = torch.randperm(H * W, generator=gv)[:n].sort().values
else:
    vv = torch.randint(0, V, (n, 3), generator=gv)
    hv = torch.randperm(H * W, generator=gv)[:n]
uv = -torch.log(torch.rand((n, 3), generator=gv).clamp_min(1e-12))
src = runtime.RaySource(E, vv.cuda(), (uv / uv.sum(1, keepdim=True)).cuda(), None, validate=False)
T = src.table_for(plan)
P = plan.project_table(T)
b = plan.make_batch(source=src, offset=0, batch=n, projected=P)
hv = hv.cuda()
img = torch.ones((H, W, 3), device="cuda")
plan.render(b, hv, None, img)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(frames):
    plan.render(b, hv, None, img)
e1.record()
torch.cuda.synchronize()
print(f"{kind}: {e0.elapsed_time(e1) / frames:.4f} ms per render launch ({n} hits)", flush=True)
