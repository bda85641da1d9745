"""Tile variants of the projection GEMM (csrc/ptab.hip, INF_PTAB_TILE) against hipBLASLt at
config E's shape (V = 400k, k = 1024, 2H = 512), interleaved rounds in one process
(guide §5.4 rule 24).  Prints ms per projection (median over rounds) and TFLOP/s; checks
every variant's output against variant 0 (bf16 rounding of the same fp32 sums)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import model as M  # noqa: E402
from inf_hip import runtime  # noqa: E402

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
variants = [v for v in os.environ.get("PTAB_VARIANTS", "1,5,0,blaslt").split(",")]
outs = {}
times = {v: [] for v in variants}


def setv(v):
    os.environ.pop("INF_PROJECT_GEMM", None)
    os.environ.pop("INF_PTAB_TILE", None)
    if v == "blaslt":
        os.environ["INF_PROJECT_GEMM"] = "blaslt"
    else:
        os.environ["INF_PTAB_TILE"] = v


for v in variants:
    setv(v)
    outs[v] = plan.project_table(T)
torch.cuda.synchronize()
ref = outs["1"][:V].float()
for v in variants:
    d = (outs[v][:V].float() - ref).abs()
    print(v, "max |d| vs variant 0", float(d.max()), "rel", float((d / ref.abs().clamp_min(1e-3)).max()), flush=True)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(5):
    for v in variants:
        setv(v)
        plan.project_table(T, out=outs[v])
        torch.cuda.synchronize()
        e0.record()
        for _ in range(5):
            plan.project_table(T, out=outs[v])
        e1.record()
        torch.cuda.synchronize()
        times[v].append(e0.elapsed_time(e1) / 5)
flops = 2 * (-(-V // 128) * 128) * 2 * H * plan.in_pad
for v in variants:
    t = sorted(times[v])[len(times[v]) // 2]
    print(f"variant {v}: median {t:.4f} ms (min {min(times[v]):.4f})  {flops / (t * 1e-3) / 1e12:.0f} TFLOP/s", flush=True)
