"""Diagnostic: inf_project_table through hipBLASLt vs torch on the bf16 operands, a small
table first, then config E's 400k-vertex table (a sample of rows), and its time."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import torch

import model as M
from inf_hip import runtime

torch.manual_seed(0)
m = M.make_model({"k": 1024, "num_layers": 8, "mlp_hidden_dim": 256, "skip_layer_idx": 4}).cuda()
m.kernel_mode = "bf16"
plan = m.hip_plan(1024)
W = [p.detach() for n, p in m.named_parameters() if n.endswith("weight") and p.shape == (256, 1024)]
Wc = torch.cat([w.bfloat16().float() for w in W], 0)
for V in (1000, 400_000):
    E = torch.randn((V, 1024), device="cuda") * 0.3
    T = runtime.pack_table(E, plan.in_pad, torch.bfloat16)
    P = plan.project_table(T)
    torch.cuda.synchronize()
    rows = torch.arange(0, V, max(1, V // 2000), device="cuda")
    ref = T[rows].float() @ Wc.t()
    err = (P[rows].float() - ref).abs().max().item() / ref.abs().max().item()
    print(f"V={V}: rel err {err:.2e}", flush=True)
    assert err < 1e-2
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(10):
        plan.project_table(T, out=P)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"   {ms * 1e3:.1f} us -> {V * 512 * 1024 * 2 / ms / 1e9:.0f} TFLOP/s", flush=True)
    Wb = Wc.bfloat16()
    for _ in range(3):
        torch.matmul(T, Wb.t())
    e0.record()
    for _ in range(10):
        torch.matmul(T, Wb.t())
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 10
    print(f"   torch.matmul {ms * 1e3:.1f} us -> {V * 512 * 1024 * 2 / ms / 1e9:.0f} TFLOP/s", flush=True)
