"""Diagnostics for the split-bf16 chain (chain3.hip X3): predicted RGB of one gradient step
at config B / R against the fp32 oracle, for the default library and the libraries named on
the command line (INF_LIB variants), plus the plain bf16 chain as a reference point."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "intrinsic-neural-fields_amd"), ROOT, os.path.join(ROOT, "tests")]
from conftest import golden  # noqa: E402
from oracle import inf_oracle as O  # noqa: E402
from inf_hip import runtime  # noqa: E402

CFG = {"A": (64, 128, 4, 2), "R": (1023, 128, 6, 3), "B": (1024, 256, 8, 4)}
for name, B in (("B", 4096), ("R", 2048)):
    k, H, L, s = CFG[name]
    d = golden(f"g2_forward_{name}.npz")
    w = {kk[2:]: d[kk] for kk in d.files if kk.startswith("w:")}
    rng = np.random.default_rng(31)
    V = 2000
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= E.max(0) - E.min(0)
    vids = rng.integers(0, V, (B, 3))
    bary = rng.dirichlet([1, 1, 1], B).astype(np.float32)
    rgb = rng.random((B, 3)).astype(np.float32)
    src = runtime.RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(),
                            torch.from_numpy(rgb).cuda())
    p_ref, _ = O.mlp_forward(w, O.gather(E, vids, bary), L, s)
    for mode in ("bf16x3", "bf16"):
        params = torch.cat([torch.from_numpy(np.ascontiguousarray(w[n])).reshape(-1) for n in O.layer_names(L, s)]).cuda()
        plan = runtime.Plan(k, H, L, s, mode, "L2", B, params, torch.zeros_like(params), torch.zeros_like(params),
                            torch.zeros_like(params))
        pred = torch.empty((B, 3), device="cuda")
        plan.train_step(plan.make_batch(source=src, batch=B), pred, apply_adam=False)
        err = np.abs(pred.cpu().numpy() - p_ref)
        print(name, mode, plan.last_step_path(), "RGB err max", float(err.max()), "mean", float(err.mean()),
              "rows>1e-3", int((err.max(1) > 1e-3).sum()), "first bad rows", np.nonzero(err.max(1) > 1e-3)[0][:8].tolist())
