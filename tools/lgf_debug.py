"""Diagnostics for the fused dW + update (lgemm GT): one step without Adam, gradients of the
LGF path vs the split-K slab path (the default; LGF is INF_LGF=1) per layer -- max error, where it sits."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "intrinsic-neural-fields_amd"), ROOT, os.path.join(ROOT, "tests")]
from test_gpu_kernels import CFG, arena_to_dict, make_plan, rt  # noqa: E402
from oracle import inf_oracle as O  # noqa: E402

for name, B in (("A", 4096), ("B", 8192), ("B", 4096), ("R", 4096)):
    rng = np.random.default_rng(15)
    k, H, L, s = CFG[name]
    V = 3000
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                         torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                         torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
    out = {}
    for tag in ("lgf", "slab"):
        os.environ["INF_LGF"] = "1" if tag == "lgf" else "0"
        plan, params, w = make_plan(name, mode="bf16", max_batch=B, adam=True)
        b = plan.make_batch(source=src, batch=B)
        plan.grads.fill_(float("nan"))
        plan.train_step(b, None, apply_adam=False)
        torch.cuda.synchronize()
        out[tag] = (arena_to_dict(plan.grads, w, L, s), plan.last_step_fused_update(), plan.dw_splits if hasattr(plan, "dw_splits") else None)
    os.environ.pop("INF_LGF", None)
    print(f"== {name} B={B} fused: lgf {out['lgf'][1]} slab {out['slab'][1]}")
    for n in O.layer_names(L, s):
        a, r = out["lgf"][0][n], out["slab"][0][n]
        d = np.abs(a - r)
        scale = max(float(np.nanmax(np.abs(r))), 1e-30)
        nan = int(np.isnan(a).sum())
        bad = d > 1e-5 * scale
        msg = f"{n:24s} shape {a.shape} max|ref| {scale:.3e} rel err {float(np.nanmax(d)) / scale:.3e} nan {nan} bad {int(bad.sum())}"
        if bad.any() and a.ndim == 2:
            rows = np.nonzero(bad.any(1))[0]
            cols = np.nonzero(bad.any(0))[0]
            msg += f" rows {rows.min()}..{rows.max()} ({len(rows)}) cols {cols.min()}..{cols.max()} ({len(cols)})"
            i, j = np.unravel_index(np.nanargmax(d), d.shape)
            msg += f" worst ({i},{j}) got {a[i, j]:.4e} ref {r[i, j]:.4e}"
        print(msg)
