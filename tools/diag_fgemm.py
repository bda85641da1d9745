"""Diagnostic: config B weight gradients of one 8192-ray step on 64-ray chain3 tiles, with
the dW on fgemm.hip vs lgemm.hip (INF_NO_FGEMM) and on 16-ray tiles; prints max error per
tensor relative to its max."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd")); sys.path.insert(0, ROOT)
import numpy as np, torch
from test_gpu_kernels import CFG, arena_to_dict, make_plan, rt
from oracle import inf_oracle as O
name, B = "B", 8192
k, H, L, s = CFG[name]
rng = np.random.default_rng(5)
E = rng.standard_normal((2000, k)).astype(np.float32); E /= (E.max(0) - E.min(0))
src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, 2000, (B, 3))).cuda(),
                     torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                     torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
out = {}
for tag, env in (("narrow", {}), ("wide_fgemm", {"INF_CHAIN3_WIDE": "1"}), ("wide_lgemm", {"INF_CHAIN3_WIDE": "1", "INF_NO_FGEMM": "1"})):
    for kk in ("INF_CHAIN3_WIDE", "INF_NO_FGEMM"):
        os.environ.pop(kk, None)
    os.environ.update(env)
    plan, params, w = make_plan(name, mode="bf16", max_batch=B, adam=True)
    plan.train_step(plan.make_batch(source=src, batch=B), None, apply_adam=False)
    torch.cuda.synchronize()
    out[tag] = arena_to_dict(plan.grads, w, L, s)
    print(tag, plan.last_step_path(), flush=True)
for tag in ("wide_fgemm", "wide_lgemm"):
    for n in O.layer_names(L, s):
        ref = out["narrow"][n]; g = out[tag][n]
        print(tag, n, float(np.abs(g - ref).max() / max(np.abs(ref).max(), 1e-12)), float(np.abs(g).max()), float(np.abs(ref).max()))
