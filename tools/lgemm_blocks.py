"""Diagnostic: per-workgroup schedule of the weight-gradient GEMM (lgemm.hip) in the
register-streamed training step: entry / prologue done / main loop done / exit clocks of
every block (inf_debug_block_times).

    python tools/lgemm_blocks.py [batch] [k]

(k > 1024: config D's shape, whose dW runs the update fused in -- LGB_STEP=1 times the
step's launch with it)
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from inf_hip import lib, runtime, STAGE_DW_GEMM

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k, H, L, s = (int(sys.argv[2]) if len(sys.argv) > 2 else 1024), 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V = 50000 if k <= 1024 else 20000
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
plan.set_lr(1e-4)
b = plan.make_batch(source=src, batch=B)
for _ in range(3):
    plan.train_step(b, None, apply_adam=True)
torch.cuda.synchronize()
NB = 8192
st = torch.zeros(NB * 8, dtype=torch.int64, device="cuda")
for _ in range(3):
    plan.run_stage(STAGE_DW_GEMM, 0, b)
torch.cuda.synchronize()
lib.inf_debug_block_times(plan.handle, ctypes.c_void_p(st.data_ptr()))
if os.environ.get("LGB_STEP"):
    plan.train_step(b, None, apply_adam=True)  # the step's launch (update fused in)
else:
    plan.run_stage(STAGE_DW_GEMM, 0, b)
torch.cuda.synchronize()
lib.inf_debug_block_times(plan.handle, None)
t = st.cpu().numpy().reshape(NB, 8).astype(np.float64)
n = int((t[:, 0] > 0).sum())
t = t[:n] * 10.0 / 1e3  # 100 MHz -> us
raw = t.copy()
t = t - t[:, 0].min()
pro, main, epi, tot = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2], t[:, 3] - t[:, 0]
print(f"{n} blocks, kernel span {t[:, 3].max():.2f} us")
q = lambda v: f"median {np.median(v):.2f}  p10 {np.percentile(v, 10):.2f}  p90 {np.percentile(v, 90):.2f}  max {v.max():.2f}"
print("  start    ", q(t[:, 0]))
print("  prologue ", q(pro))
print("  main     ", q(main))
print("  epilogue ", q(epi))
print("  total    ", q(tot))
if (raw[:, 4] > 0).any():
    ep = raw[:, 4] > 0
    print("  fused: ticket after main", q(raw[ep, 4] - raw[ep, 2]), "\n         wait/claim   ", q(raw[ep, 5] - raw[ep, 4]))
    it = raw[:, 6] > 0
    print(f"         items run by {int(it.sum())} blocks: ", q(raw[it, 7] - raw[it, 6]))
late = t[:, 0] > 1.0
print(f"  blocks starting after 1 us: {int(late.sum())} (start median {np.median(t[late, 0]) if late.any() else 0:.2f})")
