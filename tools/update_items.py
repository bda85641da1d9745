"""Diagnostic: per-workgroup schedule of the update launch (adam.hip update_kernel) of the
headline step: entry / item + segment loaded / data loaded / stores issued / stores done
clocks of every matrix item (inf_debug_block_times, region UPDATE_STAMP_BLOCK0), and the
update stage's HIP-event time.

    python tools/update_items.py [batch] [k H L s]
"""
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)
import numpy as np
import torch

from inf_hip import lib, runtime, STAGE_UPDATE

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k, H, L, s = (int(x) for x in sys.argv[2:6]) if len(sys.argv) > 5 else (1024, 256, 8, 4)
rng = np.random.default_rng(0)
kin = k
P = H * kin + H + (L - 3) * (H * H + H) + (H * H + H + H * kin + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V = 50000
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (B, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], B).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((B, 3)).astype(np.float32)).cuda())
plan.set_lr(1e-4)
b = plan.make_batch(source=src, batch=B)
for _ in range(3):
    plan.train_step(b, None, apply_adam=True)
torch.cuda.synchronize()

# stage time (HIP events over repeated launches, as bench.py's stages)
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for rep in range(3):
    torch.cuda.synchronize()
    e0.record()
    for _ in range(200):
        plan.run_stage(STAGE_UPDATE, 1, b)
    e1.record()
    torch.cuda.synchronize()
    print(f"update stage: {e0.elapsed_time(e1) / 200 * 1e3:.2f} us")

NB, B0 = 8192, 6144
st = torch.zeros(NB * 8, dtype=torch.int64, device="cuda")
for trial in range(3):
    st.zero_()
    for _ in range(20):
        plan.run_stage(STAGE_UPDATE, 1, b)  # warm
    torch.cuda.synchronize()
    lib.inf_debug_block_times(plan.handle, ctypes.c_void_p(st.data_ptr()))
    if os.environ.get("UPD_STEP"):
        plan.train_step(b, None, apply_adam=True)
    else:
        plan.run_stage(STAGE_UPDATE, 1, b)
    torch.cuda.synchronize()
    lib.inf_debug_block_times(plan.handle, None)
    t = st.cpu().numpy().reshape(NB, 8)[B0:].astype(np.float64)
    m = (t[:, 0] > 0) & (t[:, 4] > 0)
    n = int(m.sum())
    if n == 0:
        print("no update stamps (library without them)")
        break
    t = t[m] * 10.0 / 1e3  # 100 MHz -> us
    t0 = t[:, 0].min()
    t = t - t0
    q = lambda v: f"median {np.median(v):5.2f}  p10 {np.percentile(v, 10):5.2f}  p90 {np.percentile(v, 90):5.2f}  max {v.max():5.2f}"
    print(f"trial {trial}: {n} matrix items, span entry-min -> exit-max {t[:, 4].max():.2f} us")
    print("  entry           ", q(t[:, 0]))
    print("  item+seg loaded ", q(t[:, 1] - t[:, 0]))
    print("  data loaded     ", q(t[:, 2] - t[:, 1]))
    print("  apply + issue   ", q(t[:, 3] - t[:, 2]))
    print("  stores drained  ", q(t[:, 4] - t[:, 3]))
    print("  total           ", q(t[:, 4] - t[:, 0]))
