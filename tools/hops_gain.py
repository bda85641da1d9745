"""Diagnostic: what the dependent loads ahead of chain3's gather cost on the config-B step
(graph-replayed, 8 steps per graph, after a settle).  Variants of the same batch shape:
  perm+ctrl  production: ctrl.batch_index -> ray_idx[offset + b] -> vids / bary -> rows
  ctrl       no permutation: ctrl.batch_index -> vids / bary -> rows
  fixed      no permutation, fixed offset: vids / bary -> rows
  xslot      rows pre-gathered once (no gather at all: tools/xslot_gain.py's bound)

    python tools/hops_gain.py [batch]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from inf_hip import runtime  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
k, H, L, s = 1024, 256, 8, 4
rng = np.random.default_rng(0)
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                    exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
V, N = 50000, 400 * B
E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                        torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                        torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
perm = torch.randperm(N, device="cuda")
plan.set_lr(1e-5)
variants = {
    "perm+ctrl": (plan.make_batch(source=src, ray_idx=perm, batch=B, offset_from_ctrl=True), True, None),
    "ctrl": (plan.make_batch(source=src, batch=B, offset_from_ctrl=True), True, None),
    "fixed": (plan.make_batch(source=src, offset=3 * B, batch=B), False, None),
    "xslot": (plan.make_batch(source=src, ray_idx=perm, batch=B, offset_from_ctrl=True), False, 0),
}
plan.set_prefetch_index(3)
assert plan.prefetch(variants["xslot"][0], 0)
for b, adv, xs in variants.values():
    for _ in range(3):
        plan.set_batch_index(0)
        plan.train_step(b, None, apply_adam=True, xslot=xs, advance=adv)
torch.cuda.synchronize()


def timed(b, adv, xs):
    g = torch.cuda.CUDAGraph()
    s_ = torch.cuda.Stream()
    s_.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s_):
        with torch.cuda.graph(g, stream=s_):
            for _ in range(8):
                plan.train_step(b, None, apply_adam=True, xslot=xs, advance=adv)
    torch.cuda.current_stream().wait_stream(s_)
    plan.set_batch_index(0)
    for _ in range(200):  # settle the clocks (~15 ms)
        g.replay()
    plan.set_batch_index(0)
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ev0.record()
    for _ in range(40):
        g.replay()
    ev1.record()
    torch.cuda.synchronize()
    return ev0.elapsed_time(ev1) / 320 * 1e3


for rep in range(3):
    print(" ".join(f"{n} {timed(*v):.2f}" for n, v in variants.items()), "us/step", flush=True)
