"""Bitwise fingerprint of graph-replayed training steps (the trainer's shape: one captured
sequence of steps over a permuted ray source, batch index from ctrl, Adam, advance) -- run it
under two libraries (INF_LIB=...) to check that a change to the replayed step left its
arithmetic untouched.  Cases: full batches; a batch that is not a multiple of the tile (padded
rays); a ray bound that ends inside the last batch (out-of-range rays).

    python tools/graph_hash.py
"""
import hashlib
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from inf_hip import runtime  # noqa: E402

k, H, L, s = 1024, 256, 8, 4
P = H * k + H + (L - 3) * (H * H + H) + (H * H + H + H * k + H) + 3 * H + 3
V = 20000


def case(B, nsteps, replays, num_rays=None, seed=5):
    rng = np.random.default_rng(seed)
    params = torch.from_numpy((rng.standard_normal(P) * 0.03).astype(np.float32)).cuda()
    plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                        exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
    N = B * nsteps * replays
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32)).cuda()
    vids = rng.integers(0, V, (N, 3))
    vids[::97, 1] = V + 3  # out-of-range vertices: zero feature rows
    src = runtime.RaySource(E, torch.from_numpy(vids).cuda(),
                            torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                            torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda(), validate=False)
    perm = torch.from_numpy(rng.permutation(N)).cuda()
    plan.set_lr(1e-3)
    b = plan.make_batch(source=src, ray_idx=perm[:num_rays] if num_rays else perm, batch=B, offset_from_ctrl=True)
    plan.set_batch_index(0)
    plan.train_step(b, None, apply_adam=True, advance=True)  # eager warm-up step (batch 0)
    g = torch.cuda.CUDAGraph()
    st = torch.cuda.Stream()
    st.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(st):
        with torch.cuda.graph(g, stream=st):
            for _ in range(nsteps):
                plan.train_step(b, None, apply_adam=True, advance=True)
    torch.cuda.current_stream().wait_stream(st)
    losses = []
    for r in range(replays):
        plan.set_batch_index(r * nsteps if r else 1)
        plan.reset_epoch_sums()
        g.replay()
        torch.cuda.synchronize()
        losses.append(plan.read_ctrl()["epoch_loss"])
    h = hashlib.sha256()
    for t in (params, plan.exp_avg, plan.exp_avg_sq):
        h.update(t.cpu().numpy().tobytes())
    return f"B={B} steps={nsteps}x{replays} rays={num_rays} loss={losses[-1]!r} sha={h.hexdigest()[:20]}"


print(case(4096, 8, 3), flush=True)
print(case(4000, 6, 2), flush=True)
print(case(4096, 5, 2, num_rays=4096 * 9 + 1000), flush=True)
