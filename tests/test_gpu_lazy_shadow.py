"""Lazy row-major weight shadows (plan.hip ensure_rowmajor): the fused chain3 step's update
writes only the MFMA fragment images; the row-major W / W^T shadows that the layered GEMMs
and the table projection read are rewritten from the fp32 masters before those launches.
After eager and graph-replayed fused steps, every forward path -- the register chain
(fragment images), the projected table (W rows) and the layered GEMMs (W) -- must see the
UPDATED weights: each is checked against the oracle forward on the current parameters."""
import os

import numpy as np
import pytest
import torch

from oracle import inf_oracle as O
from test_gpu_kernels import CFG, arena_to_dict, make_plan, rt

pytestmark = pytest.mark.gpu


def _forwards(plan, src, B):
    """RGB of the three bf16 forward paths on rays 0..B-1 of `src`."""
    out = {}
    pred = torch.empty((B, 3), device="cuda")
    plan.forward(plan.make_batch(source=src, batch=B), pred, save=False)
    out["chain"] = pred.clone()
    P = plan.project_table(src.table_for(plan))
    plan.forward(plan.make_batch(source=src, batch=B, projected=P), pred, save=False)
    out["projected"] = pred.clone()
    os.environ["INF_NO_CHAIN"] = "1"
    try:
        plan.forward(plan.make_batch(source=src, batch=B), pred, save=False)
    finally:
        del os.environ["INF_NO_CHAIN"]
    out["layered"] = pred.clone()
    torch.cuda.synchronize()
    return {k: v.cpu().numpy() for k, v in out.items()}


def test_rowmajor_shadows_follow_fused_steps():
    k, H, L, s = CFG["A"]
    B, V, nb = 256, 700, 6
    rng = np.random.default_rng(5)
    plan, params, w0 = make_plan("A", mode="bf16", max_batch=B, adam=True)
    plan.set_lr(2e-2)  # large steps: stale shadows would be far outside the bf16 bar
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    N = nb * B
    vids = rng.integers(0, V, (N, 3))
    bary = rng.dirichlet([1, 1, 1], N).astype(np.float32)
    src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(),
                         torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
    idx = torch.arange(N, device="cuda")
    b = plan.make_batch(source=src, ray_idx=idx, offset=0, batch=B,
                        offset_from_ctrl=True, loss_count=3 * B)
    X = O.gather(E, vids[:B], bary[:B])

    def check(tag):
        torch.cuda.synchronize()
        ref, _ = O.mlp_forward(arena_to_dict(params, w0, L, s), X, L, s)
        got = _forwards(plan, src, B)
        for path, rgb in got.items():
            err = float(np.abs(rgb - ref).max())
            assert err < 2e-2, f"{tag}: {path} forward differs from the oracle on the updated weights by {err}"

    before, _ = O.mlp_forward(w0, X, L, s)
    for _ in range(3):  # eager fused steps (lazy shadows)
        plan.train_step(b, None, apply_adam=True, advance=True)
    assert plan.last_step_path() == "chain3"
    check("eager")
    ref_now, _ = O.mlp_forward(arena_to_dict(params, w0, L, s), X, L, s)
    assert float(np.abs(ref_now - before).max()) > 5e-2  # the steps moved the outputs
    # captured fused steps: the host cannot see the replays, so every consumer rewrites
    plan.set_batch_index(0)
    stream = torch.cuda.Stream()
    stream.wait_stream(torch.cuda.current_stream())
    g = torch.cuda.CUDAGraph()
    with torch.cuda.stream(stream):
        with torch.cuda.graph(g, stream=stream):
            plan.train_step(b, None, apply_adam=True, advance=True)
            plan.train_step(b, None, apply_adam=True, advance=True)
    torch.cuda.current_stream().wait_stream(stream)
    plan.set_batch_index(0)
    g.replay()
    check("graph replay 1")
    g.replay()  # after a consumer already rewrote the shadows
    check("graph replay 2")
