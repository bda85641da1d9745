"""Render slice at config E's size (k = 1024, 8 x 256 MLP, skip 4, a
400k-vertex table, a 2048 x 2048 frame with half the pixels hit), bf16: the forward-only
register chain (csrc/rchain.hip) against the oracle on a sample of hits (predicted RGB
within 2e-2, the bf16 bar of test_gpu_kernels.py) and against the LDS-ring chain on the
whole frame (5e-4), plus whole-frame properties: background pixels untouched, every hit
pixel written, values in (0, 1), no NaN; and the no-grad forward of loader batches
(shuffled ray indices) through the same kernel."""
import numpy as np
import pytest
import torch

from oracle import inf_oracle as O

pytestmark = pytest.mark.gpu


def _setup(k=1024, H=256, L=8, s=4, V=400_000, HW=2048 * 2048, seed=0):
    import model as M
    from inf_hip import runtime
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
    m.kernel_mode = "bf16"
    w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
    g = torch.Generator(device="cuda").manual_seed(seed)
    E = torch.randn((V, k), generator=g, device="cuda")
    E /= E.max(0, keepdim=True).values - E.min(0, keepdim=True).values
    nhit = HW // 2
    gc = torch.Generator().manual_seed(seed)
    # spatially coherent hits, as a cast produces: neighbouring pixels on nearby faces
    base = torch.randint(0, V - 64, (nhit // 64,), generator=gc).repeat_interleave(64)
    vids = (base[:, None] + torch.randint(0, 64, (nhit, 3), generator=gc)).clamp_max(V - 1)
    u = -torch.log(torch.rand((nhit, 3), generator=gc).clamp_min(1e-12))
    bary = u / u.sum(1, keepdim=True)
    hit = torch.randperm(HW, generator=gc)[:nhit].sort().values
    src = runtime.RaySource(E, vids.cuda(), bary.cuda(), None)
    return m, w, E, src, vids, bary, hit.cuda(), HW


def _render(m, src, hit, HW, chunk=1 << 18):
    rt = m.hip_runtime()
    plan = m.hip_plan(chunk)
    img = torch.ones((HW, 3), device="cuda")
    n = hit.shape[0]
    for lo in range(0, n, chunk):
        b = plan.make_batch(source=src, offset=lo, batch=min(chunk, n - lo))
        plan.render(b, hit[lo:lo + b.batch], None, img)
    torch.cuda.synchronize()
    del rt
    return img


def test_render_config_e(monkeypatch):
    m, w, E, src, vids, bary, hit, HW = _setup()
    img = _render(m, src, hit, HW)
    monkeypatch.setenv("INF_NO_RCHAIN", "1")
    m._rt.plan = None  # a fresh plan on the LDS-ring chain
    img_chain = _render(m, src, hit, HW)
    monkeypatch.delenv("INF_NO_RCHAIN")
    a = img.cpu().numpy()
    assert np.isfinite(a).all()
    hit_np = hit.cpu().numpy()
    mask = np.zeros(HW, bool)
    mask[hit_np] = True
    assert (a[~mask] == 1.0).all()                       # background untouched
    assert ((a[mask] > 0) & (a[mask] < 1)).all()          # every hit pixel written by the sigmoid
    np.testing.assert_allclose(a, img_chain.cpu().numpy(), atol=5e-4)
    # oracle on a sample of hits (fp32 weights and table; the kernel computes in bf16)
    rng = np.random.default_rng(3)
    sample = np.concatenate([rng.choice(hit_np.shape[0], 1000, replace=False), [0, hit_np.shape[0] - 1]])
    sv = vids.numpy()[sample]
    rows, inv = np.unique(sv.reshape(-1), return_inverse=True)
    E_sub = E[torch.from_numpy(rows).cuda()].cpu().numpy()
    X = O.gather(E_sub, inv.reshape(sv.shape), bary.numpy()[sample])
    p_ref, _ = O.mlp_forward(w, X, 8, 4)
    err = np.abs(a[hit_np[sample]] - p_ref).max()
    assert err < 2e-2, err


def test_forward_loader_batches_rchain(monkeypatch):
    """model(batch) under no_grad on shuffled loader batches (Trainer.evaluate's call,
    trainer.py:164-187): the register chain reads the rays through the permutation."""
    from ray_dataloader import RayDataLoader
    import model as M
    rng = np.random.default_rng(4)
    V, N, B, k = 3000, 5000, 2048, 1024
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3)
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    rgb = torch.from_numpy(rng.random((N, 3)).astype(np.float32))
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": 8, "mlp_hidden_dim": 256, "skip_layer_idx": 4}).cuda()
    m.kernel_mode = "bf16"
    w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
    ld = RayDataLoader(E, "efuncs", vids, bary, rgb, None, None, B, True, False, device="cuda")
    preds, idx = [], []
    with torch.no_grad():
        for batch in ld:
            preds.append(m(batch).cpu().numpy())
            idx.append(ld.idxs[batch._offset:batch._offset + batch.batch_size].cpu().numpy())
    plan = m._rt.plan
    assert plan is not None
    pred = np.concatenate(preds)
    rows = np.concatenate(idx)
    p_ref, _ = O.mlp_forward(w, O.gather(E.numpy(), vids.numpy()[rows], bary.numpy()[rows]), 8, 4)
    assert np.abs(pred - p_ref).max() < 2e-2
