"""Render slice at config E's size (k = 1024, 8 x 256 MLP, skip 4, a
400k-vertex table, a 2048 x 2048 frame with half the pixels hit), bf16: the forward-only
register chain (csrc/rchain.hip) against the oracle on a sample of hits (predicted RGB
within 2e-2, the bf16 bar of test_gpu_kernels.py) and against the LDS-ring chain on the
whole frame (5e-4), plus whole-frame properties: background pixels untouched, every hit
pixel written, values in (0, 1), no NaN; and the no-grad forward of loader batches
(shuffled ray indices) through the same kernel.  The projected-table render
(inf_project_table + INF_ENC_PROJECTED batches: the vertices' W_0 / W_y rows interpolated
per hit) against the oracle, the feature-gather chain and a torch fp32 projection, with
tail tiles, out-of-range ids, the 128-wide MLP and the forward-only guard."""
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


def _render(m, src, hit, HW, chunk=1 << 18, project=False):
    rt = m.hip_runtime()
    plan = m.hip_plan(chunk)
    img = torch.ones((HW, 3), device="cuda")
    n = hit.shape[0]
    proj = plan.project_table(src.table_for(plan)) if project else None
    if project:
        chunk = n  # projected batches are not bounded by the plan's max batch: one launch
    for lo in range(0, n, chunk):
        b = plan.make_batch(source=src, offset=lo, batch=min(chunk, n - lo), projected=proj)
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


def _oracle_sample(w, E, vids, bary, hit_np, L, s, n=1000, seed=3):
    rng = np.random.default_rng(seed)
    sample = np.concatenate([rng.choice(hit_np.shape[0], min(n, hit_np.shape[0]), replace=False),
                             [0, hit_np.shape[0] - 1]])
    sv = vids.numpy()[sample]
    rows, inv = np.unique(sv.reshape(-1), return_inverse=True)
    E_sub = E[torch.from_numpy(rows).cuda()].cpu().numpy()
    X = O.gather(E_sub, inv.reshape(sv.shape), bary.numpy()[sample])
    p_ref, _ = O.mlp_forward(w, X, L, s)
    return sample, p_ref


def test_render_projected_config_e():
    """The projected render at config E's size: the oracle bar (2e-2) on a sample, and
    the feature-gather register chain on the whole frame.  The two differ by where bf16
    rounds (the interpolated features vs the vertices' projections): 5e-3 in RGB."""
    m, w, E, src, vids, bary, hit, HW = _setup()
    img = _render(m, src, hit, HW, project=True).cpu().numpy()
    img_g = _render(m, src, hit, HW).cpu().numpy()
    hit_np = hit.cpu().numpy()
    mask = np.zeros(HW, bool)
    mask[hit_np] = True
    assert np.isfinite(img).all() and (img[~mask] == 1.0).all()
    assert ((img[mask] > 0) & (img[mask] < 1)).all()
    np.testing.assert_allclose(img, img_g, atol=5e-3)
    sample, p_ref = _oracle_sample(w, E, vids, bary, hit_np, 8, 4)
    assert np.abs(img[hit_np[sample]] - p_ref).max() < 2e-2


@pytest.mark.parametrize("gemm", ["ptab", "hipblaslt", "own"])
@pytest.mark.parametrize("V,H", [(100, 256), (256, 256), (1000, 256), (5000, 256), (777, 128)])
def test_project_table_vs_torch(V, H, gemm, monkeypatch):
    """inf_project_table against torch fp32 on the bf16 operands: whole tiles, tail tiles
    (V % 256 != 0) and a table smaller than one tile; through the hand-written 256 x 256
    GEMM (csrc/ptab.hip, the default), hipBLASLt (INF_PROJECT_GEMM=blaslt) and the plan's
    own grouped GEMM (INF_PROJECT_GEMM=own).  Every element within the bf16 rounding of
    the fp32 product (2^-9 relative) plus summation-order slack; rows past V untouched."""
    if gemm != "ptab":
        monkeypatch.setenv("INF_PROJECT_GEMM", "own" if gemm == "own" else "blaslt")
    import model as M
    torch.manual_seed(1)
    k = 512
    m = M.make_model({"k": k, "num_layers": 8, "mlp_hidden_dim": H, "skip_layer_idx": 4}).cuda()
    m.kernel_mode = "bf16"
    plan = m.hip_plan(1024)
    E = torch.randn((V, k), device="cuda") * 0.3
    from inf_hip import runtime
    T = runtime.pack_table(E, plan.in_pad, torch.bfloat16)
    P = plan.project_table(T)
    torch.cuda.synchronize()
    assert P.shape == (((V + 127) // 128) * 128, 2 * H)
    sd = {n: p.detach() for n, p in m.named_parameters()}
    W0 = [v for n, v in sd.items() if n.endswith("weight") and v.shape == (H, k)]
    assert len(W0) == 2  # layer 0 and the skip layer's Ly (parameter order)
    Eb = T[:, :k].float()
    ref = torch.cat([Eb @ W.bfloat16().float().t() for W in W0], 1)
    got = P[:V].float()
    err = (got - ref).abs()
    bound = 4e-3 * ref.abs() + 1e-4 * ref.abs().max()
    assert bool((err <= bound).all()), (err - bound).max().item()
    if gemm == "ptab" and P.shape[0] > V:  # rows past V keep what the caller put there
        P2 = torch.full_like(P, 7.0)
        plan.project_table(T, out=P2)
        torch.cuda.synchronize()
        assert bool((P2[V:] == 7.0).all())
        assert torch.equal(P2[:V], P[:V])


def test_render_projected_small_models(monkeypatch):
    """The 128-wide MLP (TN = 1 per wave), ragged batches and out-of-range vertex ids
    (rows read as zero, as the gather does) against the oracle and the gather chain."""
    import model as M
    from inf_hip import runtime
    rng = np.random.default_rng(5)
    for (k, H, L, s) in [(256, 128, 6, 3), (1024, 256, 8, 4)]:
        V, N, HW = 777, 3001, 4096
        E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3).cuda()
        vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
        vids[7, 1] = V + 5  # out of range: the whole feature row reads as zero
        bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
        hit = torch.from_numpy(np.sort(rng.choice(HW, N, replace=False))).cuda()
        torch.manual_seed(0)
        m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
        m.kernel_mode = "bf16"
        w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
        src = runtime.RaySource(E, vids.cuda(), bary.cuda(), None, validate=False)
        img = _render(m, src, hit, HW, chunk=1024, project=True).cpu().numpy()
        img_g = _render(m, src, hit, HW, chunk=1024).cpu().numpy()
        np.testing.assert_allclose(img, img_g, atol=5e-3)
        hit_np = hit.cpu().numpy()
        X = O.gather(E.cpu().numpy(), np.minimum(vids.numpy(), V - 1), bary.numpy())
        X[7] = 0.0
        p_ref, _ = O.mlp_forward(w, X, L, s)
        assert np.abs(img[hit_np] - p_ref).max() < 2e-2


def test_projected_batches_are_forward_only():
    import model as M
    from inf_hip import runtime
    torch.manual_seed(0)
    m = M.make_model({"k": 256, "num_layers": 6, "mlp_hidden_dim": 128, "skip_layer_idx": 3}).cuda()
    m.kernel_mode = "bf16"
    plan = m.hip_plan(1024)
    E = torch.randn((300, 256), device="cuda")
    vids = torch.randint(0, 300, (1024, 3), device="cuda")
    bary = torch.full((1024, 3), 1 / 3, device="cuda")
    rgb = torch.rand((1024, 3), device="cuda")
    src = runtime.RaySource(E, vids, bary, rgb)
    P = plan.project_table(src.table_for(plan))
    b = plan.make_batch(source=src, offset=0, batch=1024, projected=P)
    pred = torch.empty((1024, 3), device="cuda")
    plan.forward(b, pred, save=False)  # the no-grad forward runs
    with pytest.raises(RuntimeError):
        plan.train_step(b, pred, apply_adam=True)
    with pytest.raises(RuntimeError):
        plan.forward(b, pred, save=True)


def test_renderer_projected_matches_gather(monkeypatch):
    """Renderer.render_hits with the projection forced on and off."""
    import model as M
    from renderer import Renderer
    rng = np.random.default_rng(6)
    V, N, Hh, Ww, k = 500, 2000, 64, 64, 256
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3)
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": 6, "mlp_hidden_dim": 128, "skip_layer_idx": 3}).cuda()
    m.kernel_mode = "bf16"
    r = Renderer(m, None, eigenfunctions=E, H=Hh, W=Ww, device="cuda")
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    hit = torch.from_numpy(np.sort(rng.choice(Hh * Ww, N, replace=False)))
    monkeypatch.setenv("INF_RENDER_PROJECT", "1")
    a = r.render_hits(vids, bary, hit)
    monkeypatch.setenv("INF_RENDER_PROJECT", "0")
    b = r.render_hits(vids, bary, hit)
    np.testing.assert_allclose(a, b, atol=5e-3)


@pytest.mark.parametrize("L,s", [(3, 1), (4, 1), (4, 2), (5, 3), (6, 4), (8, 4)])
def test_render_projected_layer_schedules(L, s):
    """rproj's loader/compute barrier schedule for every depth / skip position class: one
    hidden layer (all row groups in extra intervals), the skip layer last (W_y half after
    the final hidden layer), the defaults; 40k hits so every workgroup pipelines several
    tiles (the loader's next-tile work runs)."""
    import model as M
    from inf_hip import runtime
    rng = np.random.default_rng(10 + L)
    k, H, V, N, HW = 256, 128, 3000, 40_000, 65536
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3).cuda()
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    hit = torch.from_numpy(np.sort(rng.choice(HW, N, replace=False))).cuda()
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
    m.kernel_mode = "bf16"
    w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
    src = runtime.RaySource(E, vids.cuda(), bary.cuda(), None)
    img = _render(m, src, hit, HW, chunk=4096, project=True).cpu().numpy()
    img_g = _render(m, src, hit, HW, chunk=4096).cpu().numpy()
    np.testing.assert_allclose(img, img_g, atol=5e-3)
    hit_np = hit.cpu().numpy()
    X = O.gather(E.cpu().numpy(), vids.numpy(), bary.numpy())
    p_ref, _ = O.mlp_forward(w, X, L, s)
    assert np.abs(img[hit_np] - p_ref).max() < 2e-2


def test_renderer_projection_cache_follows_weights(monkeypatch):
    """Renderer.render_hits keeps the projected table across frames while the plan's weight
    generation is unchanged, and recomputes it after a device-side training step (the
    cached frame would otherwise show the old weights) and after host-side edits."""
    import model as M
    from inf_hip import runtime
    from renderer import Renderer
    rng = np.random.default_rng(9)
    V, N, Hh, Ww, k = 500, 2000, 64, 64, 256
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3)
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": 6, "mlp_hidden_dim": 128, "skip_layer_idx": 3}).cuda()
    m.kernel_mode = "bf16"
    m.hip_runtime().ensure_optimizer_arenas()
    r = Renderer(m, None, eigenfunctions=E, H=Hh, W=Ww, device="cuda")
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    hit = torch.from_numpy(np.sort(rng.choice(Hh * Ww, N, replace=False)))
    monkeypatch.setenv("INF_RENDER_PROJECT", "1")
    a = r.render_hits(vids, bary, hit)
    cached = r._table_cache["proj"]
    assert cached is not None and cached[1] >= 0
    a2 = r.render_hits(vids, bary, hit)
    assert r._table_cache["proj"][3] is cached[3]  # reused, not recomputed
    np.testing.assert_array_equal(a, a2)
    # a device-side Adam step through the same plan
    plan = m.hip_plan(N)
    plan.set_lr(3e-2)
    src = runtime.RaySource(E.cuda(), vids.cuda(), bary.cuda(), torch.rand((N, 3), device="cuda"))
    for _ in range(3):
        plan.train_step(plan.make_batch(source=src, batch=N, loss_count=3 * N), None, apply_adam=True)
    b = r.render_hits(vids, bary, hit)
    assert r._table_cache["proj"][3] is not cached[3]
    monkeypatch.setenv("INF_RENDER_PROJECT", "0")
    b_gather = r.render_hits(vids, bary, hit)
    np.testing.assert_allclose(b, b_gather, atol=5e-3)
    assert np.abs(b - a).max() > 2e-2  # the steps moved the frame
    # host-side edit of the parameters (sync_shadow through hip_plan)
    monkeypatch.setenv("INF_RENDER_PROJECT", "1")
    with torch.no_grad():
        for p in m.parameters():
            p.mul_(0.5)
    c = r.render_hits(vids, bary, hit)
    monkeypatch.setenv("INF_RENDER_PROJECT", "0")
    c_gather = r.render_hits(vids, bary, hit)
    np.testing.assert_allclose(c, c_gather, atol=5e-3)


@pytest.mark.parametrize("k,H,L,s,V,N", [(1024, 256, 8, 4, 20000, 8192), (64, 128, 4, 2, 2000, 4096)])
def test_projected_render_matches_bf16_oracle(k, H, L, s, V, N):
    """The projected-table render (inf_project_table + csrc/rproj.hip) against an independent
    restatement of its bf16 arithmetic (oracle.mlp_forward_bf16_projected), not against the
    builder's own feature-gather chain."""
    import model as M
    from inf_hip import runtime
    rng = np.random.default_rng(41)
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
    m.kernel_mode = "bf16"
    w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    vids = rng.integers(0, V, (N, 3))
    bary = rng.dirichlet([1, 1, 1], N).astype(np.float32)
    src = runtime.RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(),
                            None)
    plan = m.hip_plan(min(N, 4096))
    P = plan.project_table(src.table_for(plan))
    pred = torch.empty((N, 3), device="cuda")
    plan.forward(plan.make_batch(source=src, batch=N, projected=P), pred, save=False)
    ref = O.mlp_forward_bf16_projected(w, E, vids, bary, L, s)
    err = float(np.abs(pred.cpu().numpy() - ref).max())
    print("projected vs bf16 oracle", k, H, L, s, err)
    assert err < PROJ_BF16_ORACLE_RGB, err


PROJ_BF16_ORACLE_RGB = 1e-3  # seen 1.7e-4 (k=1024, 8 x 256) / 5e-5 (k=64); profiles/r02/bf16_oracle_parity_render.log


@pytest.mark.parametrize("N,bad", [(1, False), (1000, True), (33_077, False), (200_000, True)])
def test_rprojw_matches_rproj(N, bad, monkeypatch):
    """rprojw.hip (128-ray tiles, the default for the 8 x 256 field with skip 4) against
    rproj.hip's 64-ray tiles (INF_RPROJ_WIDE=0) on the same projected batches.  Up to the
    last hidden layer both run the same arithmetic (the rows' fp32 fold and one bf16
    rounding, the MFMA k order, the epilogues); the head then sums W7 h in another fp32
    order (MFMAs over W7's bf16 hi + lo parts, 2^-17 of |W7| left out) -- RGB within 5e-5
    (seen below 1e-6), the background bitwise.  N = 1 (one tile), 1000 with out-of-range
    vertex ids and ray-index values (zero rows), 33,077 (259 tiles: a second tile on a few
    workgroups, a ragged last one), 200,000 (about 6 tiles per workgroup: the loader's
    zy / records / z0 pipeline across tiles).  The first workgroup's stamps tell which
    kernel ran: 14 stamped barriers per 128-ray tile."""
    import ctypes
    import model as M
    from inf_hip import lib, runtime
    rng = np.random.default_rng(50 + N)
    k, H, L, s, V, HW = 1024, 256, 8, 4, 5000, 1 << 19
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
    m.kernel_mode = "bf16"
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32) * 0.3).cuda()
    vids = rng.integers(0, V, (N, 3))
    perm = torch.from_numpy(rng.permutation(N))
    if bad:
        vids[7 % N, 1] = V + 5
        perm[::131] = N + 7
    bary = rng.dirichlet([1, 1, 1], N).astype(np.float32)
    hit = torch.from_numpy(np.sort(rng.choice(HW, N, replace=False))).cuda()
    src = runtime.RaySource(E, torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(), None,
                            validate=not bad)
    plan = m.hip_plan(4096)
    P = plan.project_table(src.table_for(plan))
    out = {}
    for wide in ("1", "0"):
        monkeypatch.setenv("INF_RPROJ_WIDE", wide)
        pred = torch.empty((N, 3), device="cuda")
        plan.forward(plan.make_batch(source=src, batch=N, ray_idx=perm.cuda(), projected=P), pred, save=False)
        img = torch.ones((HW, 3), device="cuda")
        st = torch.zeros(2 * 68, dtype=torch.int64, device="cuda")
        lib.inf_debug_timing(plan.handle, ctypes.c_void_p(st.data_ptr()), 0)
        plan.render(plan.make_batch(source=src, batch=N, projected=P), hit, None, img)
        torch.cuda.synchronize()
        lib.inf_debug_timing(plan.handle, None, 0)
        nst = int((st[:68] != 0).sum())
        if wide == "1":  # the first workgroup's tiles (ntile // grid of them), two stamped
            ntile = -(-N // 128)
            want = 3 + 14 * min(2, ntile // min(ntile, 256))
            assert nst == want, (nst, want)
        out[wide] = (pred.cpu().numpy(), img.cpu().numpy())
    assert np.isfinite(out["1"][0]).all()
    err_p = float(np.abs(out["1"][0] - out["0"][0]).max())
    err_i = float(np.abs(out["1"][1] - out["0"][1]).max())
    print("rprojw vs rproj", N, err_p, err_i)
    assert err_p < 5e-5 and err_i < 5e-5, (err_p, err_i)
    assert (out["1"][1] == 1.0).sum() == (out["0"][1] == 1.0).sum() == out["1"][1].size - 3 * N
