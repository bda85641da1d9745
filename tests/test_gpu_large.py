"""GPU parity at the large configurations of SURVEY.md §8(d): config D (human_dense,
k = 4096, 8x256 MLP, skip 4; configs/discretization_agnostic/human_dense.yaml) and a
config-B table above 2 GiB.

The tables are larger than 2 GiB in bf16 (one buffer descriptor with unsigned 32-bit
offsets serves tables below 4 GiB) and two are larger than 4 GiB, where the fused chain's
gather (csrc/chain3.hip) addresses rows with 64-bit offsets; at k = 4096 the 16-ray feature tile (128 KiB) does
not fit next to the chain's other LDS, so it is streamed in 1024-column chunks with both
input layers run over each chunk (chain3.hip, XC).  The oracle (oracle/inf_oracle.py) sees
only the table rows the sampled rays reference.  Tolerances are those of
test_gpu_kernels.py: fp32 mode RGB <= 1e-5 of the oracle and gradients <= 1e-4 of each
tensor's max; bf16 RGB <= 2e-2 and gradients <= 0.25 of max vs the oracle, and the fused
chain within 5e-4 RGB / 1e-2 of max gradients of the layered bf16 kernels."""
import numpy as np
import pytest
import torch

from oracle import inf_oracle as O

pytestmark = pytest.mark.gpu


def rt():
    from inf_hip import runtime
    return runtime


def seed0_weights(k, H, L, s):
    """The reference's seed-0 initialisation (model.py:194-258) of this architecture."""
    import model as M
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s})
    return {n: p.detach().numpy().copy() for n, p in m.named_parameters()}


def device_table(V, k, seed):
    """randn(V, k) with the reference's 'standard' column rescale (mesh.py:99-102), made on
    the device (a 300k x 4096 table is 4.9 GB in fp32)."""
    g = torch.Generator(device="cuda").manual_seed(seed)
    E = torch.randn((V, k), generator=g, device="cuda")
    E /= E.max(0, keepdim=True).values - E.min(0, keepdim=True).values
    return E


def run_step(w, k, H, L, s, mode, src, B, env, monkeypatch):
    for key in ("INF_NO_CHAIN3", "INF_NO_CHAIN"):
        monkeypatch.delenv(key, raising=False)
    for key in env:
        monkeypatch.setenv(key, "1")
    params = torch.cat([torch.from_numpy(w[n]).reshape(-1) for n in O.layer_names(L, s)]).cuda()
    plan = rt().Plan(k, H, L, s, mode, "L2", B, params, grads=torch.zeros_like(params),
                     exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
    pred = torch.empty((B, 3), device="cuda")
    plan.train_step(plan.make_batch(source=src, batch=B), pred, apply_adam=False)
    want = {"INF_NO_CHAIN": "layered", "INF_NO_CHAIN3": "chain"}
    # (k > 1024 at H = 256: zg.hip's gather + input GEMM ahead of the chain, the default)
    path = want[env[0]] if env else (("chain3_zg" if H == 256 else "chain3_chunked") if k > 1024 else "chain3") \
        if mode == "bf16" else "layered"
    assert plan.last_step_path() == path, (plan.last_step_path(), path)
    g = plan.grads.cpu().numpy()
    out, off = {}, 0
    for n in O.layer_names(L, s):
        out[n] = g[off:off + w[n].size].reshape(w[n].shape)
        off += w[n].size
    c = plan.read_ctrl()
    del plan
    torch.cuda.empty_cache()
    return pred.cpu().numpy(), out, c["loss_sum"], c["step"]


def oracle_step(w, E, vids, bary, rgb, L, s):
    """Oracle forward / backward on the rows the rays reference (fetched from the device)."""
    rows, inv = np.unique(vids.reshape(-1), return_inverse=True)
    E_sub = E[torch.from_numpy(rows).cuda()].cpu().numpy()
    X = O.gather(E_sub, inv.reshape(vids.shape), bary)
    _, cache = O.mlp_forward(w, X, L, s)
    p_ref = cache["out"][-1]
    g_ref = O.mlp_backward(w, cache, O.loss_grad(p_ref, rgb, "L2"), L, s)
    return p_ref, g_ref


def rays(rng, V, B):
    vids = rng.integers(0, V, (B, 3))
    vids[:8] = V - 1          # rows past the 2 GiB mark of the bf16 table
    vids[8:16, 0] = 0
    bary = rng.dirichlet([1, 1, 1], B).astype(np.float32)
    bary[16] = (1.0, 0.0, 0.0)  # an exact vertex hit
    rgb = rng.random((B, 3)).astype(np.float32)
    return vids, bary, rgb


def check(outs, p_ref, g_ref, rgb, L, s, B):
    errs = {}
    for tag, (p, g, lsum, step) in outs.items():
        assert step == 1, tag
        lim = 1e-5 if tag == "fp32" else 2e-2
        assert np.abs(p - p_ref).max() < lim, (tag, float(np.abs(p - p_ref).max()))
        assert abs(lsum / (3 * B) - O.loss_value(p_ref, rgb, "L2")) < (1e-6 if tag == "fp32" else 2e-3), tag
        for n in O.layer_names(L, s):
            scale = max(np.abs(g_ref[n]).max(), 1e-12)
            errs[(tag, n)] = float(np.abs(g[n] - g_ref[n]).max() / scale)
    print({f"{t}:{n}": round(e, 5) for (t, n), e in errs.items()})
    for (tag, n), e in errs.items():
        assert e < (1e-4 if tag == "fp32" else 0.25), (tag, n, e)
    if "layered" in outs:
        # the chunked schedule adds W_y x (K = 4096) to the skip layer's Lx h as a separate
        # fp32 sum, so a bf16 activation can round the other way and flip a ReLU: gradients
        # within 5e-2 of max (2.5e-2 seen on layers.4.Ly.weight at 1024 rays; both paths are
        # 0.1214 / 0.1213 of max from the oracle there), 1e-2 for the whole-tile chain
        gtol = 5e-2 if outs["chain3"][1]["layers.0.0.weight"].shape[1] > 1024 else 1e-2
        np.testing.assert_allclose(outs["chain3"][0], outs["layered"][0], atol=5e-4)
        for n in O.layer_names(L, s):
            scale = max(np.abs(outs["layered"][1][n]).max(), 1e-12)
            assert np.abs(outs["chain3"][1][n] - outs["layered"][1][n]).max() / scale < gtol, n


@pytest.mark.parametrize("B,V", [(1024, 300_000), (4096, 600_000)])
def test_config_d_k4096_large_table(B, V, monkeypatch):
    """Config D (k = 4096, 8 x 256, skip 4) on a 300k-vertex (2.46 GB in bf16) and a
    600k-vertex table (4.9 GB, above 4 GiB): the fused bf16 chain (chunked feature tile) and
    the layered bf16 (and fp32) kernels against the oracle."""
    k, H, L, s = 4096, 256, 8, 4
    rng = np.random.default_rng(40 + B)
    w = seed0_weights(k, H, L, s)
    E = device_table(V, k, seed=4)
    vids, bary, rgb = rays(rng, V, B)
    src = rt().RaySource(E, torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(), torch.from_numpy(rgb).cuda())
    outs = {"chain3": run_step(w, k, H, L, s, "bf16", src, B, (), monkeypatch),
            "layered": run_step(w, k, H, L, s, "bf16", src, B, ("INF_NO_CHAIN",), monkeypatch)}
    if B == 1024:
        outs["fp32"] = run_step(w, k, H, L, s, "fp32", src, B, (), monkeypatch)
    src._tables.clear()
    p_ref, g_ref = oracle_step(w, E, vids, bary, rgb, L, s)
    check(outs, p_ref, g_ref, rgb, L, s, B)


def test_config_b_table_over_4gib(monkeypatch):
    """k = 1024 with 2.2M vertices (a 4.5 GB bf16 table): the register-streamed chain keeps
    its whole-tile gather and must still reach every row (64-bit row addressing)."""
    k, H, L, s, V, B = 1024, 256, 8, 4, 2_200_000, 4096
    rng = np.random.default_rng(7)
    w = seed0_weights(k, H, L, s)
    E = device_table(V, k, seed=5)
    vids, bary, rgb = rays(rng, V, B)
    src = rt().RaySource(E, torch.from_numpy(vids).cuda(), torch.from_numpy(bary).cuda(), torch.from_numpy(rgb).cuda())
    outs = {"chain3": run_step(w, k, H, L, s, "bf16", src, B, (), monkeypatch),
            "layered": run_step(w, k, H, L, s, "bf16", src, B, ("INF_NO_CHAIN",), monkeypatch)}
    src._tables.clear()
    p_ref, g_ref = oracle_step(w, E, vids, bary, rgb, L, s)
    check(outs, p_ref, g_ref, rgb, L, s, B)
