"""The view-dependent texture field (reference model.py:115-191, make_model :240-256) on the
generic dense kernels (csrc/dense.hip) against the reference's own outputs (G11:
seed-0 init, forward, one L1 Adam step; intrinsic and extrinsic view strategies).
Tolerances: RGB 1e-5 abs, L1 loss 1e-6, gradients 1e-4 of each tensor's max, weights
after one Adam step (lr 1e-3) 1e-5 abs."""
import types

import numpy as np
import pytest
import torch

from conftest import golden
from oracle import inf_oracle as O

pytestmark = pytest.mark.gpu


def cfg_of(strategy):
    dview = 1 if strategy == "intrinsic" else 3
    return {"model": {"k": 64, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2,
                      "view_dependence": {"bottleneck_vec_dim": 16, "in_dim_view_dir": dview,
                                          "include_view_dir": True, "embed_size": 4, "directional_hidden_dim": 32,
                                          "strategy": strategy}},
            "training": {"lr": 1e-3, "loss_type": "L1"}}


@pytest.mark.parametrize("strategy", ["intrinsic", "extrinsic"])
def test_viewdep_forward_and_step_match_reference(strategy):
    import config
    from trainer import Trainer
    d = golden(f"g11_viewdep_{strategy}.npz")
    mesh = types.SimpleNamespace(face_normals=d["normals"].astype(np.float64))
    cfg = cfg_of(strategy)
    torch.manual_seed(0)
    model, optim = config.get_model_and_optim(cfg, mesh, "cuda")
    batch = {"eigenfunctions": torch.from_numpy(d["features"]).cuda(), "unit_ray_dirs": torch.from_numpy(d["dirs"]).cuda(),
             "hit_face_idxs": torch.from_numpy(d["faces"]).cuda(), "expected_rgbs": torch.from_numpy(d["rgb"]).cuda()}
    with torch.no_grad():
        pred = model(batch).cpu().numpy()
    np.testing.assert_allclose(pred, d["pred"], atol=1e-5)
    loss_fn = config.get_loss_fn(cfg)
    p = model(batch)
    lval = loss_fn(p, batch["expected_rgbs"])
    optim.zero_grad(set_to_none=True)
    lval.backward()
    assert abs(lval.item() - float(d["loss"])) < 1e-6
    for n, prm in model.named_parameters():
        ref = d["g:" + n]
        err = np.abs(prm.grad.cpu().numpy() - ref).max() / max(np.abs(ref).max(), 1e-12)
        assert err < 1e-4, (n, err)
    optim.step()
    for n, prm in model.named_parameters():
        np.testing.assert_allclose(prm.detach().cpu().numpy(), d["w1:" + n], atol=1e-5, err_msg=n)
    # the trainer's (non-fused) step on a fresh model: the same first step
    torch.manual_seed(0)
    m2, o2 = config.get_model_and_optim(cfg, mesh, "cuda")
    tr = Trainer.__new__(Trainer)
    tr.model, tr.optim, tr.loss_fn, tr.device = m2, o2, loss_fn, "cuda"
    assert not tr._can_fuse(batch)
    loss, _ = tr._train_step(batch)
    assert abs(loss - float(d["loss"])) < 1e-6


def test_viewdep_state_dict_roundtrip_and_cpu_refusal(tmp_path):
    import model as M
    d = golden("g11_viewdep_intrinsic.npz")
    mesh = types.SimpleNamespace(face_normals=d["normals"].astype(np.float64))
    torch.manual_seed(0)
    m = M.make_model(cfg_of("intrinsic")["model"], mesh=mesh)
    torch.save(m.state_dict(), tmp_path / "m.pt")
    m2 = M.make_model(cfg_of("intrinsic")["model"], mesh=mesh)
    m2.load_state_dict(torch.load(tmp_path / "m.pt", weights_only=True))
    with pytest.raises(RuntimeError, match="HIP"):
        m2({"eigenfunctions": torch.zeros(4, 64), "unit_ray_dirs": torch.zeros(4, 3),
            "hit_face_idxs": torch.zeros(4, dtype=torch.int64)})


def test_viewdep_render_matches_model_on_hits():
    """Renderer.render of a view-dependent field: the device cast, then model(batch) on the
    hits (features, directions, faces) placed into the white image (renderer.py:64-146)."""
    import mesh as MS
    import model as M
    from oracle import raycast_oracle as R
    from renderer import Renderer
    V, F = R.icosphere(2)
    tri = V[F]
    n = np.cross(tri[:, 1] - tri[:, 0], tri[:, 2] - tri[:, 0])
    mesh = MS.TriMesh(V, F)
    mesh.face_normals = n / np.linalg.norm(n, axis=1, keepdims=True)
    torch.manual_seed(0)
    m = M.make_model(cfg_of("intrinsic")["model"], mesh=mesh).cuda().eval()
    E = torch.randn((V.shape[0], 64))
    H = W = 32
    r = Renderer(m, mesh, eigenfunctions=E, H=H, W=W, device="cuda")
    cam = np.concatenate([np.eye(3), np.array([[0.0], [0.0], [-3.0]])], 1)
    K = np.array([[32.0, 0, 16], [0, 32.0, 16], [0, 0, 1]])
    c, Kt = torch.tensor(cam).float(), torch.tensor(K).float()
    img = r.render(c, Kt)
    vids, bary, hit, face, dirs = MS.cast_camera_rays(r.ray_mesh_intersector, c, Kt, None, H=H, W=W)
    from inf_hip import runtime
    feats = runtime.gather(E.cuda(), vids, bary)
    with torch.no_grad():
        pred = m({"eigenfunctions": feats, "unit_ray_dirs": dirs[hit], "hit_face_idxs": face}).cpu().numpy()
    flat = img.reshape(-1, 3)
    np.testing.assert_allclose(flat[hit.cpu().numpy()], pred, atol=1e-6)
    miss = np.ones(H * W, bool)
    miss[hit.cpu().numpy()] = False
    assert hit.numel() > 100 and (flat[miss] == 1.0).all()


@pytest.mark.parametrize("name,L,s", [("A", 4, 2), ("R", 6, 3), ("B", 8, 4)])
def test_concat_layer_standalone(name, L, s):
    """LinearWithConcatAndActivation called on its own (layers.py:60-62) with the G2
    weights: its output on the G2 features' skip-layer input matches the oracle's skip
    layer (fp32 dense kernels, <= 1e-5), and autograd's gradients match the oracle's
    (relu' masked) products."""
    from layers import LinearWithConcatAndActivation
    d = golden(f"g2_forward_{name}.npz")
    w = {k[2:]: d[k] for k in d.files if k.startswith("w:")}
    x = d["features"]
    _, cache = O.mlp_forward(w, x, L, s)
    h_in, ref = cache["in"][s], cache["out"][s]
    H, k = w[f"layers.{s}.Lx.weight"].shape[0], x.shape[1]
    layer = LinearWithConcatAndActivation(H, k, H).cuda()
    with torch.no_grad():
        for sub in ("Lx", "Ly"):
            getattr(layer, sub).weight.copy_(torch.from_numpy(w[f"layers.{s}.{sub}.weight"]))
            getattr(layer, sub).bias.copy_(torch.from_numpy(w[f"layers.{s}.{sub}.bias"]))
    hx = torch.from_numpy(h_in).cuda().requires_grad_(True)
    xx = torch.from_numpy(x).cuda().requires_grad_(True)
    out = layer(hx, xx)
    np.testing.assert_allclose(out.detach().cpu().numpy(), ref, atol=1e-5)
    g = np.random.default_rng(1).standard_normal(ref.shape).astype(np.float32)
    out.backward(torch.from_numpy(g).cuda())
    dz = g * (cache["z"][s] > 0)
    np.testing.assert_allclose(layer.Lx.weight.grad.cpu().numpy(), dz.T @ h_in, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(layer.Ly.weight.grad.cpu().numpy(), dz.T @ x, rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(layer.Lx.bias.grad.cpu().numpy(), dz.sum(0), rtol=1e-4, atol=1e-4)
    np.testing.assert_allclose(hx.grad.cpu().numpy(), dz @ w[f"layers.{s}.Lx.weight"], rtol=1e-4, atol=1e-5)
    np.testing.assert_allclose(xx.grad.cpu().numpy(), dz @ w[f"layers.{s}.Ly.weight"], rtol=1e-4, atol=1e-5)
