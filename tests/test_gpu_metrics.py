"""Device evaluation metrics (csrc/metrics.hip) against the oracle's restatement of
skimage's structural_similarity (PARITY UNPINNED: scikit-image is absent; the oracle is
pinned by known answers in test_oracle_golden.py) and against the reference's host psnr.
Tolerances: SSIM 1e-10 abs (both fp64, different summation order); PSNR 1e-5 dB (the
reference averages in fp32, the device in fp64)."""
import numpy as np
import pytest
import torch

from conftest import golden
from oracle import inf_oracle as O

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("H,W", [(7, 7), (37, 53), (512, 512), (130, 17)])
def test_ssim_matches_oracle(H, W):
    from inf_hip import runtime
    rng = np.random.default_rng(H * 1000 + W)
    a = rng.random((H, W, 3)).astype(np.float32)
    b = np.clip(a + 0.2 * rng.standard_normal(a.shape), 0, 1).astype(np.float32)
    b[: H // 3] = 1.0  # a flat (white background) band: zero-variance windows
    a[: H // 4] = 1.0
    got = runtime.ssim(torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda())
    assert got == pytest.approx(O.structural_similarity(a, b), abs=1e-10)


def test_dssim_wrapper_and_uint8_range():
    import evaluation_metrics as em
    rng = np.random.default_rng(1)
    a = rng.random((64, 48, 3)).astype(np.float32)
    b = rng.random((64, 48, 3)).astype(np.float32)
    assert em.dssim(a, b) == pytest.approx(O.dssim(a, b), abs=1e-10)
    assert em.dssim(a, a) == pytest.approx(0.0, abs=1e-12)
    a8 = (a * 255).astype(np.uint8)
    b8 = (b * 255).astype(np.uint8)
    assert em.dssim(a8, b8) == pytest.approx(O.dssim(a8, b8, data_range=255.0), abs=1e-10)
    with pytest.raises(Exception):
        em.dssim(a[:5, :5], b[:5, :5])  # smaller than the 7 x 7 window


def test_device_psnr_matches_reference():
    import evaluation_metrics as em
    d = golden("g6_psnr.npz")
    a, b, m = d["a"], d["b"], d["mask"]
    ta, tb = torch.from_numpy(a).cuda(), torch.from_numpy(b).cuda()
    assert em.psnr(ta, tb) == pytest.approx(float(d["psnr_full"]), abs=1e-5)  # fp32 vs fp64 mean
    assert em.psnr(ta, tb, torch.from_numpy(m)) == pytest.approx(float(d["psnr_mask"]), abs=1e-5)
    assert em.psnr(ta, ta) == float("inf")


def test_evaluate_view_end_to_end():
    """eval.py's per-view metrics on a rendered icosphere view against the oracle metrics
    of the same rendered image."""
    import evaluation_metrics as em
    import mesh as MS
    import model as M
    from oracle import raycast_oracle as R
    from renderer import Renderer
    V, F = R.icosphere(2)
    torch.manual_seed(0)
    m = M.make_model({"feature_strategy": "xyz", "k": 3, "num_layers": 4, "mlp_hidden_dim": 64, "skip_layer_idx": 2,
                      "kernels": {"mode": "fp32"}}).cuda()
    m.kernel_mode = "fp32"
    H = W = 40
    r = Renderer(m, MS.TriMesh(V, F), feature_strategy="xyz", device="cuda", H=H, W=W)
    cam = np.concatenate([np.eye(3), np.array([[0.0], [0.0], [-3.0]])], 1)
    K = np.array([[40.0, 0, 20], [0, 40.0, 20], [0, 0, 1]])
    rng = np.random.default_rng(3)
    real = rng.random((H, W, 3)).astype(np.float32)
    mask = np.ones(H * W, dtype=bool)
    mask[:40] = False
    met, raw, fake, real_w = em.evaluate_view(r, torch.tensor(cam).float(), torch.tensor(K).float(), real, mask)
    assert (fake[0, 0] == 1).all() and (real_w[0, 0] == 1).all()
    sel = ~np.all(fake.reshape(-1, 3) == 1.0, axis=1)
    assert sel.sum() > 100
    assert met["dssim_rescaled"] == pytest.approx(O.dssim(fake, real_w) * 100, abs=1e-8)
    hit_mask = np.zeros(H * W, bool)
    _, _, hit, _ = R.ray_mesh_intersect(V, F, *R.create_ray_origins_and_directions(cam, K, None, H, W))
    hit_mask[hit] = True
    m2 = hit_mask & mask
    mse = np.mean((fake.reshape(-1, 3)[m2] - real_w.reshape(-1, 3)[m2]) ** 2)
    assert abs(met["psnr"] - 20 * np.log10(1 / np.sqrt(mse))) < 0.05  # a grazing ray may flip
