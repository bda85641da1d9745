"""The §8(f) oracles against fixtures produced by the reference itself
(tests/golden/make_golden.py, G14 / G15): the texture bake's texel search, barycentrics
and hole filling (bake_texture_field.py:134-264, 356-397: get_tris_fast, bary_matched,
uv_fill_holes, run in the reference's float128) and the camera-ray generation
(mesh.py:171-207 create_ray_origins_and_directions).  CPU only: the oracles are the
checkers of the GPU tests (tests/test_gpu_bake.py, tests/test_gpu_raycast.py)."""
import numpy as np
import pytest

from oracle import bake_oracle as B
from oracle import raycast_oracle as R


def uv_px(d):
    H, W = int(d["H"]), int(d["W"])
    return np.stack([(W - 1) * d["uv"][:, 0], (H - 1) * (1 - d["uv"][:, 1])], -1), H, W


def horizon_misses(face, ref):
    """Texels the reference leaves empty although a containing triangle exists: its
    get_tris_fast only tests the 10 nearest centroids (bake_texture_field.py:141-148)."""
    return (ref < 0) & (face >= 0)


@pytest.mark.parametrize("tag", ["grid", "jitter"])
def test_bake_oracle_matches_reference_g14(g, tag):
    d = g(f"g14_bake_{tag}.npz")
    uv, H, W = uv_px(d)
    face, bary = B.texel_faces(uv, d["faces"], H, W)
    ref = d["texel_face"]
    miss = horizon_misses(face, ref)
    assert miss.sum() == 0, int(miss.sum())  # these meshes keep every container within 10
    np.testing.assert_array_equal(face, ref)
    hit = ref >= 0
    np.testing.assert_allclose(bary[hit], d["texel_bary"][hit], atol=1e-12)
    assert 0.5 < hit.mean() < 1.0  # strict interiors leave the grid's edge texels empty
    np.testing.assert_allclose(B.uv_fill_holes(d["tex"]), d["tex_filled"], atol=1e-12)


def test_raygen_oracle_matches_reference_g15(g):
    import torch
    d = g("g15_raygen.npz")
    H, W = int(d["H"]), int(d["W"])
    for tag in ("full", "mask"):
        o, dirs = R.create_ray_origins_and_directions(torch.from_numpy(d["cam"]), torch.from_numpy(d["K"]),
                                                      torch.from_numpy(d[f"mask_{tag}"]), H, W)
        np.testing.assert_allclose(np.asarray(o), d[f"origins_{tag}"], atol=1e-6)
        np.testing.assert_allclose(np.asarray(dirs), d[f"dirs_{tag}"], atol=2e-7)
