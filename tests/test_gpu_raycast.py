"""GPU ray casting (csrc/raycast.hip) against the float64 CPU
oracle (oracle/raycast_oracle.py, parity unpinned: trimesh/embree are absent).

Bars: unit ray directions within 1e-6; hit/miss and hit face agree for >= 99.5 % of the
rays (fp32 vs fp64 can flip rays that graze an edge shared by two faces, or the mesh's
silhouette); barycentrics within 2e-4 where the face agrees; rendering through
Renderer.render equals rendering the oracle's hits wherever the two agree."""
import numpy as np
import pytest
import torch

from oracle import raycast_oracle as R

pytestmark = pytest.mark.gpu


def _scene(sub=4, seed=0):
    rng = np.random.default_rng(seed)
    V, F = R.icosphere(sub)
    V = V * (1.0 + 0.05 * rng.standard_normal((V.shape[0], 1)))  # no symmetric ties
    V = V @ np.diag([1.0, 0.8, 1.2]) + np.array([0.1, -0.05, 0.0])
    cam = np.concatenate([np.eye(3), [[0.0], [0.0], [-3.0]]], 1)
    K = np.array([[60.0, 0, 32], [0, 60, 32], [0, 0, 1]])
    return V, F, cam, K


def _compare(gpu, ref, L):
    vids_g, bary_g, hit_g, face_g = [t.cpu().numpy() for t in gpu]
    vids_r, bary_r, hit_r, face_r = ref
    fg = np.full(L, -1)
    fg[hit_g] = face_g
    fr = np.full(L, -1)
    fr[hit_r] = face_r
    agree = fg == fr
    assert agree.mean() >= 0.995, (agree.mean(), np.nonzero(~agree)[0][:10])
    assert (hit_g[1:] > hit_g[:-1]).all()  # ray order
    bg = np.zeros((L, 3))
    bg[hit_g] = bary_g
    br = np.zeros((L, 3))
    br[hit_r] = bary_r
    both = agree & (fg >= 0)
    assert both.sum() > 0.3 * L
    np.testing.assert_allclose(bg[both], br[both], atol=2e-4)
    vg = np.zeros((L, 3), dtype=np.int64)
    vg[hit_g] = vids_g
    vr = np.zeros((L, 3), dtype=np.int64)
    vr[hit_r] = vids_r
    np.testing.assert_array_equal(vg[both], vr[both])
    return agree


@pytest.mark.parametrize("masked", [False, True])
def test_camera_rays_match_oracle(masked):
    import mesh as MS
    V, F, cam, K = _scene()
    H = W = 64
    mask = None
    if masked:
        mask = np.random.default_rng(1).random(H * W) < 0.7
    bvh = MS.get_ray_mesh_intersector(MS.TriMesh(V, F))
    assert bvh.depth < 64 and bvh.num_nodes > 1
    vids, bary, hit, face, dirs = MS.cast_camera_rays(bvh, torch.from_numpy(cam).float(), torch.from_numpy(K).float(),
                                                      None if mask is None else torch.from_numpy(mask), H=H, W=W)
    o, d = R.create_ray_origins_and_directions(cam, K, mask, H, W)
    np.testing.assert_allclose(dirs.cpu().numpy(), d, atol=1e-6)
    _compare((vids, bary, hit, face), R.ray_mesh_intersect(V, F, o, d), d.shape[0])


def test_explicit_rays_match_oracle():
    import mesh as MS
    V, F, _, _ = _scene(3, seed=2)
    rng = np.random.default_rng(3)
    n = 3000
    o = rng.standard_normal((n, 3))
    o = 3.0 * o / np.linalg.norm(o, axis=-1, keepdims=True)
    tgt = 0.9 * rng.uniform(-1, 1, (n, 3))
    d = tgt - o
    d /= np.linalg.norm(d, axis=-1, keepdims=True)
    inter = MS.get_ray_mesh_intersector(MS.TriMesh(V, F))
    gpu = MS.ray_mesh_intersect(inter, None, torch.from_numpy(o), torch.from_numpy(d))
    _compare(gpu, R.ray_mesh_intersect(V, F, o.astype(np.float32), d.astype(np.float32)), n)
    # rays that miss everything and an empty ray list
    far = MS.ray_mesh_intersect(inter, None, torch.tensor([[0.0, 0, 10]]), torch.tensor([[0.0, 1.0, 0]]))
    assert far[2].numel() == 0
    empty = MS.ray_mesh_intersect(inter, None, torch.zeros((0, 3)), torch.zeros((0, 3)))
    assert empty[0].shape == (0, 3)


def test_render_end_to_end_matches_oracle_hits():
    """Renderer.render (camera rays cast on the device, then gather + MLP + scatter) vs
    render_hits of the oracle's hit lists: equal on every pixel whose hit agrees."""
    import mesh as MS
    import model as M
    from renderer import Renderer
    V, F, cam, K = _scene()
    H = W = 64
    k = 64
    rng = np.random.default_rng(4)
    E = torch.from_numpy(rng.standard_normal((V.shape[0], k)).astype(np.float32))
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2,
                      "kernels": {"mode": "fp32"}}).cuda()
    m.kernel_mode = "fp32"
    r = Renderer(m, MS.TriMesh(V, F), eigenfunctions=E, H=H, W=W, device="cuda")
    img = r.render(torch.from_numpy(cam).float(), torch.from_numpy(K).float())
    o, d = R.create_ray_origins_and_directions(cam, K, None, H, W)
    vids, bary, hit, face = R.ray_mesh_intersect(V, F, o, d)
    ref = r.render_hits(torch.from_numpy(vids), torch.from_numpy(bary).float(), torch.from_numpy(hit))
    fg = np.full(H * W, -1)
    _, _, hg, fcg, _ = MS.cast_camera_rays(r.ray_mesh_intersector, torch.from_numpy(cam).float(),
                                           torch.from_numpy(K).float(), None, H=H, W=W)
    fg[hg.cpu().numpy()] = fcg.cpu().numpy()
    fr = np.full(H * W, -1)
    fr[hit] = face
    same = (fg == fr).reshape(H, W)
    assert same.mean() >= 0.995
    np.testing.assert_allclose(img[same], ref[same], atol=1e-4)
    assert (img[fg.reshape(H, W) < 0] == 1.0).all()  # background where nothing is hit


def test_view_preprocessor_writes_reference_format(tmp_path):
    """mesh.MeshViewPreProcessor (mesh.py:430-548) on two synthetic views: the files that
    dataset.load_preprocessed_data reads, with the oracle's hits, colours and directions."""
    import dataset as DS
    import mesh as MS
    V, F, cam, K = _scene(3, seed=5)
    H = W = 48
    rng = np.random.default_rng(6)
    pre = MS.MeshViewPreProcessor(None, str(tmp_path / "train"), mesh=MS.TriMesh(V, F))
    views = []
    for v in range(2):
        th = 0.4 * v
        Rm = np.array([[np.cos(th), 0, np.sin(th)], [0, 1, 0], [-np.sin(th), 0, np.cos(th)]])
        c = np.concatenate([Rm, (Rm @ np.array([0.0, 0, -3.0]))[:, None]], 1)
        mask = rng.random((H, W)) < 0.8
        img = rng.random((H, W, 3)).astype(np.float32)
        pre.cache_single_view(torch.from_numpy(c).float(), torch.from_numpy(K).float(), torch.from_numpy(mask),
                              torch.from_numpy(img))
        views.append((c, mask, img))
    pre.write_to_disk()
    d = DS.load_preprocessed_data(str(tmp_path / "train"))
    assert np.load(tmp_path / "train" / "vids_of_hit_faces.npy").dtype == np.int32
    ref = {k: [] for k in ("v", "b", "c", "d", "f")}
    for c, mask, img in views:
        o, dd = R.create_ray_origins_and_directions(c, K, mask.reshape(-1), H, W)
        vids, bary, hit, face = R.ray_mesh_intersect(V, F, o, dd)
        ref["v"].append(vids)
        ref["b"].append(bary)
        ref["c"].append(img.reshape(-1, 3)[mask.reshape(-1)][hit])
        ref["d"].append(dd[hit])
        ref["f"].append(face)
    n_ref = sum(len(f) for f in ref["f"])
    n = d["face_idxs"].shape[0]
    assert abs(n - n_ref) <= 0.005 * n_ref
    if n == n_ref and np.array_equal(d["face_idxs"].numpy(), np.concatenate(ref["f"])):
        np.testing.assert_array_equal(d["vertex_idxs_of_hit_faces"].numpy(), np.concatenate(ref["v"]))
        np.testing.assert_allclose(d["barycentric_coords"].numpy(), np.concatenate(ref["b"]), atol=2e-4)
        np.testing.assert_allclose(d["expected_rgbs"].numpy(), np.concatenate(ref["c"]), atol=0)
        np.testing.assert_allclose(d["unit_ray_dirs"].numpy(), np.concatenate(ref["d"]), atol=1e-6)
    else:  # a grazing ray flipped: compare the colours as multisets of the agreeing part
        assert np.isin(d["face_idxs"].numpy(), np.concatenate(ref["f"])).mean() > 0.995


def test_row_sharded_render_assembles_to_full_frame():
    """dp.render_distributed's per-rank work: the row shards of a frame, each cast and
    shaded on its own (as ranks 0..2 would), assembled equal the single-rank render; at
    world size 1 render_distributed is Renderer.render on the device."""
    import dp
    import mesh as MS
    import model as M
    from renderer import Renderer
    V, F, cam, K = _scene()
    H, W = 50, 64
    rng = np.random.default_rng(8)
    E = torch.from_numpy(rng.standard_normal((V.shape[0], 64)).astype(np.float32))
    torch.manual_seed(0)
    m = M.make_model({"k": 64, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2,
                      "kernels": {"mode": "fp32"}}).cuda()
    m.kernel_mode = "fp32"
    r = Renderer(m, MS.TriMesh(V, F), eigenfunctions=E, H=H, W=W, device="cuda")
    c, Kt = torch.from_numpy(cam).float(), torch.from_numpy(K).float()
    full = r.render_device(c, Kt)
    parts = []
    for rank in range(3):
        lo, hi = dp.shard_span(H, rank, 3)
        mask = torch.zeros(H * W, dtype=torch.bool)
        mask[lo * W:hi * W] = True
        parts.append(r.render_device(c, Kt, obj_mask_1d=mask)[lo:hi])
    torch.testing.assert_close(torch.cat(parts), full, atol=0, rtol=0)
    torch.testing.assert_close(dp.render_distributed(r, c, Kt), full, atol=0, rtol=0)
    np.testing.assert_array_equal(r.render(c, Kt), full.cpu().numpy())


@pytest.mark.parametrize("tag", ["full", "mask"])
def test_camera_rays_match_reference_g15(g, tag):
    """The device's camera rays (R K^-1 [x y 1] per masked pixel, normalised) against the
    reference's own create_ray_origins_and_directions (mesh.py:171-207, fixture G15 made by
    importing the reference): a rotated camera, off-centre principal point."""
    import mesh as MS
    d = g("g15_raygen.npz")
    H, W = int(d["H"]), int(d["W"])
    V, F = R.icosphere(2)
    bvh = MS.get_ray_mesh_intersector(MS.TriMesh(V + 5.0, F))
    mask = d[f"mask_{tag}"]
    pix = torch.from_numpy(np.nonzero(mask)[0]).cuda()
    face, bary, dirs = bvh.cast(torch.from_numpy(d["cam"]), torch.from_numpy(d["K"]), H, W, pixel_idx=pix)
    np.testing.assert_allclose(dirs.cpu().numpy(), d[f"dirs_{tag}"], atol=1e-6)
