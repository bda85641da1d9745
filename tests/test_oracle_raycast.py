"""The ray-casting oracle (oracle/raycast_oracle.py; parity unpinned: trimesh/embree are
absent and the reference holds no fixture for this path) against known answers, and the
product's OBJ / PLY mesh readers (mesh.load_mesh, host code) on files written here."""
import os
import struct
import sys

import numpy as np

from oracle import raycast_oracle as R

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "intrinsic-neural-fields_amd"))


def test_single_triangle_known_answer():
    V = np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0]])
    F = np.array([[0, 1, 2]])
    # rays straight down onto the z = 0 plane from z = 2 (and one from below: two-sided)
    O = np.array([[0.25, 0.25, 2.0], [0.1, 0.7, 2.0], [0.9, 0.9, 2.0], [0.2, 0.3, -1.0], [0.2, 0.2, -1.0]])
    D = np.array([[0, 0, -1.0], [0, 0, -1.0], [0, 0, -1.0], [0, 0, 1.0], [0, 0, -1.0]])
    vids, bary, hit, face = R.ray_mesh_intersect(V, F, O, D)
    assert hit.tolist() == [0, 1, 3]  # (0.9, 0.9) is outside; the last ray points away
    assert face.tolist() == [0, 0, 0]
    np.testing.assert_array_equal(vids, [[0, 1, 2]] * 3)
    np.testing.assert_allclose(bary, [[0.5, 0.25, 0.25], [0.2, 0.1, 0.7], [0.5, 0.2, 0.3]], atol=1e-12)


def test_closest_hit_wins():
    V = np.array([[0.0, 0, 0], [1, 0, 0], [0, 1, 0], [0, 0, 1], [1, 0, 1], [0, 1, 1]])
    F = np.array([[0, 1, 2], [3, 4, 5]])  # planes z = 0 and z = 1
    vids, bary, hit, face = R.ray_mesh_intersect(V, F, [[0.2, 0.2, 3.0], [0.2, 0.2, -3.0]], [[0, 0, -1.0], [0, 0, 1.0]])
    assert face.tolist() == [1, 0]


def test_camera_rays_pinhole():
    """mesh.py:171-207: identity rotation, camera at c: the ray through the principal point
    is +z, and pixel (x, y) points along ((x - cx) / fx, (y - cy) / fy, 1)."""
    K = np.array([[100.0, 0, 16], [0, 80, 12], [0, 0, 1]])
    cam = np.concatenate([np.eye(3), [[1.0], [2.0], [3.0]]], 1)
    H, W = 24, 32
    mask = np.zeros(H * W, dtype=bool)
    mask[[12 * W + 16, 5 * W + 7, 23 * W + 31]] = True
    o, d = R.create_ray_origins_and_directions(cam, K, mask, H, W)
    np.testing.assert_allclose(o, [[1, 2, 3]] * 3)
    for (x, y), u in zip([(7, 5), (16, 12), (31, 23)], d):
        v = np.array([(x - 16) / 100.0, (y - 12) / 80.0, 1.0])
        np.testing.assert_allclose(u, v / np.linalg.norm(v), atol=1e-12)


def test_icosphere_center_ray_hits_and_barycentrics_sum_to_one():
    V, F = R.icosphere(2)
    O = np.array([[0.0, 0, -5], [0.3, 0.2, -5], [5.0, 0, 0]])
    D = np.array([[0.0, 0, 1], [0.0, 0, 1], [-1.0, 0, 0]])
    vids, bary, hit, face = R.ray_mesh_intersect(V, F, O, D)
    assert hit.tolist() == [0, 1, 2]
    np.testing.assert_allclose(bary.sum(-1), 1.0, atol=1e-12)
    assert (bary >= -1e-12).all()
    # the hit points lie on the sphere's polyhedron, inside the unit ball, on the near side
    pts = (V[vids] * bary[..., None]).sum(1)
    assert (np.linalg.norm(pts, axis=-1) <= 1 + 1e-12).all() and pts[0, 2] < 0 and pts[2, 0] > 0


def test_mesh_readers_obj_ply(tmp_path):
    import mesh as MS
    V, F = R.icosphere(1)
    obj = tmp_path / "m.obj"
    with open(obj, "w") as fh:
        for v in V:
            fh.write(f"v {v[0]:.17g} {v[1]:.17g} {v[2]:.17g}\n")
        for f in F:
            fh.write(f"f {f[0] + 1}/1 {f[1] + 1}/1 {f[2] + 1}/1\n")
    m = MS.load_mesh(str(obj))
    np.testing.assert_allclose(m.vertices, V)
    np.testing.assert_array_equal(m.faces, F)
    ply = tmp_path / "m.ply"
    with open(ply, "wb") as fh:
        fh.write((f"ply\nformat binary_little_endian 1.0\nelement vertex {len(V)}\nproperty float x\n"
                  f"property float y\nproperty float z\nelement face {len(F)}\n"
                  "property list uchar int vertex_indices\nend_header\n").encode())
        fh.write(V.astype("<f4").tobytes())
        for f in F:
            fh.write(struct.pack("<B3i", 3, *f))
    m2 = MS.load_mesh(str(ply))
    np.testing.assert_allclose(m2.vertices, V.astype(np.float32))
    np.testing.assert_array_equal(m2.faces, F)


def test_bake_oracle_known_answers():
    """Texel search (strict interior: edge texels match nothing, as the reference's sign
    test), bary_matched reconstruction and hole filling on hand-checkable cases."""
    from oracle import bake_oracle as B
    uv = np.array([[0.0, 0.0], [4.0, 0.0], [0.0, 4.0], [4.0, 4.0]])
    faces = np.array([[0, 1, 2], [1, 3, 2]])
    face, bary = B.texel_faces(uv, faces, 5, 5)
    f = face.reshape(5, 5)
    assert f[1, 1] == 0 and f[3, 3] == 1 and f[0, 0] == -1 and f[2, 2] == -1  # (2,2) lies on the diagonal
    hit = face >= 0
    P = np.stack(np.meshgrid(np.arange(5), np.arange(5)), -1).reshape(-1, 2)[hit]
    rec = (bary[hit][:, :, None] * uv[faces[face[hit]]]).sum(1)
    np.testing.assert_allclose(rec, P, atol=1e-12)
    CC = np.zeros((5, 5, 3))
    CC[2, 2] = [0.5, 0.25, 1.0]
    out = B.uv_fill_holes(CC)
    np.testing.assert_allclose(out[2, 3], [0.5, 0.25, 1.0])  # one filled neighbour: its colour
    assert (out[0, 0] == 0.5 * np.array([1, 0.5, 2])).all()  # within the 5 x 5 reach
    np.testing.assert_array_equal(out[2, 2], CC[2, 2])


def test_uv_mesh_loader(tmp_path):
    import bake_texture_field as BK
    from oracle import bake_oracle as B
    text, P, F = B.grid_uv_scene(4)
    p = tmp_path / "grid.obj"
    p.write_text(text)
    m = BK.load_uv_mesh(str(p))
    assert m.faces.shape == F.shape and m.vertices.shape[0] == 4 * 16  # every cell its own 4 corners
    idx = BK.correspondences(m, np.round(P, 9))
    np.testing.assert_array_equal(idx[m.faces], F)
