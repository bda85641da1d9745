"""CPU oracle for the render path's ray casting.

TEST INFRASTRUCTURE ONLY: imported by tests/ and bench.py's CPU baseline, never by the
product path (intrinsic-neural-fields_amd/), which casts on the GPU (csrc/raycast.hip).

A numpy float64 restatement of the reference's camera rays and closest-hit ray-mesh
intersection.  The reference intersects with trimesh + pyembree (closest hit,
`multiple_hits=False`, two-sided, t > 0) and then computes the hit point's barycentric
coordinates with `trimesh.triangles.points_to_barycentric(..., method='cramer')`.
Neither trimesh nor embree is installed here, so the INTERSECTION (closest_hits,
points_to_barycentric_cramer) is PARITY UNPINNED: checked by known-answer cases
(tests/test_oracle_raycast.py) and analytic geometry only.  The camera-ray generation is
PINNED: create_ray_origins_and_directions matches the reference's own (pure torch,
mesh.py:171-207) run by tests/golden/make_golden.py (G15) within 2e-7
(tests/test_oracle_fixtures_f.py).
"""
from __future__ import annotations

import numpy as np


def create_ray_origins_and_directions(camCv2world, K, mask_1d, H: int, W: int):
    """mesh.py:171-207 without lens distortion.  Pixels (x, y) in row-major order
    (torch.meshgrid indexing='xy' reshaped to H*W x 2), the obj_mask_1d-selected ones, as
    rays from the camera centre camCv2world[:, 3] along R K^-1 [x y 1], normalised."""
    cam = np.asarray(camCv2world, dtype=np.float64)
    Kk = np.asarray(K, dtype=np.float64)[:3, :3]
    xs, ys = np.meshgrid(np.arange(W), np.arange(H), indexing="xy")
    coord = np.stack([xs, ys], -1).reshape(-1, 2).astype(np.float64)
    mask = np.ones(H * W, dtype=bool) if mask_1d is None else np.asarray(mask_1d, dtype=bool)
    sel = coord[mask]
    hom = np.concatenate([sel, np.ones((sel.shape[0], 1))], -1)
    dirs = (cam[:3, :3] @ (np.linalg.inv(Kk) @ hom.T)).T
    unit = dirs / np.linalg.norm(dirs, axis=-1, keepdims=True)
    origins = np.broadcast_to(cam[:, 3], unit.shape).copy()
    return origins, unit


def points_to_barycentric_cramer(tri: np.ndarray, pts: np.ndarray) -> np.ndarray:
    """trimesh.triangles.points_to_barycentric(method='cramer') as used at mesh.py:224:
    Cramer's rule on the Gram system of the edges (a, b, c) -> (u, v, w), u = 1 - v - w."""
    a, b, c = tri[:, 0], tri[:, 1], tri[:, 2]
    v0, v1, v2 = b - a, c - a, pts - a
    d00 = (v0 * v0).sum(-1)
    d01 = (v0 * v1).sum(-1)
    d11 = (v1 * v1).sum(-1)
    d20 = (v2 * v0).sum(-1)
    d21 = (v2 * v1).sum(-1)
    den = d00 * d11 - d01 * d01
    v = (d11 * d20 - d01 * d21) / den
    w = (d00 * d21 - d01 * d20) / den
    return np.stack([1.0 - v - w, v, w], -1)


def closest_hits(vertices, faces, origins, dirs, chunk: int = 256):
    """Closest intersection t > 0 of every ray with any face (two-sided Moller-Trumbore in
    float64, brute force).  Returns face ids (-1 = miss) and t per ray."""
    V = np.asarray(vertices, dtype=np.float64)
    F = np.asarray(faces, dtype=np.int64)
    O = np.asarray(origins, dtype=np.float64)
    D = np.asarray(dirs, dtype=np.float64)
    v0 = V[F[:, 0]]
    e1 = V[F[:, 1]] - v0
    e2 = V[F[:, 2]] - v0
    n = O.shape[0]
    face = np.full(n, -1, dtype=np.int64)
    tbest = np.full(n, np.inf)
    for lo in range(0, n, chunk):
        o = O[lo:lo + chunk, None, :]
        d = D[lo:lo + chunk, None, :]
        p = np.cross(d, e2[None])
        det = (e1[None] * p).sum(-1)
        ok = np.abs(det) > 1e-30
        inv = np.where(ok, 1.0 / np.where(ok, det, 1.0), 0.0)
        s = o - v0[None]
        u = (s * p).sum(-1) * inv
        q = np.cross(s, e1[None])
        v = (d * q).sum(-1) * inv
        t = (e2[None] * q).sum(-1) * inv
        hit = ok & (u >= 0) & (v >= 0) & (u + v <= 1) & (t > 0)
        t = np.where(hit, t, np.inf)
        j = np.argmin(t, axis=1)
        tb = t[np.arange(t.shape[0]), j]
        has = np.isfinite(tb)
        face[lo:lo + chunk] = np.where(has, j, -1)
        tbest[lo:lo + chunk] = tb
    return face, tbest


def ray_mesh_intersect(vertices, faces, origins, dirs):
    """mesh.py:210-251 (return_depth=False): the hit rays' face vertex ids, the Cramer
    barycentrics of the intersection points, hit_ray_idxs and face_idxs, in ray order."""
    V = np.asarray(vertices, dtype=np.float64)
    F = np.asarray(faces, dtype=np.int64)
    face, t = closest_hits(V, F, origins, dirs)
    hit_ray_idxs = np.nonzero(face >= 0)[0]
    face_idxs = face[hit_ray_idxs]
    locs = np.asarray(origins, dtype=np.float64)[hit_ray_idxs] + t[hit_ray_idxs, None] * np.asarray(
        dirs, dtype=np.float64)[hit_ray_idxs]
    vids = F[face_idxs]
    bary = points_to_barycentric_cramer(V[vids], locs)
    return vids, bary, hit_ray_idxs, face_idxs


def icosphere(subdivisions: int = 2, radius: float = 1.0):
    """Test geometry: a subdivided icosahedron (vertices on the sphere), faces CCW."""
    t = (1.0 + 5 ** 0.5) / 2.0
    verts = [(-1, t, 0), (1, t, 0), (-1, -t, 0), (1, -t, 0), (0, -1, t), (0, 1, t), (0, -1, -t), (0, 1, -t),
             (t, 0, -1), (t, 0, 1), (-t, 0, -1), (-t, 0, 1)]
    faces = [(0, 11, 5), (0, 5, 1), (0, 1, 7), (0, 7, 10), (0, 10, 11), (1, 5, 9), (5, 11, 4), (11, 10, 2),
             (10, 7, 6), (7, 1, 8), (3, 9, 4), (3, 4, 2), (3, 2, 6), (3, 6, 8), (3, 8, 9), (4, 9, 5), (2, 4, 11),
             (6, 2, 10), (8, 6, 7), (9, 8, 1)]
    V = [np.asarray(v, dtype=np.float64) / np.linalg.norm(v) for v in verts]
    for _ in range(subdivisions):
        cache = {}

        def mid(i, j):
            key = (min(i, j), max(i, j))
            if key not in cache:
                m = V[i] + V[j]
                V.append(m / np.linalg.norm(m))
                cache[key] = len(V) - 1
            return cache[key]
        nf = []
        for a, b, c in faces:
            ab, bc, ca = mid(a, b), mid(b, c), mid(c, a)
            nf += [(a, ab, ca), (b, bc, ab), (c, ca, bc), (ab, bc, ca)]
        faces = nf
    return np.asarray(V) * radius, np.asarray(faces, dtype=np.int64)
