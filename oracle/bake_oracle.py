"""CPU oracle for texture baking.

TEST INFRASTRUCTURE ONLY: imported by tests/, never by the product path, which bakes on
the GPU (csrc/bake.hip + the plan's render path).

A float64 numpy restatement of bake_texture_field.py's texel search (point_in_tri
:37-63 strict-interior test, clean_tris :96-112, nearest-centroid choice of
get_tris_fast :134-161 without its 10-candidate horizon), bary_matched (:196-228) and
uv_fill_holes (:245-264, scipy.signal.convolve2d as in the reference).  PINNED against the
reference's own get_tris_fast / bary_matched / uv_fill_holes run by
tests/golden/make_golden.py (G14: a regular and a jittered UV triangulation, the
reference's float128 arithmetic): identical texel -> triangle assignment, barycentrics
within 1e-12, hole filling within 1e-12 (tests/test_oracle_fixtures_f.py); plus known
answers in tests/test_oracle_raycast.py.  The reference's whole bake_texture still needs
trimesh (mesh + material loading) and cv2, absent here.
"""
from __future__ import annotations

import numpy as np


def _sign(p1, p2, p3):
    return (p1[..., 0] - p3[..., 0]) * (p2[..., 1] - p3[..., 1]) - (p2[..., 0] - p3[..., 0]) * (p1[..., 1] - p3[..., 1])


def texel_faces(uv_px: np.ndarray, faces: np.ndarray, H: int, W: int, min_area: float = 1e-4):
    """Per texel (row-major y * W + x): the strictly containing triangle of area >= min_area
    with the nearest centroid (ties: lowest index), -1 if none; and bary_matched (u, v, w)."""
    a, b, c = uv_px[faces[:, 0]], uv_px[faces[:, 1]], uv_px[faces[:, 2]]
    area = 0.5 * ((a[:, 0] - c[:, 0]) * (b[:, 1] - c[:, 1]) - (a[:, 1] - c[:, 1]) * (b[:, 0] - c[:, 0]))
    good = np.abs(area) >= min_area
    g = (a + b + c) / 3
    PX, PY = np.meshgrid(np.arange(W), np.arange(H))
    p = np.stack([PX.ravel(), PY.ravel()], -1).astype(np.float64)
    face = np.full(p.shape[0], -1, np.int64)
    best = np.full(p.shape[0], np.inf)
    for t in np.nonzero(good)[0]:
        d1 = _sign(p, a[t], b[t])
        d2 = _sign(p, b[t], c[t])
        d3 = _sign(p, c[t], a[t])
        inside = ~(((d1 <= 0) | (d2 <= 0) | (d3 <= 0)) & ((d1 >= 0) | (d2 >= 0) | (d3 >= 0)))
        dist = ((p - g[t]) ** 2).sum(-1)
        upd = inside & (dist < best)
        face[upd] = t
        best[upd] = dist[upd]
    bary = np.zeros((p.shape[0], 3))
    hit = face >= 0
    fa, fb, fc = a[face[hit]], b[face[hit]], c[face[hit]]
    v0, v1, v2 = fb - fa, fc - fa, p[hit] - fa
    d00, d01, d11 = (v0 * v0).sum(-1), (v0 * v1).sum(-1), (v1 * v1).sum(-1)
    d20, d21 = (v2 * v0).sum(-1), (v2 * v1).sum(-1)
    den = np.maximum(d00 * d11 - d01 * d01, 0)
    v = (d11 * d20 - d01 * d21) / den
    w = (d00 * d21 - d01 * d20) / den
    bary[hit] = np.stack([1 - v - w, v, w], -1)
    return face, bary


def uv_fill_holes(CC: np.ndarray) -> np.ndarray:
    """bake_texture_field.py:245-264."""
    from scipy.signal import convolve2d
    k = np.array([1., 4, 6, 4, 1])
    k = k[:, None] * k[None, :]
    k = k / k.sum()
    CCf = np.stack([convolve2d(CC[..., i], k, mode="same", boundary="fill", fillvalue=0.0) for i in range(3)], -1)
    out = np.copy(CC)
    mask = np.any(CC != 0, axis=-1)
    Wf = convolve2d(mask, k, mode="same", boundary="fill", fillvalue=0.0)
    fill = ~mask & (Wf > 0)
    out[fill] = CCf[fill] / Wf[fill, None]
    return out


def grid_uv_scene(n: int = 6, gap: float = 0.15, seed: int = 0):
    """Test geometry: an n x n height-field grid (two triangles per cell) whose UV map
    gives every cell its own island shrunk by `gap` (so the texture has holes between
    islands).  Returns the OBJ text and (positions, faces over positions)."""
    rng = np.random.default_rng(seed)
    xs = np.linspace(0, 1, n + 1)
    P = np.array([[x, y, 0.2 * np.sin(3 * x) * np.cos(2 * y) + 0.01 * rng.random()] for y in xs for x in xs])
    lines = [f"v {p[0]:.9f} {p[1]:.9f} {p[2]:.9f}" for p in P]
    faces, vt, fl = [], [], []
    for j in range(n):
        for i in range(n):
            c = [j * (n + 1) + i, j * (n + 1) + i + 1, (j + 1) * (n + 1) + i + 1, (j + 1) * (n + 1) + i]
            lo, hi = gap / n, (1 - gap) / n
            base = len(vt)
            for du, dv in ((lo, lo), (hi, lo), (hi, hi), (lo, hi)):
                vt.append((i / n + du, j / n + dv))
            for tri in ((0, 1, 2), (0, 2, 3)):
                faces.append([c[t] for t in tri])
                fl.append("f " + " ".join(f"{c[t] + 1}/{base + t + 1}" for t in tri))
    lines += [f"vt {u:.9f} {v:.9f}" for u, v in vt] + fl
    return "\n".join(lines) + "\n", P, np.asarray(faces, np.int64)
