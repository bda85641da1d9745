"""Host mirror of the reference mesh.py -- the hot-path subset.

* `load_first_k_eigenfunctions` (reference mesh.py:53-108) is the table producer: host
  numpy at setup time, exactly as in the reference (it runs once per loader).
* `get_k_eigenfunc_vec_vals` (mesh.py:313-324) and `get_k_eigenfunc_vec_vals_batched`
  (mesh.py:327-339) run the HIP gather kernel (csrc/gather.hip).  Unlike the reference's
  batched variant, which fills a host buffer, the batched form keeps the result on the
  table's device.

* Ray casting runs on the GPU (csrc/raycast.hip):
  `get_ray_mesh_intersector` builds a device BVH in place of trimesh/embree (mesh.py:111-117);
  `ray_mesh_intersect` / `ray_mesh_intersect_batched` (mesh.py:210-310) and `ray_tracing`
  (mesh.py:342-390) return the reference's hit lists (closest hit, two-sided, t > 0, Cramer
  barycentrics), in ray order, on the device.  `load_mesh` reads OBJ / PLY triangle meshes
  with numpy in place of igl (mesh.py:39-50).

The Laplace-Beltrami eigensolve, point clouds and lens undistortion (mesh.py:111-165,
392-605) need igl / scipy-sparse LBO tooling and stay out of scope.
"""
from __future__ import annotations

import numpy as np
import torch


def _first_k(values, k, axis):
    """Columns (axis 1) or entries (axis 0) `k` of a stored spectrum: an explicit index list,
    or the first k (which must be stored)."""
    if isinstance(k, list):
        return np.take(values, np.array(k), axis=axis)
    assert k <= values.shape[axis]
    return values[:, :k] if axis == 1 else values[:k]


def _spectrum(eigenvalues_path, k):
    """The eigenvalues matching the selected eigenfunctions, the first one's sign fixed (a
    tiny negative lambda_0 is solver noise); all must then be positive."""
    lam = np.load(eigenvalues_path)
    lam = _first_k(lam, k, axis=1 if isinstance(k, list) and lam.ndim > 1 else 0)
    if lam[0] < 0 and np.abs(lam[0]) < 1e-10:
        lam[0] *= -1
    assert np.all(lam > 0), f"Min value: {lam.min()}"
    return lam


def _heat_kernel_signature(phi, lam, ts):
    # sum_i phi_i(v)^2 exp(-lambda_i t) at ts log-spaced t in [1e-2, 1]
    t = np.logspace(-2, 0, num=ts)
    return (phi * phi) @ np.exp(-lam[..., None] @ t[None, ...])


def _column_range(phi):
    return np.max(phi, axis=0, keepdims=True) - np.min(phi, axis=0, keepdims=True)


_RESCALE = {
    "standard": lambda phi: phi / _column_range(phi),  # each column into a unit-width range
    "one-norm": lambda phi: phi / np.linalg.norm(phi, ord=2, axis=-1, keepdims=True),  # unit rows
    "unscaled": lambda phi: phi,
}


def load_first_k_eigenfunctions(eigenfunctions_path, k, rescale_strategy="standard", embed_strategy=None,
                                eigenvalues_path=None, ts=128):
    """The per-vertex input table (reference mesh.py:53-108): eigenfunction columns `k`, an
    optional spectral embedding -- "gps" (phi_i / sqrt(lambda_i / lambda_0), returned as is,
    a numpy array, like the reference) or "hks" (heat kernel signature) -- then a rescale.
    Same float64 expressions as the reference, so the table is bitwise the same."""
    phi = _first_k(np.load(eigenfunctions_path), k, axis=1)
    lam = _spectrum(eigenvalues_path, k) if eigenvalues_path is not None else None
    if embed_strategy == "gps":
        assert lam is not None
        w = np.sqrt(lam)
        w /= w[0]
        return phi / w
    if embed_strategy == "hks":
        assert lam is not None
        phi = _heat_kernel_signature(phi, lam, ts)
    elif embed_strategy is not None:
        raise ValueError(f"Unknown embedding strategy {embed_strategy}")
    if rescale_strategy not in _RESCALE:
        raise RuntimeError(f"Unknown rescaling strategy: {rescale_strategy}")
    return torch.from_numpy(np.ascontiguousarray(_RESCALE[rescale_strategy](phi))).to(dtype=torch.float32)


def get_k_eigenfunc_vec_vals(E, vertex_idxs_of_hit_faces, barycentric_coords):
    """Reference mesh.py:313-324: [B,k] = sum_i bary[:, i] * E[vids[:, i]], on the HIP device."""
    from inf_hip import runtime
    vids = vertex_idxs_of_hit_faces.contiguous()
    bary = barycentric_coords.to(torch.float32).contiguous()
    return runtime.gather(E.contiguous(), vids, bary, out_dtype=torch.float32)


def get_k_eigenfunc_vec_vals_batched(E, vertex_idxs_of_hit_faces, barycentric_coords):
    """Reference mesh.py:327-339 (2^18-ray chunks), result kept on E's device."""
    from inf_hip import runtime
    batch_size = 1 << 18
    B = vertex_idxs_of_hit_faces.shape[0]
    out = torch.empty((B, E.shape[1]), dtype=torch.float32, device=E.device)
    vids = vertex_idxs_of_hit_faces.contiguous()
    bary = barycentric_coords.to(torch.float32).contiguous()
    Ec = E.contiguous()
    for low in range(0, B, batch_size):
        high = min(B, low + batch_size)
        runtime.gather(Ec, vids, bary, offset=low, batch=high - low, out=out[low:high])
    return out


def _out_of_scope(name):
    def f(*args, **kwargs):
        raise NotImplementedError(f"mesh.{name} needs igl / the LBO eigensolve and is outside this build's hot path "
                                  "(SURVEY.md §2)")
    f.__name__ = name
    return f


load_pointcloud = _out_of_scope("load_pointcloud")
compute_first_k_eigenfunctions = _out_of_scope("compute_first_k_eigenfunctions")


class TriMesh:
    """The subset of trimesh.Trimesh the hot path uses: vertices [V][3] float64, faces
    [F][3] int64 (mesh order kept, as the reference's igl-based loader does)."""

    def __init__(self, vertices, faces):
        self.vertices = np.asarray(vertices, dtype=np.float64).reshape(-1, 3)
        self.faces = np.asarray(faces, dtype=np.int64).reshape(-1, 3)
        self._face_normals = None

    @property
    def face_normals(self):
        """trimesh.Trimesh.face_normals (make_model's view dependence, model.py:244): unit
        (v1 - v0) x (v2 - v0) per face."""
        if self._face_normals is None:
            t = self.vertices[self.faces]
            n = np.cross(t[:, 1] - t[:, 0], t[:, 2] - t[:, 0])
            ln = np.linalg.norm(n, axis=1, keepdims=True)
            self._face_normals = n / np.where(ln > 0, ln, 1.0)
        return self._face_normals

    @face_normals.setter
    def face_normals(self, value):
        self._face_normals = np.asarray(value, dtype=np.float64)


def _read_obj(path):
    verts, faces = [], []
    with open(path) as fh:
        for line in fh:
            parts = line.split()
            if not parts:
                continue
            if parts[0] == "v":
                verts.append([float(x) for x in parts[1:4]])
            elif parts[0] == "f":
                idx = [int(p.split("/")[0]) for p in parts[1:]]
                idx = [i - 1 if i > 0 else len(verts) + i for i in idx]
                for j in range(1, len(idx) - 1):  # fan-triangulate polygons
                    faces.append([idx[0], idx[j], idx[j + 1]])
    return np.asarray(verts, dtype=np.float64), np.asarray(faces, dtype=np.int64)


def _read_ply(path):
    with open(path, "rb") as fh:
        header = []
        while True:
            line = fh.readline().decode("ascii", errors="replace").strip()
            header.append(line)
            if line == "end_header":
                break
        fmt = next(h.split()[1] for h in header if h.startswith("format"))
        elems, cur = [], None
        for h in header:
            p = h.split()
            if p and p[0] == "element":
                cur = [p[1], int(p[2]), []]
                elems.append(cur)
            elif p and p[0] == "property" and cur is not None:
                cur[2].append(p[1:])
        tmap = {"char": "i1", "uchar": "u1", "int8": "i1", "uint8": "u1", "short": "i2", "ushort": "u2",
                "int16": "i2", "uint16": "u2", "int": "i4", "uint": "u4", "int32": "i4", "uint32": "u4",
                "float": "f4", "float32": "f4", "double": "f8", "float64": "f8"}
        end = "<" if fmt == "binary_little_endian" else ">"
        V = F = None
        for name, n, props in elems:
            if fmt == "ascii":
                rows = [fh.readline().split() for _ in range(n)]
                if name == "vertex":
                    names = [q[-1] for q in props]
                    cols = [names.index(c) for c in ("x", "y", "z")]
                    V = np.asarray([[float(r[c]) for c in cols] for r in rows])
                elif name == "face":
                    F = np.asarray([[int(x) for x in r[1:4]] for r in rows], dtype=np.int64)
                continue
            if name == "vertex":
                dt = np.dtype([(q[-1], end + tmap[q[0]]) for q in props])
                arr = np.frombuffer(fh.read(dt.itemsize * n), dtype=dt, count=n)
                V = np.stack([arr["x"], arr["y"], arr["z"]], -1).astype(np.float64)
            elif name == "face":
                lp = props[0]  # "list <count type> <index type> vertex_indices"
                ct, it = np.dtype(end + tmap[lp[1]]), np.dtype(end + tmap[lp[2]])
                F = np.empty((n, 3), dtype=np.int64)
                for i in range(n):
                    c = int(np.frombuffer(fh.read(ct.itemsize), dtype=ct)[0])
                    F[i] = np.frombuffer(fh.read(it.itemsize * c), dtype=it)[:3]
            else:
                dt = np.dtype([(q[-1], end + tmap[q[0]]) for q in props])
                fh.read(dt.itemsize * n)
    return V, F


def load_mesh(path):
    """Reference mesh.py:39-50 (igl.read_triangle_mesh -> trimesh, order kept): OBJ / PLY."""
    ext = path.lower().rsplit(".", 1)[-1]
    if ext == "obj":
        v, f = _read_obj(path)
    elif ext == "ply":
        v, f = _read_ply(path)
    else:
        raise NotImplementedError(f"mesh format .{ext}: OBJ and PLY are supported")
    return TriMesh(v, f)


def get_ray_mesh_intersector(mesh):
    """Reference mesh.py:111-117 (trimesh + pyembree): a device BVH (csrc/raycast.hip)."""
    from inf_hip import runtime
    return runtime.Bvh(mesh.vertices, mesh.faces)


def create_ray_origins_and_directions(camCv2world, K, mask_1d, *, H, W, distortion_coeffs=None, distortion_type=None):
    """Reference mesh.py:171-207 on the device: (ray_origins [L][3], unit_ray_dirs [L][3])
    for the mask-selected pixels, generated by the ray-casting kernel."""
    if distortion_type is not None:
        raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
    from inf_hip import runtime
    pixel_idx = None if mask_1d is None else torch.nonzero(torch.as_tensor(mask_1d).reshape(-1).cuda()).reshape(-1)
    cam = torch.as_tensor(camCv2world, dtype=torch.float32)
    # a one-face dummy scene is enough to generate the rays
    bvh = runtime.Bvh(np.zeros((3, 3), np.float32), np.asarray([[0, 1, 2]]))
    _, _, dirs = bvh.cast(camCv2world, K, H, W, pixel_idx)
    origins = cam[:3, 3].to(dirs.device).expand(dirs.shape[0], -1)
    return origins, dirs


def ray_mesh_intersect(ray_mesh_intersector, mesh, ray_origins, ray_directions, return_depth=False, camCv2world=None):
    """Reference mesh.py:210-251: (vertex_idxs_of_hit_faces [M][3], barycentric_coords
    [M][3], hit_ray_idxs [M], face_idxs [M]) of the closest hits, in ray order, on the
    device.  return_depth is not supported."""
    if return_depth:
        raise NotImplementedError("return_depth (mesh.py:226-243) is outside this build's scope")
    o = torch.as_tensor(ray_origins, dtype=torch.float32).cuda()
    d = torch.as_tensor(ray_directions, dtype=torch.float32).cuda()
    face, bary = ray_mesh_intersector.cast_rays(o, d)
    return ray_mesh_intersector.compact(face, bary)


def ray_mesh_intersect_batched(ray_mesh_intersector, mesh, ray_origins, ray_directions):
    """Reference mesh.py:254-310: the GPU casts all rays in one launch (no 2^18 batching)."""
    return ray_mesh_intersect(ray_mesh_intersector, mesh, ray_origins, ray_directions)


def cast_camera_rays(ray_mesh_intersector, camCv2world, K, obj_mask_1d=None, *, H, W):
    """Camera rays of the mask-selected pixels cast in one launch: (vids, bary, hit_ray_idxs,
    face_idxs, unit_ray_dirs) -- the hit lists of ray_mesh_intersect plus all L directions."""
    pixel_idx = None
    if obj_mask_1d is not None:
        pixel_idx = torch.nonzero(torch.as_tensor(obj_mask_1d).reshape(-1).cuda()).reshape(-1)
    face, bary, dirs = ray_mesh_intersector.cast(camCv2world, K, H, W, pixel_idx)
    vids, b, hit, fidx = ray_mesh_intersector.compact(face, bary)
    return vids, b, hit, fidx, dirs


def ray_tracing(ray_mesh_intersector, mesh, eigenfunctions, camCv2world, K, obj_mask_1d=None, *, H, W, batched=True,
                distortion_coeffs=None, distortion_type=None):
    """Reference mesh.py:342-390: (first_k_eigenfunctions [M][k], hit_ray_idxs,
    unit_ray_dirs[hit_ray_idxs], face_idxs), ray casting and gather on the device."""
    if distortion_type is not None:
        raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
    vids, bary, hit, fidx, dirs = cast_camera_rays(ray_mesh_intersector, camCv2world, K, obj_mask_1d, H=H, W=W)
    E = torch.as_tensor(eigenfunctions)
    if not E.is_cuda:
        E = E.to(vids.device)
    feats = get_k_eigenfunc_vec_vals_batched(E, vids, bary)
    return feats, hit, dirs[hit], fidx


def ray_tracing_xyz(ray_mesh_intersector, mesh, vertices, camCv2world, K, obj_mask_1d=None, *, H, W, batched=True,
                    distortion_coeffs=None, distortion_type=None):
    """Reference mesh.py:388-428: (hit_points_xyz [M][3], hit_ray_idxs, unit_ray_dirs[hit],
    face_idxs), the hit points being the barycentric sums over the hit faces' vertices."""
    if distortion_type is not None:
        raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
    vids, bary, hit, fidx, dirs = cast_camera_rays(ray_mesh_intersector, camCv2world, K, obj_mask_1d, H=H, W=W)
    P = torch.as_tensor(vertices if vertices is not None else mesh.vertices).to(vids.device, torch.float32)
    xyz = get_k_eigenfunc_vec_vals_batched(P.contiguous(), vids, bary)
    return xyz, hit, dirs[hit], fidx


class MeshViewPreProcessor:
    """Reference mesh.py:430-548: turns calibrated views (camera, intrinsics, object mask,
    image) into the training-ray files dataset.load_preprocessed_data reads -- the hit
    faces' vertex ids (int32), Cramer barycentrics, expected RGBs, unit ray directions and
    face ids -- with the rays cast on the device.  Hits are kept in ray order per view
    (the reference's order is embree's)."""

    def __init__(self, path_to_mesh, out_directory, mesh=None):
        self.out_dir = out_directory
        self.mesh = mesh if mesh is not None else load_mesh(path_to_mesh)
        self.ray_mesh_intersector = get_ray_mesh_intersector(self.mesh)
        self.cache_vertex_idxs_of_hit_faces = []
        self.cache_barycentric_coords = []
        self.cache_expected_rgbs = []
        self.cache_unit_ray_dirs = []
        self.cache_face_idxs = []

    def cache_single_view(self, camCv2world, K, mask, img, depth_check=None, distortion_coeffs=None,
                          distortion_type=None):
        if distortion_type is not None:
            raise NotImplementedError("lens undistortion (mesh.py:186-193) is outside this build's scope")
        mask = torch.as_tensor(mask)
        H, W = mask.shape
        mask = mask.reshape(-1).to(torch.bool)
        img = torch.as_tensor(img).reshape(H * W, -1)
        vids, bary, hit, face, dirs = cast_camera_rays(self.ray_mesh_intersector, camCv2world, K, mask, H=H, W=W)
        expected_rgbs = img[mask.cpu()].to(hit.device)[hit]  # L x 3 -> hits
        dirs = dirs[hit]
        if depth_check is not None:
            # mesh.py:226-243 + 475-491: depth of the hit from the camera, 1 % outlier threshold
            cam = np.concatenate([np.asarray(torch.as_tensor(camCv2world).cpu(), dtype=np.float64)[:3, :4],
                                  [[0.0, 0, 0, 1]]], 0)
            vw = np.concatenate([self.mesh.vertices, np.ones_like(self.mesh.vertices[:, :1])], -1)
            z = (vw @ np.linalg.inv(cam).T)[:, 2]
            hv, hb = vids.cpu().numpy(), bary.cpu().numpy()
            hit_depth = (z[hv] * hb).sum(-1)
            dc = np.asarray(depth_check).reshape(-1)[mask.cpu().numpy()][hit.cpu().numpy()]
            inlier = np.abs(hit_depth - dc) < np.mean(dc) * 1e-2
            keep = torch.from_numpy(inlier).to(vids.device)
            vids, bary, face, expected_rgbs, dirs = vids[keep], bary[keep], face[keep], expected_rgbs[keep], dirs[keep]
        assert int(face.max().item() if face.numel() else 0) < 2 ** 31
        self.cache_face_idxs.append(face.to(torch.int32).cpu())
        self.cache_vertex_idxs_of_hit_faces.append(vids.to(torch.int32).cpu())
        self.cache_barycentric_coords.append(bary.to(torch.float32).cpu())
        self.cache_expected_rgbs.append(expected_rgbs.to(torch.float32).cpu())
        self.cache_unit_ray_dirs.append(dirs.to(torch.float32).cpu())

    def write_to_disk(self):
        import os
        os.makedirs(self.out_dir, exist_ok=True)
        for name, parts in (("face_idxs", self.cache_face_idxs), ("vids_of_hit_faces", self.cache_vertex_idxs_of_hit_faces),
                            ("barycentric_coords", self.cache_barycentric_coords),
                            ("expected_rgbs", self.cache_expected_rgbs), ("unit_ray_dirs", self.cache_unit_ray_dirs)):
            np.save(os.path.join(self.out_dir, f"{name}.npy"), torch.cat(parts).numpy(), allow_pickle=False)
