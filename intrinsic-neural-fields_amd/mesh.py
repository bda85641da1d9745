"""Host mirror of the reference mesh.py -- the hot-path subset.

* `load_first_k_eigenfunctions` (reference mesh.py:53-108) is the table producer: host
  numpy at setup time, exactly as in the reference (it runs once per loader).
* `get_k_eigenfunc_vec_vals` (mesh.py:313-324) and `get_k_eigenfunc_vec_vals_batched`
  (mesh.py:327-339) run the HIP gather kernel (csrc/gather.hip).  Unlike the reference's
  batched variant, which fills a host buffer, the batched form keeps the result on the
  table's device.

Mesh IO, the Laplace-Beltrami eigensolve and ray casting (mesh.py:19-50, 111-310,
342-605) need igl / trimesh / embree and are outside this build's scope
(SURVEY.md §2, §8(f) rank 1).
"""
from __future__ import annotations

import numpy as np
import torch


def load_first_k_eigenfunctions(eigenfunctions_path, k, rescale_strategy="standard", embed_strategy=None,
                                eigenvalues_path=None, ts=128):
    """Reference mesh.py:53-108: column select, optional GPS/HKS embedding, rescale."""
    all_eigenfunctions = np.load(eigenfunctions_path)
    if isinstance(k, list):
        eigenfunctions = all_eigenfunctions[:, np.array(k)]
    else:
        stored_k = all_eigenfunctions.shape[1]
        assert k <= stored_k
        eigenfunctions = all_eigenfunctions[:, :k]

    eigenvalues = None
    if eigenvalues_path is not None:
        all_eigenvalues = np.load(eigenvalues_path)
        if isinstance(k, list):
            eigenvalues = all_eigenvalues[np.array(k)] if all_eigenvalues.ndim == 1 else \
                all_eigenvalues[:, np.array(k)]
        else:
            assert k <= all_eigenvalues.shape[0]
            eigenvalues = all_eigenvalues[:k]
        if np.abs(eigenvalues[0]) < 1e-10 and eigenvalues[0] < 0:
            eigenvalues[0] *= -1
        assert np.all(eigenvalues > 0), f"Min value: {eigenvalues.min()}"

    if embed_strategy is not None:
        if embed_strategy == "gps":
            assert eigenvalues is not None
            weights = np.sqrt(eigenvalues)
            weights /= weights[0]
            return eigenfunctions / weights
        elif embed_strategy == "hks":
            assert eigenvalues is not None
            timesteps = np.logspace(-2, 0, num=ts)
            eigenfunctions = (eigenfunctions * eigenfunctions) @ np.exp(-eigenvalues[..., None] @ timesteps[None, ...])
        else:
            raise ValueError(f"Unknown embedding strategy {embed_strategy}")

    if rescale_strategy == "standard":
        eigenfunctions = eigenfunctions / (np.max(eigenfunctions, axis=0, keepdims=True) -
                                           np.min(eigenfunctions, axis=0, keepdims=True))
    elif rescale_strategy == "one-norm":
        eigenfunctions = eigenfunctions / np.linalg.norm(eigenfunctions, ord=2, axis=-1, keepdims=True)
    elif rescale_strategy != "unscaled":
        raise RuntimeError(f"Unknown rescaling strategy: {rescale_strategy}")

    return torch.from_numpy(np.ascontiguousarray(eigenfunctions)).to(dtype=torch.float32)


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
        raise NotImplementedError(f"mesh.{name} needs igl/trimesh/embree and is outside this build's hot path "
                                  "(SURVEY.md §8(f)); provide precomputed hits instead")
    f.__name__ = name
    return f


load_mesh = _out_of_scope("load_mesh")
load_pointcloud = _out_of_scope("load_pointcloud")
compute_first_k_eigenfunctions = _out_of_scope("compute_first_k_eigenfunctions")
get_ray_mesh_intersector = _out_of_scope("get_ray_mesh_intersector")
ray_tracing = _out_of_scope("ray_tracing")
ray_tracing_xyz = _out_of_scope("ray_tracing_xyz")
