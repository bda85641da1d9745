"""Host mirror of the reference dataset.py -- the on-disk ray format only.

`load_preprocessed_data` (reference dataset.py:12-33): five .npy files per split with
the reference's dtype promotion (vertex ids -> int64, floats -> fp32, face ids -> int64).
The per-view image datasets (dataset.py:36-202) serve evaluation/visualisation and are
outside this build's scope.
"""
import os

import numpy as np
import torch


def load_preprocessed_data(preproc_data_path):
    data = {}
    v = np.load(os.path.join(preproc_data_path, "vids_of_hit_faces.npy"))
    data["vertex_idxs_of_hit_faces"] = torch.from_numpy(v).to(dtype=torch.int64)
    b = np.load(os.path.join(preproc_data_path, "barycentric_coords.npy"))
    data["barycentric_coords"] = torch.from_numpy(b).to(dtype=torch.float32)
    c = np.load(os.path.join(preproc_data_path, "expected_rgbs.npy"))
    data["expected_rgbs"] = torch.from_numpy(c).to(dtype=torch.float32)
    dirs_path = os.path.join(preproc_data_path, "unit_ray_dirs.npy")
    face_path = os.path.join(preproc_data_path, "face_idxs.npy")
    if os.path.exists(dirs_path) and os.path.exists(face_path):
        data["unit_ray_dirs"] = torch.from_numpy(np.load(dirs_path)).to(dtype=torch.float32)
        data["face_idxs"] = torch.from_numpy(np.load(face_path)).to(dtype=torch.int64)
    return data


def save_preprocessed_data(preproc_data_path, vertex_idxs_of_hit_faces, barycentric_coords, expected_rgbs,
                           unit_ray_dirs=None, face_idxs=None):
    """Writer for the same format (the reference writes it in mesh.py:510-569; used here to
    build synthetic datasets for tests and benchmarks)."""
    os.makedirs(preproc_data_path, exist_ok=True)
    np.save(os.path.join(preproc_data_path, "vids_of_hit_faces.npy"), np.asarray(vertex_idxs_of_hit_faces, np.int32))
    np.save(os.path.join(preproc_data_path, "barycentric_coords.npy"), np.asarray(barycentric_coords, np.float32))
    np.save(os.path.join(preproc_data_path, "expected_rgbs.npy"), np.asarray(expected_rgbs, np.float32))
    if unit_ray_dirs is not None and face_idxs is not None:
        np.save(os.path.join(preproc_data_path, "unit_ray_dirs.npy"), np.asarray(unit_ray_dirs, np.float32))
        np.save(os.path.join(preproc_data_path, "face_idxs.npy"), np.asarray(face_idxs, np.int32))
