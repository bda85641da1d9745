"""Host mirror of the reference dataset.py.

`load_preprocessed_data` (reference dataset.py:12-33): five .npy files per split with
the reference's dtype promotion (vertex ids -> int64, floats -> fp32, face ids -> int64).
`MeshViewsDataset` (:108-149) and `MeshroomRadialK3Dataset` (:160-202): the per-view
image datasets eval.py and the trainer's visualisation iterate (camera, intrinsics,
image with a white background, object mask).  The per-ray `MeshViewsPreprocessedDataset`
(:36-105) is replaced by the device-resident ray_dataloader.RayDataLoader.
"""
import json
import os

import numpy as np
import torch


# (file, key in the returned dict, dtype) of a preprocessed split; the last two files are
# written only for the view-dependent / extrinsic strategies and load as a pair
_PREPROC_FILES = (("vids_of_hit_faces.npy", "vertex_idxs_of_hit_faces", torch.int64),
                  ("barycentric_coords.npy", "barycentric_coords", torch.float32),
                  ("expected_rgbs.npy", "expected_rgbs", torch.float32))
_PREPROC_OPTIONAL = (("unit_ray_dirs.npy", "unit_ray_dirs", torch.float32),
                     ("face_idxs.npy", "face_idxs", torch.int64))


def load_preprocessed_data(preproc_data_path):
    """Reference dataset.py:12-33: the split's ray arrays as tensors of the reference's
    dtypes (the optional direction / face-id pair only when both files exist)."""
    def load(name, dtype):
        return torch.from_numpy(np.load(os.path.join(preproc_data_path, name))).to(dtype=dtype)

    data = {key: load(name, dt) for name, key, dt in _PREPROC_FILES}
    if all(os.path.exists(os.path.join(preproc_data_path, name)) for name, _, _ in _PREPROC_OPTIONAL):
        data.update({key: load(name, dt) for name, key, dt in _PREPROC_OPTIONAL})
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


class MeshViewsDataset(torch.utils.data.Dataset):
    """Reference dataset.py:108-149: views listed in <dataset>/<split>.lst, each a directory
    with depth/cameras.npz, an object mask (utils.load_obj_mask_as_tensor) and
    image/000.png; the image's background is painted white."""

    def __init__(self, dataset_path, split, H=512, W=512, background="white"):
        self.dataset_path = dataset_path
        self.H = H
        self.W = W
        self.background = background
        with open(os.path.join(self.dataset_path, f"{split}.lst")) as fh:
            self.mesh_views_list = [ln[:-1] if ln.endswith("\n") else ln for ln in fh.readlines()]

    def __len__(self):
        return len(self.mesh_views_list)

    def __getitem__(self, idx):
        from utils import imread, load_cameras, load_obj_mask_as_tensor
        assert idx < len(self.mesh_views_list)
        view = os.path.join(self.dataset_path, self.mesh_views_list[idx])
        camCv2world, K = load_cameras(view)
        obj_mask = torch.as_tensor(load_obj_mask_as_tensor(view))
        bg_mask_1d = (obj_mask == False).reshape(-1)  # noqa: E712
        obj_mask_1d = obj_mask.reshape(-1)
        img = torch.from_numpy(imread(os.path.join(view, "image", "000.png"))[..., :3].copy()).to(torch.float32)
        img /= 255.
        img = img.reshape(-1, 3)
        if self.background == "white":
            img[bg_mask_1d] = 1.0
        else:
            assert False, "Currently only white background is supported"
        img = img.reshape(self.H, self.W, 3)
        return {"camCv2world": camCv2world, "K": K, "img": img, "obj_mask_1d": obj_mask_1d}


def load_meshroom_metadata(dataset_path, split):
    """Reference dataset.py:155-158."""
    with open(os.path.join(dataset_path, f"{split}_data.json")) as fh:
        return json.load(fh)


class MeshroomRadialK3Dataset(torch.utils.data.Dataset):
    """Reference dataset.py:160-202 (views with a radial-K3 lens model; rendering them
    needs the lens undistortion the renderer does not implement, see renderer.py)."""

    MESHROOM_RADIAL_K3 = "meshroom_radial_k3"  # cameras.DistortionTypes.MESHROOM_RADIAL_K3

    def __init__(self, dataset_path, split, *, H, W):
        self.dataset_path = dataset_path
        self.H = H
        self.W = W
        self.metadata = load_meshroom_metadata(dataset_path, split)
        self.K = torch.from_numpy(np.array(self.metadata["K"]).astype(np.float32))
        self.distortion_params = list(map(float, self.metadata["distortion_params"]))

    def __len__(self):
        return len(self.metadata["views"])

    def __getitem__(self, idx):
        from utils import imread
        assert idx < len(self.metadata["views"])
        cur = self.metadata["views"][idx]
        img = torch.from_numpy(imread(os.path.join(self.dataset_path, cur["view_file"])) / 255.).to(torch.float32)
        obj_mask = np.load(os.path.join(self.dataset_path, cur["obj_mask_file"]))
        img[torch.from_numpy(obj_mask == False)] = 1.  # noqa: E712
        cam2world = torch.from_numpy(np.array(cur["cam2world"]).astype(np.float32))[:3]
        return {"camCv2world": cam2world, "K": self.K, "distortion_params": self.distortion_params,
                "distortion_type": self.MESHROOM_RADIAL_K3, "img": img, "obj_mask_1d": obj_mask.reshape(-1)}
