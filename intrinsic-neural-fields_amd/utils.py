"""Host mirror of the reference utils.py.

load_trained_model (utils.py:22-29), load_cameras (:32-36), model_summary (:39-41),
load_obj_mask_as_tensor (:44-61), batchify_dict_data (:72-83) and to_device (:137-144).
Images are read with PIL (imageio is not installed here); the reference's OpenEXR depth
maps need imageio's freeimage plugin, so a view's object mask is read from
depth/mask.png (the reference's own fallback, utils.py:55-58) or an .npy file, and an
EXR-only view raises.  The tandem helpers are outside this build's scope.
"""
import os
import sys

import numpy as np
import torch

from model import make_model


def tensor_mem_size_in_bytes(x):
    return x.element_size() * x.nelement()


def load_trained_model(model_config, weights_path, device, mesh=None):
    """Reference utils.py:22-29 (weights_only load: state dicts hold tensors only)."""
    model = make_model(model_config, mesh=mesh)
    data = torch.load(weights_path, map_location="cpu", weights_only=True)
    if "model_state_dict" in data:
        model.load_state_dict(data["model_state_dict"])
    else:
        model.load_state_dict(data)
    return model.to(device)


def load_cameras(view_path):
    """Reference utils.py:32-36: camCv2world and K of a view (depth/cameras.npz)."""
    cameras = np.load(os.path.join(view_path, "depth", "cameras.npz"))
    camCv2world = torch.from_numpy(cameras["world_mat_0"]).to(dtype=torch.float32)
    K = torch.from_numpy(cameras["camera_mat_0"]).to(dtype=torch.float32)
    return camCv2world, K


def imread(path):
    """An image file as a numpy array (PIL; uint8 for PNG / JPEG)."""
    from PIL import Image
    with Image.open(path) as im:
        return np.asarray(im)


def load_obj_mask_as_tensor(view_path):
    """Reference utils.py:44-61: the view's object mask (H x W bool).  A .npy path is
    loaded as is; a view directory uses depth/depth_0000.exr (depth != 1e10) when present
    -- which needs imageio's EXR plugin, absent here -- else depth/mask.png (!= 0)."""
    if view_path.endswith(".npy"):
        return np.load(view_path)
    mask_path = os.path.join(view_path, "depth", "mask.png")
    depth_path = os.path.join(view_path, "depth", "depth_0000.exr")
    if os.path.exists(depth_path) and not os.path.exists(mask_path):
        raise NotImplementedError(f"{depth_path}: OpenEXR depth maps need imageio's freeimage plugin, which is not "
                                  "installed; provide depth/mask.png")
    assert os.path.exists(mask_path), "Must have depth or mask"
    mask = imread(mask_path)
    if mask.ndim == 3:
        mask = mask[..., 0]
    return torch.from_numpy(mask != 0)


def model_summary(model, data):
    """Reference utils.py:39-41 uses torchinfo.summary on one batch; this prints the
    parameter table without running a batch (torchinfo is not installed here)."""
    total = 0
    print(f"{type(model).__name__}")
    for name, p in model.named_parameters():
        print(f"  {name:32s} {tuple(p.shape)}")
        total += p.numel()
    print(f"Total params: {total:,}")
    sys.stdout.flush()


def batchify_dict_data(data_dict, input_total_size, batch_size):
    """Reference utils.py:72-83: consecutive batch_size-row batches of every entry (the
    last one shorter; one empty batch for an empty input), indexed by numpy index arrays."""
    starts = range(0, max(input_total_size, 1), batch_size)
    return [{key: val[np.arange(lo, min(lo + batch_size, input_total_size))] for key, val in data_dict.items()}
            for lo in starts]


def to_device(x, *, device):
    """Reference utils.py:137-144 (recursive .to; lazy RayBatch objects stay as they are)."""
    if hasattr(x, "is_lazy_rays"):
        return x
    if torch.is_tensor(x):
        return x.to(device)
    if isinstance(x, str):
        return x
    if isinstance(x, dict):
        return {k: to_device(v, device=device) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(to_device(v, device=device) for v in x)
    raise NotImplementedError(f"Invalid type for to_device: {type(x)}")
