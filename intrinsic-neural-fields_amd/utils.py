"""Host mirror of the reference utils.py -- the helpers on the hot path.

load_trained_model (utils.py:22-29), model_summary (:39-41), batchify_dict_data
(:72-83) and to_device (:137-144).  Camera / mask / depth IO (:32-36, 44-69) and the
tandem helpers are outside this build's scope.
"""
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
    """Reference utils.py:72-83."""
    idxs = np.arange(0, input_total_size)
    batch_idxs = np.split(idxs, np.arange(batch_size, input_total_size, batch_size), axis=0)
    batches = []
    for cur_idxs in batch_idxs:
        data = {}
        for key in data_dict.keys():
            data[key] = data_dict[key][cur_idxs]
        batches.append(data)
    return batches


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
