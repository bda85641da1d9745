"""Host mirror of the reference config.py (YAML schema and factories, config.py:26-139).

Same YAML keys and defaults.  Differences, all on the device side: the optimizer is the
HIP Adam (inf_optim.Adam, a torch.optim.Adam subclass with the same state layout), the
loss functions carry the tag the fused training step needs, and an optional
`model.kernels` section ({mode: fp32|bf16, max_batch: N}) selects the GEMM arithmetic
(the reference ignores unknown keys, so these YAMLs still load there).
"""
import os
from shutil import copyfile

import torch
import torch.nn.functional as F
import yaml

from inf_optim import Adam
from mesh import load_first_k_eigenfunctions
from model import make_model
from ray_dataloader import create_ray_dataloader
from renderer import Renderer


def _read_yaml(path):
    with open(path, "r") as fh:
        return yaml.safe_load(fh)


def _announce(config, path):
    """The banner the reference prints for a loaded training config."""
    rule = "=" * 64
    print("\n".join(["-" * 64, f"Loaded Config from {path}", rule,
                     yaml.dump(config, default_flow_style=False), rule + "\n"]))


def load_config_file(path, allow_checkpoint_loading=False, follower=False):
    """Reference config.py:26-36: read the YAML, refuse an existing out_dir unless resuming,
    print it, and keep a copy of the file as out_dir/config.yaml.  follower: a data-parallel
    rank other than 0 only reads the file (rank 0 checks and creates out_dir; the others
    would find it existing)."""
    config = _read_yaml(path)
    if follower:
        return config
    out_dir = config["training"]["out_dir"]
    if os.path.exists(out_dir) and not allow_checkpoint_loading:
        raise RuntimeError(f"out_dir '{out_dir}' exists. Exit to not overwrite old results.")
    _announce(config, path)
    os.makedirs(out_dir, exist_ok=True)
    copyfile(path, os.path.join(out_dir, "config.yaml"))
    return config


def load_config(path):
    """A config file as a dict, nothing else (eval.py, renderer helpers)."""
    return _read_yaml(path)


def get_seed(config):
    return config.get("seed", 0)


def get_log_dir(config):
    """out_dir/logs; out_dir is created if missing."""
    out_dir = config["training"]["out_dir"]
    os.makedirs(out_dir, exist_ok=True)
    return os.path.join(out_dir, "logs")


def get_data(config, device, num_workers_per_data_loader=6):
    """Reference config.py:56-99.  The mesh (config.py:58) supplies the vertex positions of
    the extrinsic (xyz/ff/rff) strategies; efuncs runs do not need it.  Like the reference
    (config.py:85, hasattr on a dict), no test loader is built."""
    mesh = None
    if config["model"].get("feature_strategy", "efuncs") in ("ff", "rff", "xyz"):
        from mesh import load_mesh
        mesh = load_mesh(config["data"]["mesh_path"])
    common = dict(eigenfunctions_path=config["data"]["eigenfunctions_path"], k=config["model"].get("k"),
                  feature_strategy=config["model"].get("feature_strategy", "efuncs"), mesh=mesh,
                  rescale_strategy=config["data"].get("rescale_strategy", "standard"),
                  # the reference passes these two swapped (config.py:63-64); no config sets either
                  eigenvalues_path=config["data"].get("embed_strategy"),
                  embed_strategy=config["data"].get("eigenvalues_path"),
                  batch_size=config["training"]["batch_size"], device=device)
    data = {
        "train": create_ray_dataloader(config["data"]["preproc_data_path_train"], shuffle=True,
                                       drop_last=config["data"].get("train_drop_last", True), **common),
        "val": create_ray_dataloader(config["data"]["preproc_data_path_eval"], shuffle=False, drop_last=False,
                                     **common),
    }
    return data


def get_model_and_optim(config, mesh, device):
    """Reference config.py:102-110 (model.to(device) before the optimizer)."""
    model = make_model(config["model"], mesh=mesh)
    model = model.to(device)
    if hasattr(model, "max_batch_hint"):  # fused-plan models size their workspace for the batch
        model.max_batch_hint = max(model.max_batch_hint, int(config.get("training", {}).get("batch_size", 0) or 0))
    optim = Adam(model.parameters(), lr=config["training"]["lr"])
    return model, optim


def _tag(fn, name):
    fn.loss_type = name
    return fn


def get_loss_fn(config):
    """Reference config.py:113-122."""
    loss_type = config["training"]["loss_type"]
    if loss_type == "L2":
        return _tag(lambda rgb_pred, rgb_gt: F.mse_loss(rgb_pred, rgb_gt), "L2")
    if loss_type == "L1":
        return _tag(lambda rgb_pred, rgb_gt: F.l1_loss(rgb_pred, rgb_gt), "L1")
    if loss_type == "cauchy":
        return _tag(lambda rgb_pred, rgb_gt: ((20 / 255) * (20 / 255) * torch.log(
            1 + (rgb_pred - rgb_gt) ** 2 / ((20 / 255) * (20 / 255)))).mean(), "cauchy")
    raise RuntimeError(f"Unknown loss function: {loss_type}. Please use either 'L1', 'L2' or 'cauchy'")


def get_renderer(config, model, mesh, device):
    """Reference config.py:125-139."""
    feature_strategy = config["model"].get("feature_strategy", "efuncs")
    if feature_strategy in ("ff", "rff", "xyz"):
        return Renderer(model, mesh, feature_strategy=feature_strategy, H=config["data"]["img_height"],
                        W=config["data"]["img_width"], device=device)
    if feature_strategy != "efuncs":
        raise ValueError(f"Unknown feature strategy: {feature_strategy}")
    E = load_first_k_eigenfunctions(config["data"]["eigenfunctions_path"], config["model"]["k"],
                                    rescale_strategy=config["data"].get("rescale_strategy", "standard"),
                                    embed_strategy=config["data"].get("embed_strategy"),
                                    eigenvalues_path=config["data"].get("eigenvalues_path"))
    return Renderer(model, mesh, eigenfunctions=E, H=config["data"]["img_height"], W=config["data"]["img_width"],
                    device=device)
