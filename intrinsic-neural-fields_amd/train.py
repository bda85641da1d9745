"""Host mirror of the reference train.py (CLI entry, train.py:13-63).

    python train.py <config.yaml> [--allow_checkpoint_loading] [--data_parallel]

--data_parallel: the reference wraps the model in torch.nn.DataParallel (train.py:46-48).
Here data parallelism is one process per GPU (launch with torchrun); the global batch
of the YAML is split evenly over the ranks and the gradients are all-reduced over RCCL
before the Adam step, inside the same Trainer (evaluation, checkpoints, scalars and
models from rank 0; see dp.py).  Without torchrun the flag is a no-op on one GPU.
"""
import argparse
import os
import random

import numpy as np
import torch

from config import get_data, get_loss_fn, get_model_and_optim, get_renderer, get_seed, load_config_file
from trainer import Trainer
from utils import model_summary


def parse_args():
    parser = argparse.ArgumentParser()
    parser.add_argument("config_path", type=str)
    parser.add_argument('--allow_checkpoint_loading', default=False, action="store_true")
    parser.add_argument('--data_parallel', default=False, action="store_true")
    return parser.parse_args()


def main():
    args = parse_args()
    distributed = args.data_parallel and "WORLD_SIZE" in os.environ  # launched by torchrun
    follower = distributed and int(os.environ.get("RANK", "0")) != 0
    config = load_config_file(args.config_path, args.allow_checkpoint_loading, follower=follower)
    seed = get_seed(config)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    if not torch.cuda.is_available():
        raise RuntimeError("this build trains on MI355X (HIP) devices; no GPU is visible")
    device = "cuda"
    if distributed:
        import dp
        return dp.main_distributed(config, seed)
    # train.py:38 loads the mesh: the renderer casts against it and the extrinsic
    # strategies read its vertex positions
    mesh_path = config["data"].get("mesh_path")
    if mesh_path is not None and os.path.exists(mesh_path):
        from mesh import load_mesh
        mesh = load_mesh(mesh_path)
    else:
        mesh = None
    data = get_data(config, device)
    model, optim = get_model_and_optim(config, mesh, device)
    model_summary(model, data)
    loss_fn = get_loss_fn(config)
    renderer = get_renderer(config, model, mesh, device)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    trainer = Trainer(model, optim, loss_fn, renderer, data, mesh, config, device)
    trainer.train()


if __name__ == "__main__":
    main()
