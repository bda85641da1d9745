"""Data parallelism: one process per GPU, gradients all-reduced over RCCL.

Replaces `torch.nn.DataParallel(model, device_ids)` (reference train.py:46-48), which
scatters each global batch over the GPUs of one process, gathers the predictions to
GPU 0 and computes the loss there over the GLOBAL batch, so the gradient is the mean over
all rays.  Here every rank:
  * draws the same seeded permutation of the training rays (no communication),
  * takes its contiguous shard of each global batch (DataParallel's scatter split:
    chunks of ceil(B / world) rays, the last one shorter),
  * runs the fused gather -> forward -> loss -> backward step with the loss normalised by
    the GLOBAL element count (3 x B), leaving its partial gradient in the flat arena,
  * all-reduces (sum) that one flat fp32 bucket (P floats, 3.68 MB for k=1024 8x256) over
    RCCL -- the only collective -- and
  * applies the identical Adam update, so replicas stay bitwise equal without any
    parameter broadcast (DataParallel re-broadcasts parameters on every forward).
"""
from __future__ import annotations

import math
import os

import torch
import torch.distributed as dist


def shard_span(global_batch: int, rank: int, world: int):
    """[lo, hi) rows of a global batch owned by `rank` (torch.chunk split, as the scatter
    inside nn.DataParallel does)."""
    size = math.ceil(global_batch / world)
    lo = min(rank * size, global_batch)
    hi = min(lo + size, global_batch)
    return lo, hi


def epoch_permutation(n: int, seed: int, epoch: int, device) -> torch.Tensor:
    """The same permutation on every rank: a generator seeded by (seed, epoch)."""
    g = torch.Generator(device=device)
    g.manual_seed(int(seed) * 1_000_003 + int(epoch))
    return torch.randperm(n, generator=g, device=device)


def allreduce_grads(flat_grads: torch.Tensor, group=None) -> torch.Tensor:
    """Sum the flat gradient bucket over all ranks (RCCL on HIP devices, gloo on CPU)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(flat_grads, op=dist.ReduceOp.SUM, group=group)
    return flat_grads


def allreduce_scalars(values, device) -> list:
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        dist.all_reduce(t)
    return [float(x) for x in t.cpu()]


def render_distributed(renderer, camCv2world, K, obj_mask_1d=None, group=None):
    """One frame rendered by all ranks (SURVEY.md §8(e) render row; renderer.py:64-146):
    rank r casts and shades only the pixel rows shard_span(H, r, world) -- its own rays,
    hits and MLP rows, no exchange on the data path -- then the row slices are assembled
    by one all_gather of equal-height (padded) slices.  Returns the H x W x 3 image as a
    tensor on the renderer's device, identical on every rank."""
    H, W = renderer.H, renderer.W
    world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
    rank = dist.get_rank(group) if world > 1 else 0
    lo, hi = shard_span(H, rank, world)
    mask = torch.zeros(H * W, dtype=torch.bool)
    mask[lo * W:hi * W] = True
    if obj_mask_1d is not None:
        mask &= torch.as_tensor(obj_mask_1d).reshape(-1).bool().cpu()
    img = renderer.render_device(camCv2world, K, obj_mask_1d=mask)  # H x W x 3, rows lo..hi shaded
    if world == 1:
        return img
    rows = math.ceil(H / world)
    part = torch.empty((rows, W, 3), dtype=img.dtype, device=img.device)
    part[:hi - lo] = img[lo:hi]
    parts = [torch.empty_like(part) for _ in range(world)]
    dist.all_gather(parts, part, group=group)
    return torch.cat([parts[r][:shard_span(H, r, world)[1] - shard_span(H, r, world)[0]] for r in range(world)])


class DataParallelTrainer:
    """Fused training epochs of one TextureField replica (see module docstring)."""

    def __init__(self, model, optim, loss_type: str, loader, seed: int = 0):
        self.model, self.optim, self.loss_type, self.loader, self.seed = model, optim, loss_type, loader, seed
        self.rank = dist.get_rank() if dist.is_initialized() else 0
        self.world = dist.get_world_size() if dist.is_initialized() else 1

    def train_epoch(self, epoch: int):
        ld = self.loader
        B, N = ld.B, ld.N
        nb = len(ld)
        perm = epoch_permutation(N, self.seed, epoch, ld.device)
        model, optim = self.model, self.optim
        rt = model.hip_runtime()
        group = optim.fused_group_for(model)
        rt.ensure_optimizer_arenas()
        lo, hi = shard_span(B, self.rank, self.world)
        plan = model.hip_plan(max(hi - lo, 1), self.loss_type)
        optim.sync_runtime_state(model, rt, plan, group)
        plan.reset_epoch_sums()
        total = 0
        for i in range(nb):
            b0 = i * B
            gb = min(B, N - b0)
            slo, shi = shard_span(gb, self.rank, self.world)
            if shi > slo:
                b = plan.make_batch(source=ld.source, ray_idx=perm, offset=b0 + slo, batch=shi - slo,
                                    loss_count=3 * gb, loss=self.loss_type)
                plan.train_step(b, None, apply_adam=False)
            else:  # an empty shard still joins the all-reduce with a zero gradient
                rt.grads.zero_()
                plan.set_step(rt.dev_step + 1)
            allreduce_grads(rt.grads)
            plan.adam(0, 0.0)
            optim.after_fused_step(model, rt, group)
            total += gb
        c = plan.read_ctrl()
        loss_sum, sse = allreduce_scalars([c["epoch_loss"], c["epoch_sse"]], rt.device)
        return loss_sum / (3 * total), sse / total


def main_distributed(config, seed):
    """`train.py --data_parallel` under torchrun: one process per GPU."""
    import random

    import numpy as np

    from config import get_data, get_loss_fn, get_model_and_optim
    from evaluation_metrics import epoch_psnr
    local = int(os.environ.get("LOCAL_RANK", "0"))
    torch.cuda.set_device(local)
    dist.init_process_group("nccl")
    device = f"cuda:{local}"
    data = get_data(config, device)
    model, optim = get_model_and_optim(config, None, device)
    loss_fn = get_loss_fn(config)
    random.seed(seed)
    np.random.seed(seed)
    torch.manual_seed(seed)
    dpt = DataParallelTrainer(model, optim, loss_fn.loss_type, data["train"], seed)
    out_dir = config["training"]["out_dir"]
    for epoch in range(config["training"]["epochs"]):
        train_loss, mse = dpt.train_epoch(epoch)
        if dpt.rank == 0:
            print(f"Epoch: {epoch + 1} / {config['training']['epochs']}, Train Loss: {train_loss}, "
                  f"Train PSNR: {epoch_psnr(mse)}")
    if dpt.rank == 0:
        torch.save(model.state_dict(), os.path.join(out_dir, "model_last_epoch.pt"))
    dist.destroy_process_group()
