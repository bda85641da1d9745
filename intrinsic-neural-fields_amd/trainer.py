"""Host mirror of the reference trainer.py (Trainer, trainer.py:18-337).

Public behaviour is the reference's: the same epoch loop, train/val metrics and
TensorBoard tags (Train_Loss, Train Epoch-PSNR, Val_Loss, Val Epoch-PSNR, Test Loss),
best-model tracking starting at min_val_loss = 1.0, checkpoint files and keys
(checkpoint.pt every `checkpoint_every` epochs from epoch 0, checkpoint_{199}.pt /
best_model_checkpoint_{199}.pt, model.pt, model_last_epoch.pt) and resume.

The inner loop is where it differs (trainer.py:248-256): with a TextureField, the HIP
Adam and a tagged loss, every batch runs as ONE fused launch sequence (gather ->
forward -> loss -> backward -> Adam, csrc/plan.hip inf_train_step); the full batches
of an epoch replay a captured HIP graph, and the loss / squared-error sums stay on the
device, read once per epoch instead of the reference's two host syncs per step.  Any
other model / optimizer / loss falls back to the reference's autograd step.
"""
from __future__ import annotations

import copy
import json
import os
import random
import time

import numpy as np
import torch
import torch.nn.functional as F

from evaluation_metrics import epoch_psnr
from utils import to_device


class _JsonlWriter:
    """Stand-in for tensorboardX.SummaryWriter (absent here): scalars to logs/scalars.jsonl."""

    def __init__(self, log_dir):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, "scalars.jsonl")

    def add_scalar(self, tag, value, global_step=None):
        with open(self.path, "a") as f:
            f.write(json.dumps({"tag": tag, "value": float(value), "step": global_step}) + "\n")

    def add_image(self, *args, **kwargs):
        pass


class _NullWriter:
    """Ranks other than 0 of a data-parallel run log nothing (rank 0 logs the all-reduced
    epoch metrics)."""

    def add_scalar(self, *args, **kwargs):
        pass

    def add_image(self, *args, **kwargs):
        pass


def _summary_writer(log_dir):
    try:
        from tensorboardX import SummaryWriter
        return SummaryWriter(log_dir)
    except ImportError:
        return _JsonlWriter(log_dir)


# Steps per captured graph of a replayed epoch: the epoch's full batches replay as the
# greedy decomposition of their count into these sizes (32-step graphs, then 8, 4, 2, 1).
# Each replay launch costs ~5-8 us of idle GPU at its boundary (tools/launch_window.py:
# 61.7 us per step inside a graph, 69.8 us as single-step replays), so long epochs replay
# the largest graph and an epoch's remainder takes at most four launches, not up to 7.
GRAPH_SIZES = (32, 8, 4, 2, 1)
# Round 6: an epoch's full batches replay as ONE captured graph (up to MAX_GRAPH_STEPS steps;
# longer epochs as several of those plus one graph of the remainder), so an epoch pays one
# replay boundary instead of one per 32 steps (+ up to four for its remainder).
MAX_GRAPH_STEPS = 512


def graph_replays(n, sizes=GRAPH_SIZES):
    """The graph sizes, in replay order, that cover n consecutive steps (sizes: descending)."""
    out = []
    for g in sorted(sizes, reverse=True):
        while n >= g:
            out.append(g)
            n -= g
    return out


def epoch_graph_sizes(full):
    """The graph sizes an epoch of `full` full batches captures: one graph of the whole epoch
    (at most MAX_GRAPH_STEPS steps; a longer epoch replays that graph, then one graph of what
    is left over)."""
    if full <= 0:
        return []
    head = min(full, MAX_GRAPH_STEPS)
    return sorted({head} | ({full % head} if full % head else set()), reverse=True)


class _FusedEpoch:
    """Replays captured fused steps over the full batches of an epoch -- one graph of the
    whole epoch (epoch_graph_sizes); the batch index advances on the device.  The gather runs
    inside the fused chain by default; INF_PREFETCH=1 moves the next batch's gather to a
    side stream (runtime.StepPipeline: each step then reads pre-gathered feature rows),
    which measured slower on one GPU (see StepPipeline)."""

    def __init__(self, trainer):
        self.t = trainer
        self.graph = None
        self.key = None
        self.perm = None
        self.pipe = None

    GRAPH_STEPS = 8  # even: the pre-gather slots alternate

    def run(self, loader):
        t = self.t
        model, optim = t.model, t.optim
        loss_type = t.loss_fn.loss_type
        it = iter(loader)  # reshuffles like the reference (randperm on the device)
        B, N, nb = loader.B, loader.N, len(loader)
        full = N // B if nb * B > N else nb
        rt = model.hip_runtime()
        group = optim.fused_group_for(model)
        rt.ensure_optimizer_arenas()
        plan = model.hip_plan(B, loss_type)
        use_graph = os.environ.get("INF_GRAPH", "1") != "0" and full >= 2
        # the captured graph bakes in the plan's workspace / ctrl / shadow pointers and the
        # source's tables: the key holds the objects themselves (compared by identity), so a
        # plan replaced by hip_plan() (a larger render batch, another kernel mode) is never
        # freed and its address reused under a stale graph
        key = (plan, B, N, loss_type, loader.source)
        if self.perm is None or self.perm.numel() != N or self.perm.device != rt.device:
            self.perm = torch.empty(N, dtype=torch.int64, device=rt.device)
        self.perm.copy_(loader.idxs)
        plan.reset_epoch_sums()
        total = 0
        done = 0
        if use_graph:
            optim.sync_runtime_state(model, rt, plan, group)
            stale = self.key is None or self.key[0] is not plan or self.key[4] is not loader.source or \
                self.key[1:4] != key[1:4]
            if self.graph is None or stale:
                self._capture(plan, loader, B, loss_type)
                self.key = key
            optim.sync_runtime_state(model, rt, plan, group)
            plan.reset_epoch_sums()
            plan.set_batch_index(0)
            graphs = self.graph
            if self.pipe is not None and self.pipe.start():
                for _ in range(full // self.GRAPH_STEPS):
                    graphs[self.GRAPH_STEPS].replay()
                b = self._batch
                self.pipe.run(full % self.GRAPH_STEPS,
                              lambda xs: plan.train_step(b, None, apply_adam=True, advance=True, xslot=xs))
                done = full
            else:
                # the captured sizes only (a pipelined capture holds GRAPH_STEPS alone); the
                # batches they do not cover run as eager steps below
                done = 0
                for n in graph_replays(full, tuple(graphs)):
                    graphs[n].replay()
                    done += n
            optim.after_fused_steps(model, rt, group, done)
            total = done * B
        # next() on the loader itself: a second iter() (as `for batch in it` would call)
        # reshuffles, and the reference draws ONE permutation per epoch (trainer.py:248)
        for i in range(nb):
            batch = next(it)
            if i < done:
                continue
            model.fused_train_step(batch, optim, loss_type, want_pred=False)
            total += batch.batch_size
        c = plan.read_ctrl()
        return c["epoch_loss"] / (3 * total), c["epoch_sse"] / total

    def _capture(self, plan, loader, B, loss_type):
        b = plan.make_batch(source=loader.source, ray_idx=self.perm, offset=0, batch=B, offset_from_ctrl=True,
                            loss=loss_type)
        self._batch = b
        # one eager step settles the plan's per-batch tables before capture, then undo it
        saved = [x.clone() for x in (plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl)]
        plan.set_batch_index(0)
        plan.train_step(b, None, apply_adam=True)
        from inf_hip import runtime
        # single-GPU epochs keep the in-kernel gather (StepPipeline's measurement); INF_PREFETCH=1
        # moves it to a side stream
        self.pipe = runtime.StepPipeline(plan, b, lead=1) if os.environ.get("INF_PREFETCH", "0") != "0" else None
        if self.pipe is not None and not self.pipe.start():  # this batch's step has no fused chain
            self.pipe = None
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        full = loader.N // B
        # one graph of the epoch's full batches (+ the pieces of a remainder past MAX_GRAPH_STEPS)
        sizes = epoch_graph_sizes(full) if self.pipe is None else [self.GRAPH_STEPS]
        graphs = {}
        with torch.cuda.stream(s):
            for n in sizes:
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s):  # n steps per replay launch
                    if self.pipe is not None:
                        self.pipe.run(n, lambda xs: plan.train_step(b, None, apply_adam=True, advance=True, xslot=xs))
                    else:
                        # the step's update launch also advances ctrl.batch_index (INF_STEP_ADVANCE)
                        for _ in range(n):
                            plan.train_step(b, None, apply_adam=True, advance=True)
                graphs[n] = g
        torch.cuda.current_stream().wait_stream(s)
        for dst, src in zip((plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl), saved):
            dst.copy_(src)
        plan.sync_shadow()
        self.graph = graphs


class Trainer:
    def __init__(self, model, optim, loss_fn, renderer, data, mesh, config, device, dp=None):
        # dp: dp.DataParallelEpoch under `train.py --data_parallel` (one process per GPU):
        # it runs the training epochs; rank 0 writes logs, checkpoints and models
        self.dp = dp
        self.rank0 = dp is None or dp.rank == 0
        self.model = model
        self.optim = optim
        self.loss_fn = loss_fn
        self.renderer = renderer
        self.mesh = mesh
        self.config = config
        self.use_lr_scheduler = config["training"].get("use_lr_scheduler", False)
        self.lr_scheduler = torch.optim.lr_scheduler.ReduceLROnPlateau(self.optim, mode="min", factor=0.2)
        self.dataset_type = self.config["data"].get("type")
        self.H = config["data"]["img_height"]
        self.W = config["data"]["img_width"]
        self.train_data_loader = data["train"]
        self.val_data_loader = data["val"]
        if self.dataset_type is None:
            self.val_render_infos = list(zip(config["data"].get("eval_render_input_paths", []),
                                             config["data"].get("eval_render_img_names", [])))
        self.test_data_loader = data.get("test", None)
        self.out_dir = self.config["training"]["out_dir"]
        log_dir = os.path.join(self.out_dir, "logs")
        if self.rank0:
            os.makedirs(log_dir, exist_ok=True)
            self.writer = _summary_writer(log_dir)
        else:
            self.writer = _NullWriter()
        self.render_every = self.config["training"]["render_every"]
        self.print_every = self.config["training"]["print_every"]
        self.epochs = self.config["training"]["epochs"]
        self.checkpoint_every = self.config["training"].get("checkpoint_every")
        if self.checkpoint_every is not None:
            self.checkpoint_path = os.path.join(self.out_dir, "checkpoint.pt")
        self.device = device
        self.model_config = self.config["model"]
        self.best_model_weights_path = os.path.join(self.out_dir, "model.pt")
        self.best_model = None
        self.model_last_epoch_path = os.path.join(self.out_dir, "model_last_epoch.pt")
        self._fused_epoch = _FusedEpoch(self)
        self._render_note = False

    # ---- fused-path eligibility ----------------------------------------------------
    def _can_fuse(self, batch=None):
        from inf_optim import Adam
        from model import TextureField
        ok = isinstance(self.model, TextureField) and isinstance(self.optim, Adam) and \
            getattr(self.loss_fn, "loss_type", None) is not None
        if batch is not None:
            ok = ok and hasattr(batch, "is_lazy_rays") and batch.is_lazy_rays()
        return ok

    def _train_step(self, batch):
        """Reference trainer.py:71-84: returns (loss.item(), pred_rgbs)."""
        if self._can_fuse(batch):
            pred = self.model.fused_train_step(batch, self.optim, self.loss_fn.loss_type, want_pred=True)
            plan = self.model._rt.plan
            return plan.read_ctrl()["loss_sum"] / (3 * batch.batch_size), pred
        pred_rgbs = self.model(batch)
        loss = self.loss_fn(pred_rgbs, batch["expected_rgbs"])
        self.optim.zero_grad(set_to_none=True)
        loss.backward()
        self.optim.step()
        return loss.item(), pred_rgbs

    @torch.no_grad()
    def _eval_step(self, model, batch):
        pred_rgbs = model(batch)
        loss = self.loss_fn(pred_rgbs, batch["expected_rgbs"])
        return loss, pred_rgbs

    # ---- visualisation (trainer.py:86-162) ---------------------------------------------
    def write_vis_metrics_to_tensorboard(self, img_name, rendered_img, gt_img, obj_mask_1d, epoch):
        """Reference trainer.py:86-104: the rendered view, its PSNR over the object mask,
        the 2D mean-distance image and the summed absolute distance."""
        from evaluation_metrics import psnr
        mask = np.asarray(torch.as_tensor(obj_mask_1d).cpu()).reshape(-1).astype(bool)
        self.writer.add_image(img_name, rendered_img.transpose(2, 0, 1), global_step=epoch)
        self.writer.add_scalar(f"{img_name}_psnr", psnr(rendered_img, gt_img, mask), epoch)
        mean_distance_2d = 1. - np.mean(np.abs(rendered_img - gt_img), -1)
        self.writer.add_image(f"{img_name}_2d_mean_distance", np.repeat(mean_distance_2d[None, ...], 3, axis=0),
                              global_step=epoch)
        total_dist = np.abs(gt_img.reshape(-1, 3)[mask] - rendered_img.reshape(-1, 3)[mask]).sum()
        self.writer.add_scalar(f"{img_name}_dist", total_dist, epoch)

    @torch.no_grad()
    def _render_view_for_tensorboard(self, input_path, img_name, epoch):
        """Reference trainer.py:106-128: one validation view rendered on the device (rays
        cast against the mesh, csrc/raycast.hip; shading by the plan's render path)."""
        from utils import imread, load_cameras, load_obj_mask_as_tensor
        obj_mask_1d = torch.as_tensor(load_obj_mask_as_tensor(input_path)).reshape(-1)
        camCv2world, K = load_cameras(input_path)
        rendered_img = self.renderer.render(camCv2world, K, obj_mask_1d=obj_mask_1d)
        gt_img = imread(os.path.join(input_path, "image", "000.png"))[..., :3].astype(np.float32) / 255.
        shape = gt_img.shape
        gt_img = gt_img.reshape(-1, 3)
        gt_img[obj_mask_1d.numpy() == False] = 1.  # noqa: E712
        self.write_vis_metrics_to_tensorboard(img_name, rendered_img, gt_img.reshape(shape), obj_mask_1d, epoch)

    @torch.no_grad()
    def _render_views_for_tensorboard_meshroom_radial_k3(self, epoch):
        """Reference trainer.py:130-156."""
        from dataset import MeshroomRadialK3Dataset
        ds = MeshroomRadialK3Dataset(self.config["data"]["vis_dataset_path"], self.config["data"]["vis_split"],
                                     H=self.H, W=self.W)
        for idx in range(len(ds)):
            item = ds[idx]
            rendered_img = self.renderer.render(item["camCv2world"], item["K"],
                                                distortion_coeffs=item["distortion_params"],
                                                distortion_type=item["distortion_type"])
            self.write_vis_metrics_to_tensorboard(f"meshroom_radial_k3_view_{idx}", rendered_img, item["img"].numpy(),
                                                  item["obj_mask_1d"], epoch)

    def _visualize(self, epoch):
        """trainer.py:285-300."""
        if self.renderer is None or getattr(self.renderer, "mesh", None) is None:
            if not self._render_note:
                print("Visualizing... skipped: no mesh to cast the validation views against (data.mesh_path)")
                self._render_note = True
            return
        self.model.eval()
        print("Visualizing...")
        t0 = time.time()
        if self.dataset_type is None:
            for i, (input_path, _name) in enumerate(self.val_render_infos):
                self._render_view_for_tensorboard(input_path, f"img{i:03d}", epoch)
        elif self.dataset_type == "meshroom_radial_k3":
            try:
                self._render_views_for_tensorboard_meshroom_radial_k3(epoch)
            except NotImplementedError as exc:  # lens undistortion is out of scope
                if not self._render_note:
                    print(f"Visualizing... skipped: {exc}")
                    self._render_note = True
                return
        else:
            raise NotImplementedError(f"Unknown dataset type: {self.dataset_type}!")
        print(f"Done with visualizations after {time.time() - t0} seconds.")

    def evaluate(self, epoch=None):
        """Reference trainer.py:164-187 (sums kept on the device, one sync)."""
        self.model.eval()
        acc_loss = torch.zeros((), dtype=torch.float64, device=self.device)
        acc_l2 = torch.zeros((), dtype=torch.float64, device=self.device)
        total = 0
        for batch in self.val_data_loader:
            batch = to_device(batch, device=self.device)
            loss, pred_rgbs = self._eval_step(self.model, batch)
            bs = batch["expected_rgbs"].size()[0]
            acc_l2 += F.mse_loss(pred_rgbs, batch["expected_rgbs"], reduction="sum").double()
            acc_loss += loss.double() * bs
            total += bs
        val_loss = float(acc_loss) / total
        self.writer.add_scalar("Val_Loss", val_loss, epoch)
        val_psnr = epoch_psnr(float(acc_l2) / total)
        self.writer.add_scalar("Val Epoch-PSNR", val_psnr, epoch)
        return val_loss, val_psnr

    def test(self):
        """Reference trainer.py:189-212 (no test loader is built, config.py:85)."""
        if self.test_data_loader is None:
            return
        model = self.best_model if self.best_model is not None else self.model
        model.eval()
        acc, total = 0.0, 0
        for batch in self.test_data_loader:
            loss, _ = self._eval_step(model, batch)
            bs = batch["expected_rgbs"].size()[0]
            acc += loss.item() * bs
            total += bs
        test_loss = acc / total
        self.writer.add_scalar("Test Loss", test_loss)
        print(f"Test Loss: {test_loss}")
        return test_loss

    def _checkpoint_dict(self, epoch):
        return {"epoch": epoch, "model_state_dict": self.model.state_dict(),
                "optimizer_state_dict": self.optim.state_dict(),
                "pytorch_random_state": torch.random.get_rng_state(), "python_random_state": random.getstate(),
                "numpy_random_state": np.random.get_state()}

    def _init_or_load_checkpoint(self):
        """Reference trainer.py:214-230.  The checkpoint is this trainer's own file
        (it holds Python/numpy RNG states, so it is not a weights-only file)."""
        if self.checkpoint_every is None or not os.path.exists(self.checkpoint_path):
            return 0
        print("Restoring from checkpoint...")
        checkpoint = torch.load(self.checkpoint_path, map_location="cpu", weights_only=False)
        self.model.load_state_dict(checkpoint["model_state_dict"])
        self.optim.load_state_dict(checkpoint["optimizer_state_dict"])
        torch.random.set_rng_state(checkpoint["pytorch_random_state"])
        random.setstate(checkpoint["python_random_state"])
        np.random.set_state(checkpoint["numpy_random_state"])
        print("Done.")
        return checkpoint["epoch"] + 1

    def _train_epoch(self):
        if self.dp is not None:
            if not (self._can_fuse() and hasattr(self.train_data_loader, "source")):
                raise NotImplementedError("--data_parallel runs the fused TextureField step (HIP Adam, L1/L2/cauchy "
                                          "loss, a RayDataLoader)")
            return self.dp.run(self, self.train_data_loader)
        if self._can_fuse() and hasattr(self.train_data_loader, "source"):
            return self._fused_epoch.run(self.train_data_loader)
        acc_loss, acc_l2, total = 0.0, 0.0, 0
        for batch in self.train_data_loader:
            batch = to_device(batch, device=self.device)
            loss, pred_rgbs = self._train_step(batch)
            bs = batch["expected_rgbs"].size()[0]
            acc_l2 += F.mse_loss(pred_rgbs, batch["expected_rgbs"], reduction="sum").item()
            acc_loss += loss * bs
            total += bs
        return acc_loss / total, acc_l2 / total

    def train(self):
        """Reference trainer.py:232-337."""
        if self.rank0:
            print("Starting training...")
        epoch_start = self._init_or_load_checkpoint()
        min_val_loss = 1.
        for epoch in range(epoch_start, self.epochs):
            self.model.train()
            t0 = time.time()
            train_loss, train_mse = self._train_epoch()
            t1 = time.time()
            self.writer.add_scalar("Train_Loss", train_loss, epoch)
            train_psnr = epoch_psnr(train_mse)
            self.writer.add_scalar("Train Epoch-PSNR", train_psnr, epoch)
            val_loss, val_psnr = self.evaluate(epoch)
            if val_loss < min_val_loss:
                min_val_loss = val_loss
                if self.rank0:
                    torch.save(self.model.state_dict(), self.best_model_weights_path)
                self.best_model = copy.deepcopy(self.model)
            if self.use_lr_scheduler:
                self.lr_scheduler.step(val_loss)
            if not self.rank0:
                continue
            if epoch == 0 or (epoch + 1) % self.print_every == 0:
                print(f"Epoch: {epoch + 1} / {self.epochs}, Train Loss: {train_loss}, Train PSNR: {train_psnr}, "
                      f"Val Loss: {val_loss}, Val PSNR: {val_psnr}"
                      f"Epoch Time: {t1 - t0}s")
            if epoch == 0 or (epoch + 1) % self.render_every == 0:
                self._visualize(epoch)
            if self.checkpoint_every is not None and epoch % self.checkpoint_every == 0:
                print("Saving checkpoint...")
                torch.save(self._checkpoint_dict(epoch), self.checkpoint_path)
                print("Done.")
            if epoch > 0 and (epoch + 1) == 200:
                print(f"Persisting checkpoint at {epoch}...")
                torch.save(self._checkpoint_dict(epoch), os.path.join(self.out_dir, f"checkpoint_{epoch}.pt"))
                best = self.best_model if self.best_model is not None else self.model
                torch.save(best.state_dict(), os.path.join(self.out_dir, f"best_model_checkpoint_{epoch}.pt"))
                print("Done.")
        self.test()
        if self.rank0:
            print("Done.")
            torch.save(self.model.state_dict(), self.model_last_epoch_path)
