"""Data parallelism: one process per GPU, gradients all-reduced over RCCL.

Shapes of the exchange: replicated parameters / Adam state, the same
shuffle on every rank, a torch.chunk split of every global batch, one flat fp32 gradient
all-reduce per step (3.68 MB at k=1024 8x256).

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


def _world(group=None) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def _via_host(t: torch.Tensor, group=None) -> bool:
    """gloo (the one-GPU rehearsal backend) runs the tensor collectives on host copies."""
    return t.is_cuda and dist.get_backend(group) == "gloo"


def reduce_scatter_grads(chunk: torch.Tensor, staging: torch.Tensor, group=None) -> torch.Tensor:
    """Sum the item-major gradient staging [world][chunk] over ranks; rank r keeps chunk r
    (RCCL reduce-scatter; the sharded step's first collective).  World 1: chunk is staging."""
    if _world(group) > 1:
        if _via_host(staging, group):
            out = torch.empty(chunk.shape, dtype=chunk.dtype)
            dist.reduce_scatter_tensor(out, staging.cpu(), op=dist.ReduceOp.SUM, group=group)
            chunk.copy_(out)
        else:
            dist.reduce_scatter_tensor(chunk, staging, op=dist.ReduceOp.SUM, group=group)
    elif chunk.data_ptr() != staging.data_ptr():
        chunk.copy_(staging[:chunk.numel()])
    return chunk


def all_gather_chunks(staging: torch.Tensor, chunk: torch.Tensor, group=None) -> torch.Tensor:
    """staging [world][chunk] = every rank's chunk (RCCL all-gather, in place when `chunk` is
    this rank's slice of `staging`).  World 1: nothing to do."""
    if _world(group) > 1:
        if _via_host(staging, group):
            out = torch.empty(staging.shape, dtype=staging.dtype)
            dist.all_gather_into_tensor(out, chunk.cpu(), group=group)
            staging.copy_(out)
        else:
            dist.all_gather_into_tensor(staging, chunk, group=group)
    elif chunk.data_ptr() != staging.data_ptr():
        staging[:chunk.numel()].copy_(chunk)
    return staging


def gather_sharded_state(plan, group=None):
    """After sharded steps the fp32 masters and the Adam state are current on each rank's own
    items only: gather the three arenas (pack this rank's items -> all-gather -> unpack), so
    every rank again holds all of them bitwise equal (evaluation, checkpoints, replica checks)."""
    for arena in (plan.params, plan.exp_avg, plan.exp_avg_sq):
        plan.shard_pack(arena)
        all_gather_chunks(plan.grad_staging, plan.grad_chunk, group)
        plan.shard_unpack(arena)


def any_rank(flag: bool, device, group=None) -> bool:
    """True on every rank when `flag` is True on at least one (one MAX all-reduce).  Used for
    decisions that change which collectives a rank issues: they must be taken together."""
    t = torch.tensor([1 if flag else 0], dtype=torch.int32, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return bool(int(t.item()))


def replica_checksum(arena: torch.Tensor) -> torch.Tensor:
    """Bit-exact fingerprint of an fp32 arena: [sum of the int32 bit patterns, the same
    weighted by position mod 65521] as int64 (any flipped bit changes the first)."""
    bits = arena.detach().reshape(-1).view(torch.int32).to(torch.int64)
    pos = torch.arange(bits.numel(), device=bits.device, dtype=torch.int64) % 65521 + 1
    return torch.stack([bits.sum(), (bits * pos).sum()])


def check_replicas(arena: torch.Tensor, group=None, what="parameters"):
    """Raise when the replicas' `what` differ on any rank (MIN vs MAX of the fingerprint):
    data parallelism here keeps replicas bitwise equal without broadcasts, so a difference
    means the ranks' collectives or updates went out of step."""
    if not (dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1):
        return
    hi = replica_checksum(arena)
    lo = hi.clone()
    dist.all_reduce(hi, op=dist.ReduceOp.MAX, group=group)
    dist.all_reduce(lo, op=dist.ReduceOp.MIN, group=group)
    if not torch.equal(hi, lo):
        raise RuntimeError(f"data-parallel replicas diverged: {what} differ across ranks "
                           f"(fingerprint min {lo.tolist()} / max {hi.tolist()})")


def allreduce_scalars(values, device, group=None) -> list:
    t = torch.tensor([float(v) for v in values], dtype=torch.float64, device=device)
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(t, group=group)
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


class DataParallelEpoch:
    """The training epoch of one rank under `train.py --data_parallel` (nn.DataParallel's
    role, reference train.py:46-48), plugged into trainer.Trainer, which keeps its
    evaluation, best-model tracking, checkpoints, visualisation and scalars (rank 0 writes).

    Per epoch: the loader's own shuffle (randperm, trainer.py:248 via
    ray_dataloader.py:105) is drawn on rank 0 and broadcast, so every rank walks the same
    batches; rank r takes its torch.chunk shard of each global batch; its shard rows of the
    full batches are laid out contiguously so a captured graph replays the epoch with the
    batch index advancing on the device.  One step = the fused gather -> forward -> loss
    (normalised by the GLOBAL 3 x B) -> backward -> slab reduction into the flat gradient,
    the flat-gradient all-reduce over RCCL, then Adam and the batch advance -- GRAPH_STEPS
    steps per graph replay, the collective captured inside (no host round trip per step).
    Replicas stay bitwise equal without parameter broadcasts.  A partial last batch
    (drop_last=False) runs eagerly.

    Re-capture is decided collectively: a rank whose plan changed (rank 0 alone renders the
    validation views, and a render can grow its model's plan) would otherwise capture on
    its own, and its capture's eager warm-up step would issue an all-reduce the other ranks
    never match -- every later gradient all-reduce would then pair steps of different ranks.
    After every epoch the replicas' parameters are compared bit for bit across ranks
    (check_replicas; INF_DP_CHECK=0 turns it off)."""

    GRAPH_STEPS = 8  # even: the pre-gather slots alternate
    # step shapes (how the gradient all-reduce sits in the step):
    #   serial   -- fused step -> all-reduce of the flat gradient -> Adam + batch advance;
    #   prefetch -- serial, plus the next batch's gather on a side stream beside the
    #               all-reduce (runtime.StepPipeline lead 0: the chain reads pre-gathered rows);
    #   bucketed -- the dW GEMM and gradient reduction in two halves (inf_train_step PART1 /
    #               PART2): bucket 1 (Ly and the layers after it) is all-reduced on a side
    #               stream while the second half's GEMM runs, then bucket 2, then Adam;
    #   sharded  -- ZeRO-1 style (include/inf_hip.h): the local gradient in item-major order,
    #               reduce-scatter, Adam on 1/world of the items, all-gather of the new weights
    #               in the GEMM dtype (bf16: half the bytes of the fp32 all-gather half of an
    #               all-reduce), every rank rewrites the weight images; masters and Adam state
    #               gathered once per epoch.
    # INF_DP_SHAPE picks one; "auto" (default at world > 1 over RCCL) captures every shape,
    # times a few replays of each on the same saved state and keeps the fastest -- the
    # decision is the MAX over ranks of each shape's time, so every rank picks the same one.
    SHAPES = ("serial", "prefetch", "bucketed", "sharded")

    def __init__(self, group=None):
        self.group = group
        self.rank = dist.get_rank(group) if dist.is_available() and dist.is_initialized() else 0
        self.world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.graph = None
        self.key = None
        self.idx = None
        self.steps_done = 0
        self.pipe = None
        self.side = None
        self.shape = "serial"
        self.shape_times = None  # {shape: ms per step} of the last autotune

    def graph_collective(self) -> bool:
        """The all-reduce can be captured into the step graphs (RCCL; not gloo)."""
        return self.world == 1 or dist.get_backend(self.group) != "gloo"

    def _tail_all_reduce(self, rt, plan):
        allreduce_grads(rt.grads, self.group)
        plan.adam(0, 0.0, advance=True)

    def _step(self, rt, plan, batch, xslot=None):
        plan.train_step(batch, None, apply_adam=False, xslot=xslot)
        self._tail_all_reduce(rt, plan)

    def _step_bucketed(self, rt, plan, batch):
        """One step with the gradient all-reduced in two buckets: bucket 1 on a side stream
        beside the second half of the dW GEMM, then bucket 2 (after bucket 1: one
        communicator, used in order), then Adam + advance."""
        split = plan.grad_split()
        plan.train_step(batch, None, apply_adam=False, part=1)
        main = torch.cuda.current_stream()
        if self.side is None:
            self.side = torch.cuda.Stream(device=rt.device)
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            allreduce_grads(rt.grads[split:], self.group)
        plan.train_step(batch, None, apply_adam=False, part=2)
        main.wait_stream(self.side)
        allreduce_grads(rt.grads[:split], self.group)
        plan.adam(0, 0.0, advance=True)

    def _step_sharded(self, rt, plan, batch):
        """One sharded step: reduce-scatter of the item-major gradient, Adam on this rank's
        items (+ the batch advance), all-gather of the new weights, image rewrite."""
        plan.train_step(batch, None, apply_adam=False, shard=True)
        reduce_scatter_grads(plan.grad_chunk, plan.grad_staging, self.group)
        plan.adam_shard(advance=True)
        all_gather_chunks(plan.weight_staging, plan.weight_chunk(), self.group)
        plan.shard_scatter()

    @staticmethod
    def _can_shard(plan, batch) -> bool:
        """The sharded step needs a fused chain for the batch (include/inf_hip.h INF_STEP_SHARD)."""
        return plan.can_shard(batch)

    def _report_shape(self):
        if self.rank == 0 and getattr(self, "_reported", None) != self.shape:
            self._reported = self.shape
            times = f" (ms per step: {self.shape_times})" if self.shape_times else ""
            print(f"[dp] world {self.world}: step shape {self.shape}{times}", flush=True)

    def _ensure_shard(self, plan):
        if getattr(plan, "shard_world", 0) != self.world or getattr(plan, "shard_rank", -1) != self.rank:
            plan.shard(self.world, self.rank)

    def _pipelined(self, count, rt, plan, batch):
        self.pipe.run(count, lambda xs: plan.train_step(batch, None, apply_adam=False, xslot=xs),
                      tail_fn=lambda: self._tail_all_reduce(rt, plan))

    def _steps(self, shape, count, rt, plan, batch):
        if shape == "prefetch" and self.pipe is not None:
            self._pipelined(count, rt, plan, batch)
        elif shape == "bucketed":
            for _ in range(count):
                self._step_bucketed(rt, plan, batch)
        elif shape == "sharded":
            self._ensure_shard(plan)
            for _ in range(count):
                self._step_sharded(rt, plan, batch)
        elif shape == "serial_fallback":  # sharded asked for, the batch's step has no fused chain
            for _ in range(count):
                self._step(rt, plan, batch)
        else:
            for _ in range(count):
                self._step(rt, plan, batch)

    def _candidate_shapes(self, full=None):
        want = os.environ.get("INF_DP_SHAPE", "auto")
        if want != "auto":
            if want not in self.SHAPES:
                raise ValueError(f"INF_DP_SHAPE must be one of {self.SHAPES} or auto")
            return [want]
        # one GPU: nothing to hide behind, the plain step is the fastest (bench.py INF_BENCH_DP).
        # Fewer full batches than one multi-step graph: _time_graphs could only time the
        # one-step graphs, which every shape captures as the serial step -- no autotune.
        if self.world == 1 or (full is not None and full < self.GRAPH_STEPS):
            return ["serial"]
        return list(self.SHAPES)

    def _common_shapes(self, candidates, captured, device):
        """The candidate shapes EVERY rank captured, in candidate order (one MIN all-reduce
        of an availability mask).  A rank may fail to capture a shape the others did -- the
        prefetch pipeline needs pre-gather slots, which a plan grown past CHAIN3_MAX_ROWS
        (rank 0 alone renders the validation views) does not allocate -- and the timing
        replays hold captured all-reduces, so every rank must time the same shapes."""
        avail = torch.tensor([1 if n in captured else 0 for n in candidates], dtype=torch.int32, device=device)
        if self.world > 1:
            dist.all_reduce(avail, op=dist.ReduceOp.MIN, group=self.group)
        names = [n for n, a in zip(candidates, avail.tolist()) if a]
        if not names:
            raise RuntimeError(f"data-parallel step: no step shape every rank can capture ({candidates})")
        return names

    def _capture_stream(self):
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        return s

    def _capture_shape(self, shape, plan, rt, batch, s):
        from inf_hip import runtime
        pipe = None
        if shape == "prefetch":
            pipe = runtime.StepPipeline(plan, batch, lead=0)
            if not pipe.start():
                return None
        self.pipe = pipe
        if shape == "sharded":
            self._ensure_shard(plan)  # allocates: before capture
            if not self._can_shard(plan, batch):
                return None
        g1, gm = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        with torch.cuda.stream(s):
            with torch.cuda.graph(g1, stream=s):
                self._steps(shape if shape in ("bucketed", "sharded") else "serial", 1, rt, plan, batch)
            if shape == "bucketed" and plan.last_part1_bucketed() != 1:
                return None  # PART1 reduced the whole gradient: no overlap, not a real shape
            with torch.cuda.graph(gm, stream=s):
                self._steps(shape, self.GRAPH_STEPS, rt, plan, batch)
        torch.cuda.current_stream().wait_stream(s)
        return (g1, gm, pipe)

    def _time_graphs(self, g, plan, full):
        """ms per step of replays of one shape's graphs (batch index from 0, within the
        epoch's full batches)."""
        g1, gm, pipe = g
        plan.set_batch_index(0)
        if pipe is not None:
            pipe.start()
        n = min(full, self.GRAPH_STEPS)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        if n == self.GRAPH_STEPS:
            gm.replay()  # warm
            plan.set_batch_index(0)
            if pipe is not None:
                pipe.start()
            e0.record()
            gm.replay()
            e1.record()
        else:
            e0.record()
            for _ in range(n):
                g1.replay()
            e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / n

    def _capture(self, plan, rt, batch, full=2):
        saved = [x.clone() for x in (plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl)]
        plan.set_batch_index(0)
        plan.train_step(batch, None, apply_adam=False)  # settles the plan's tables before capture
        self._tail_all_reduce(rt, plan)
        s = self._capture_stream()
        graphs = {}
        candidates = self._candidate_shapes(full)
        for shape in candidates:
            g = self._capture_shape(shape, plan, rt, batch, s)
            if g is not None:
                graphs[shape] = g
        names = self._common_shapes(candidates, graphs, rt.device)
        chosen = names[0]
        if len(names) > 1:
            ms = torch.tensor([self._time_graphs(graphs[n], plan, full) for n in names], dtype=torch.float64,
                              device=rt.device)
            if self.world > 1:
                dist.all_reduce(ms, op=dist.ReduceOp.MAX, group=self.group)
            self.shape_times = dict(zip(names, ms.tolist()))
            chosen = names[int(torch.argmin(ms))]
        for dst, src in zip((plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl), saved):
            dst.copy_(src)
        if getattr(plan, "shard_world", 0):
            gather_sharded_state(plan, self.group)  # restored whole on every rank: marks them so
        plan.sync_shadow()
        g1, gm, pipe = graphs[chosen]
        self.shape, self.pipe = chosen, pipe
        self.graph = (g1, gm)
        self._report_shape()

    def run(self, trainer, loader):
        """One epoch; returns (train loss, summed squared error / rays) over ALL ranks' rays,
        as the reference's single-process loop reports them (trainer.py:248-263)."""
        model, optim = trainer.model, trainer.optim
        loss_type = trainer.loss_fn.loss_type
        B, N = loader.B, loader.N
        iter(loader)  # the reference's per-epoch reshuffle (ray_dataloader.py:103-106)
        perm = loader.idxs
        if self.world > 1:
            perm = perm.contiguous()
            dist.broadcast(perm, 0, group=self.group)
        nb = len(loader)
        full = N // B
        lo, hi = shard_span(B, self.rank, self.world)
        bs = hi - lo
        if bs < 1:
            raise ValueError(f"global batch {B} too small for {self.world} ranks")
        rt = model.hip_runtime()
        group = optim.fused_group_for(model)
        rt.ensure_optimizer_arenas()
        plan = model.hip_plan(bs, loss_type)
        rows = perm[:full * B].view(full, B)[:, lo:hi].reshape(-1)
        if self.idx is None or self.idx.numel() != rows.numel() or self.idx.device != rows.device:
            self.idx = torch.empty_like(rows)
        self.idx.copy_(rows)
        optim.sync_runtime_state(model, rt, plan, group)
        plan.reset_epoch_sums()
        steps = 0
        use_graph = os.environ.get("INF_GRAPH", "1") != "0" and full >= 2 and self.graph_collective()
        if full:
            batch = plan.make_batch(source=loader.source, ray_idx=self.idx, offset=0, batch=bs,
                                    offset_from_ctrl=True, loss_count=3 * B, loss=loss_type)
            if use_graph:
                key = (plan, bs, full, loss_type, loader.source, self.idx.data_ptr())
                stale = self.graph is None or self.key is None or self.key[0] is not plan or \
                    self.key[4] is not loader.source or self.key[1:4] != key[1:4] or self.key[5] != key[5]
                if self.world > 1:  # every rank re-captures (and warms up) together
                    stale = any_rank(stale, rt.device, self.group)
                if stale:
                    self._capture(plan, rt, batch, full)
                    self.key = key
                optim.sync_runtime_state(model, rt, plan, group)
                plan.reset_epoch_sums()
                plan.set_batch_index(0)
                g1, gm = self.graph
                if self.pipe is not None and self.pipe.start():
                    for _ in range(full // self.GRAPH_STEPS):
                        gm.replay()
                    self._pipelined(full % self.GRAPH_STEPS, rt, plan, batch)
                else:
                    for _ in range(full // self.GRAPH_STEPS):
                        gm.replay()
                    for _ in range(full % self.GRAPH_STEPS):
                        g1.replay()
            else:
                plan.set_batch_index(0)
                shape = os.environ.get("INF_DP_SHAPE", "serial")
                self.shape = shape if shape in ("bucketed", "sharded") else "serial"
                if self.shape == "sharded":
                    self._ensure_shard(plan)
                    # every rank's plan has the same batch shape, so all take the same answer
                    if any_rank(not self._can_shard(plan, batch), rt.device, self.group):
                        self.shape = "serial_fallback"
                self._report_shape()
                self._steps(self.shape, full, rt, plan, batch)
            if self.shape == "sharded":
                gather_sharded_state(plan, self.group)
            steps = full
        if nb > full:  # partial last batch (drop_last=False), eager
            gb = N - full * B
            slo, shi = shard_span(gb, self.rank, self.world)
            if shi > slo:
                b = plan.make_batch(source=loader.source, ray_idx=perm, offset=full * B + slo, batch=shi - slo,
                                    loss_count=3 * gb, loss=loss_type)
                plan.train_step(b, None, apply_adam=False)
            else:  # an empty shard still joins the all-reduce with a zero gradient
                rt.grads.zero_()
                plan.set_step(rt.dev_step + full + 1)
            allreduce_grads(rt.grads, self.group)
            plan.adam(0, 0.0)
            steps += 1
        optim.after_fused_steps(model, rt, group, steps)
        self.steps_done += steps
        if os.environ.get("INF_DP_CHECK", "1") != "0":
            check_replicas(rt.arena, self.group)
        c = plan.read_ctrl()
        loss_sum, sse = allreduce_scalars([c["epoch_loss"], c["epoch_sse"]], rt.device, self.group)
        return loss_sum / (3 * N if nb > full else 3 * full * B), sse / (N if nb > full else full * B)


def main_distributed(config, seed, allow_checkpoint_loading=False):
    """`train.py --data_parallel` under torchrun: one process per GPU running the
    reference's Trainer (trainer.py:232-337) with DataParallelEpoch for its epochs."""
    import random

    import numpy as np

    from config import get_data, get_loss_fn, get_model_and_optim, get_renderer
    from trainer import Trainer
    from utils import model_summary
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # INF_DP_BACKEND=gloo: a rehearsal backend -- ranks may then share a GPU (local rank
    # modulo the visible devices; RCCL refuses two ranks on one device) and the collective
    # runs eagerly between the captured steps (gloo cannot be captured into a HIP graph)
    backend = os.environ.get("INF_DP_BACKEND", "nccl")
    if backend == "gloo":
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        dist.init_process_group("gloo")
    else:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = f"cuda:{local}"
    try:
        mesh_path = config["data"].get("mesh_path")
        mesh = None
        if mesh_path is not None and os.path.exists(mesh_path):
            from mesh import load_mesh
            mesh = load_mesh(mesh_path)
        data = get_data(config, device)
        model, optim = get_model_and_optim(config, mesh, device)
        if dist.get_rank() == 0:
            model_summary(model, data)
        loss_fn = get_loss_fn(config)
        renderer = get_renderer(config, model, mesh, device)
        random.seed(seed)
        np.random.seed(seed)
        torch.manual_seed(seed)
        trainer = Trainer(model, optim, loss_fn, renderer, data, mesh, config, device, dp=DataParallelEpoch())
        trainer.train()
    finally:
        dist.destroy_process_group()
