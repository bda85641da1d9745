#!/usr/bin/env python
"""Benchmark of the intrinsic-neural-fields hot path on MI355X.

Metric (BASELINE.json): training rays/s (+ render pixels/s) of the k=1024, 8x256-MLP
TextureField (skip 4, L2 loss, Adam lr 1e-4), bf16 MFMA with fp32 master weights.
A step = one fused training step over one batch of rays resident in HBM:
gather -> forward -> loss -> backward -> Adam (+ RCCL all-reduce of the gradient when
N > 1).  Synthetic data (no dataset in the container): table E = randn(V, k) with the
reference's per-column (max - min) rescale, uniform vertex ids, Dirichlet(1,1,1)
barycentrics, U[0,1) colours.  Weak scaling: `--batch` rays per GPU per step.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--mode bf16|fp32]
    torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

# dense MFMA TFLOP/s (MI355X_MICROARCH.md); bf16x3 runs three bf16 MFMAs per algorithmic
# product, so its ceiling in algorithmic FLOPs is a third of the bf16 peak
PEAK = {"bf16": 2500.0, "fp32": 157.3, "bf16x3": 2500.0 / 3}
HBM_PEAK = 8000.0  # GB/s
KERNEL_NAMES = {"dw_gemm": "lgemm_kernel (grouped weight-gradient GEMM, fragment-image B operand; with the "
                           "fused update: split-K 1, each block Adam on its own 64x64 tile)",
                "chain": "chain_kernel (fused forward + loss + dX chain, LDS weight ring)",
                "chain3": "chain3_kernel (fused gather + forward + loss + dX chain, register-streamed weights)"}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=200)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=4096, help="rays per GPU per step (reference batch_size 4096)")
    ap.add_argument("--mode", default="bf16", choices=["bf16", "fp32", "bf16x3"])
    ap.add_argument("--k", type=int, default=1024)
    ap.add_argument("--layers", type=int, default=8)
    ap.add_argument("--hidden", type=int, default=256)
    ap.add_argument("--skip", type=int, default=4)
    ap.add_argument("--verts", type=int, default=50000)
    ap.add_argument("--loss", default="L2", choices=["L2", "L1", "cauchy"])
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-render", action="store_true")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--extra-batches", default="65536", help="comma list of extra per-GPU batch sizes to report")
    ap.add_argument("--no-config-d", action="store_true")
    ap.add_argument("--strong-batch", type=int, default=4096,
                    help="global batch of the strong-scaling leg (the YAML batch_size, split over the GPUs)")
    ap.add_argument("--strong-local", default="512,1024,2048",
                    help="N=1: per-GPU batches of the strong-scaling points (4096 / 8, / 4, / 2) to time")
    ap.add_argument("--only", default="", help="debug: run only these comma-separated secondary sections "
                                                "(configD, render, rff, psnr, cpu) after the headline")
    return ap.parse_args()


def synthetic(V, k, N, seed, device, ray_seed=None):
    """The table from `seed` (the same on every rank: data-parallel replicas share one
    eigenfunction table), the rays from `ray_seed` (each rank's own; default: `seed`)."""
    g = torch.Generator(device="cpu").manual_seed(seed)
    if V * k > (1 << 28):  # config D's 500k x 4096 table (8.2 GB fp32): drawn on the device
        gd = torch.Generator(device=device).manual_seed(seed)
        E = torch.randn((V, k), generator=gd, device=device)
        E /= E.max(0, keepdim=True).values - E.min(0, keepdim=True).values
    else:
        E = torch.randn((V, k), generator=g)
        E = E / (E.max(0, keepdim=True).values - E.min(0, keepdim=True).values)
    if ray_seed is not None and ray_seed != seed:
        g = torch.Generator(device="cpu").manual_seed(ray_seed)
    vids = torch.randint(0, V, (N, 3), generator=g)
    u = torch.rand((N, 3), generator=g).clamp_min(1e-12)
    bary = -torch.log(u)
    bary = bary / bary.sum(1, keepdim=True)
    rgb = torch.rand((N, 3), generator=g)
    return E.to(device), vids.to(device), bary.to(device), rgb.to(device)


def build_model(args, device):
    import model as M
    torch.manual_seed(0)
    cfg = {"k": args.k, "num_layers": args.layers, "mlp_hidden_dim": args.hidden, "skip_layer_idx": args.skip,
           "kernels": {"mode": args.mode}}
    m = M.make_model(cfg).to(device)
    m.kernel_mode = args.mode
    return m


class Trainer:
    """Graph-captured fused steps over one RaySource (one rank).

    shape (the data-parallel step, world > 1 or INF_BENCH_DP=1): "serial" -- fused step,
    flat-gradient all-reduce, Adam, in order; "prefetch" -- the same with the next batch's
    gather on a side stream beside the all-reduce (runtime.StepPipeline lead 0); "bucketed" --
    the dW GEMM and gradient reduction in two halves (inf_train_step PART1 / PART2), bucket 1
    all-reduced on a side stream while the second half runs (dp.DataParallelEpoch)."""

    def __init__(self, args, device, B, rank, world, nb=32, shape="serial", global_batch=None, dp=None):
        from inf_hip import runtime
        self.args, self.B, self.world = args, B, world
        self.shape = shape
        # the loss is normalised by the GLOBAL batch: world x B (weak scaling), or the
        # reference's batch split over the ranks (strong scaling, nn.DataParallel semantics)
        self.global_batch = global_batch if global_batch is not None else B * world
        self.model = build_model(args, device)
        rt = self.model.hip_runtime()
        rt.ensure_optimizer_arenas()
        self.plan = runtime.Plan(args.k, args.hidden, args.layers, args.skip, args.mode, args.loss, B, rt.arena,
                                 rt.grads, rt.exp_avg, rt.exp_avg_sq)
        self.plan.set_lr(1e-4)
        self.nb = nb
        self.N = self.nb * B
        # one table on every rank (replicas share E), each rank its own rays
        E, vids, bary, rgb = synthetic(args.verts, args.k, self.N, seed=1, device=device, ray_seed=1 + rank)
        self.src = runtime.RaySource(E, vids, bary, rgb)
        self.perm = torch.randperm(self.N, device=device)
        self.batch = self.plan.make_batch(source=self.src, ray_idx=self.perm, offset=0, batch=B,
                                          offset_from_ctrl=True, loss_count=3 * self.global_batch, loss=args.loss)
        self.graphs = None
        self.i = 0
        # the data-parallel step shape (flat-gradient all-reduce between the update and Adam);
        # INF_BENCH_DP=1 runs it at world 1 too (rehearses RCCL capture on a one-GPU box)
        self.dp = (world > 1 or bool(os.environ.get("INF_BENCH_DP"))) if dp is None else dp
        self.ar_in_graph = False
        # shape "prefetch" (or INF_PREFETCH=1 on the single-GPU step): the next batch's gather
        # on a side stream beside the gradient all-reduce (runtime.StepPipeline lead 0)
        self.pipe = runtime.StepPipeline(self.plan, self.batch, lead=int(os.environ.get("INF_PREFETCH_LEAD", "0")))
        self.side = torch.cuda.Stream(device=device)
        want = shape == "prefetch" if self.dp else os.environ.get("INF_PREFETCH", "0") != "0"
        self.prefetch = want and self.pipe.start()
        if self.dp and shape == "sharded":
            if not self.plan.can_shard(self.batch):
                raise RuntimeError("sharded step shape: this batch's step has no fused chain")
            self.plan.shard(world, rank)  # item-major staging (dp.py shape "sharded")

    # steps per replayed graph (divides nb)
    GRAPH_STEPS = int(os.environ.get("INF_GRAPH_STEPS", "8"))

    def _launch(self, xslot=None):
        if not self.dp:
            # Adam + the batch-index advance ride in the step's update launch
            self.plan.train_step(self.batch, None, apply_adam=True, advance=True, xslot=xslot)
        else:
            self.plan.train_step(self.batch, None, apply_adam=False, xslot=xslot, shard=self.shape == "sharded")

    def _bucketed_step(self):
        plan, dist = self.plan, torch.distributed
        split = plan.grad_split()
        plan.train_step(self.batch, None, apply_adam=False, part=1)
        main = torch.cuda.current_stream()
        self.side.wait_stream(main)
        with torch.cuda.stream(self.side):
            if dist.is_initialized():
                dist.all_reduce(plan.grads[split:])
        plan.train_step(self.batch, None, apply_adam=False, part=2)
        main.wait_stream(self.side)
        if dist.is_initialized():
            dist.all_reduce(plan.grads[:split])
        plan.adam(0, 0.0, advance=True)

    def _steps(self, n):
        """n steps: pipelined (side-stream prefetch of the next batch), bucketed or plain."""
        if self.dp and self.shape == "bucketed":
            for _ in range(n):
                self._bucketed_step()
            return
        tail = self._dp_tail if self.dp else None
        if self.prefetch:
            self.pipe.run(n, self._launch, first_slot=self.i % 2, tail_fn=tail)
        else:
            for _ in range(n):
                self._launch()
                if tail is not None:
                    tail()

    def _dp_tail(self):
        """all-reduce of the flat gradient bucket, then the replicated Adam + batch advance;
        sharded: reduce-scatter, Adam on this rank's items + advance, all-gather of the new
        weights, image rewrite (dp.DataParallelEpoch._step_sharded)"""
        if self.shape == "sharded":
            import dp
            plan = self.plan
            dp.reduce_scatter_grads(plan.grad_chunk, plan.grad_staging)
            plan.adam_shard(advance=True)
            dp.all_gather_chunks(plan.weight_staging, plan.weight_chunk())
            plan.shard_scatter()
            return
        if torch.distributed.is_initialized():
            torch.distributed.all_reduce(self.plan.grads)
        self.plan.adam(0, 0.0, advance=True)

    def gather_state(self):
        """Sharded shape: masters and Adam state whole again (before stage timings read them)."""
        if self.dp and self.shape == "sharded":
            import dp
            dp.gather_sharded_state(self.plan)

    def _capture_dp_steps(self, s):
        """GRAPH_STEPS whole data-parallel steps (RCCL all-reduce included) in one graph: no
        host round trip per step.  INF_DP_EAGER_AR=1 keeps the all-reduce outside the graphs."""
        if os.environ.get("INF_DP_EAGER_AR"):
            return None
        if torch.distributed.is_initialized() and torch.distributed.get_backend() == "gloo":
            return None  # gloo cannot run inside a HIP graph capture (rehearsal backend)
        try:
            gm = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gm, stream=s):
                self._steps(self.GRAPH_STEPS)
            self.ar_in_graph = True
            return gm
        except Exception as exc:  # capture refused: per-step replays around an eager all-reduce
            print(f"[bench] all-reduce graph capture failed ({exc}); eager all-reduce", file=sys.stderr)
            torch.cuda.synchronize()
            return None

    def capture(self):
        # one eager step: settles the plan's tables before capture
        self.step_eager()
        self.step_eager()
        if self.args.no_graph:
            return
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            g1 = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g1, stream=s):
                self._launch()
            g2 = gm = None
            if self.dp:
                gm = self._capture_dp_steps(s)
                if self.shape not in ("bucketed", "sharded"):  # those step eagerly (step())
                    g2 = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(g2, stream=s):
                        self.plan.adam(0, 0.0, advance=True)
            elif not self.prefetch:
                # the production trainer's graphs (trainer.epoch_graph_sizes: ONE graph of an
                # epoch's nb batches; a replay boundary costs ~8 us of idle GPU), plus the
                # trainer.GRAPH_SIZES pieces for partial runs (settle, warmup): n steps replay as
                # trainer.graph_replays(n) -- a timed window of K steps from an epoch start of an
                # nb = K epoch is one replay, exactly what trainer.py replays for an epoch of K
                # batches
                from trainer import GRAPH_SIZES, epoch_graph_sizes
                self.gset = {}
                for n in sorted({x for x in GRAPH_SIZES if x <= self.nb} | set(epoch_graph_sizes(self.nb)), reverse=True):
                    if n <= self.nb:
                        g = torch.cuda.CUDAGraph()
                        with torch.cuda.graph(g, stream=s):
                            self.i = 0
                            self._steps(n)
                        self.gset[n] = g
                gm = self.gset.get(self.GRAPH_STEPS)
        torch.cuda.current_stream().wait_stream(s)
        self.graphs = (g1, g2, gm)
        self.plan.set_batch_index(0)
        self.i = 0
        if self.prefetch:
            self.pipe.start()

    def _wrap(self):
        if self.i == self.nb:
            self.plan.set_batch_index(0)
            self.i = 0
            if self.prefetch:
                self.pipe.start()

    def step_eager(self):
        self._wrap()
        self._steps(1)
        self.i += 1

    def step(self):
        if self.graphs is None or self.prefetch or (self.dp and self.shape in ("bucketed", "sharded")):
            return self.step_eager()
        self._wrap()
        g1, g2, _ = self.graphs
        g1.replay()
        if g2 is not None:
            if torch.distributed.is_initialized():
                torch.distributed.all_reduce(self.plan.grads)
            g2.replay()
        self.i += 1

    def run(self, n):
        """n training steps: single-GPU, the production trainer's graph replays
        (trainer.graph_replays over what is left of the epoch); data-parallel shapes,
        GRAPH_STEPS-step graphs where they fit the epoch, else single steps."""
        gset = getattr(self, "gset", None) if self.graphs is not None else None
        if gset:
            from trainer import graph_replays
            while n > 0:
                self._wrap()
                for g in graph_replays(min(n, self.nb - self.i), tuple(gset)):
                    gset[g].replay()
                    self.i += g
                    n -= g
            return
        gm = self.graphs[2] if self.graphs is not None else None
        while n > 0:
            self._wrap()
            if gm is not None and n >= self.GRAPH_STEPS and self.i + self.GRAPH_STEPS <= self.nb and self.i % 2 == 0:
                gm.replay()
                self.i += self.GRAPH_STEPS
                n -= self.GRAPH_STEPS
            else:
                self.step()
                n -= 1


# The GPU raises its clocks over the first ~25 ms of sustained load: from a cold start the
# headline step replays at ~70 us for ~6 ms and settles at ~65 us after ~27 ms (the 65,536-ray
# step: ~540 -> ~479 us after ~40 ms; tools/step_ramp.py, profiles/r04/step_ramp_*.log).  A
# short window (the driver's 5 warmup + 20 timed steps span 1.7 ms) would time that ramp, not
# the sustained rate a training run sees, so every timed leg first replays its own step,
# untimed, for SETTLE_MS of GPU time -- the count is reported in the line (clock_settle).
SETTLE_MS = float(os.environ.get("INF_BENCH_SETTLE_MS", "100"))
SETTLED = {}


def settle(tr, world, warmup=0, tag=None):
    """Untimed replays of `tr`'s step for about SETTLE_MS ms (a probe of 8 steps sizes it;
    ranks agree on the count, since data-parallel replays carry collectives)."""
    if SETTLE_MS <= 0:
        return 0
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    tr.run(8)
    e1.record()
    torch.cuda.synchronize()
    per = max(e0.elapsed_time(e1) / 8, 1e-3)
    n = min(int(SETTLE_MS / per) + 1, 100000)
    if world > 1:
        t = torch.tensor([n], device="cuda")
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
        n = int(t[0])
    tr.run(n)
    # end where the W warmup steps leave the timed window at an epoch start (single-GPU: the
    # window then replays what trainer.py replays for an epoch of K batches) or on a graph
    # boundary of the data-parallel shapes' GRAPH_STEPS-step graphs
    period = tr.nb if getattr(tr, "gset", None) else tr.GRAPH_STEPS
    extra = (-(tr.i + warmup)) % period
    tr.run(extra)
    if tag is not None:
        SETTLED[tag] = n + 8 + extra
    return n + 8 + extra


def time_steps(tr, steps, warmup, world, tag=None):
    settle(tr, world, warmup, tag)
    tr.run(warmup)
    tr._wrap()  # an epoch wrap due at the window's start (set_batch_index) happens before it
    if world > 1:
        torch.distributed.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record()
    tr.run(steps)
    e1.record()
    torch.cuda.synchronize()
    wall = time.perf_counter() - t0
    if world > 1:
        torch.distributed.barrier()
    ms = e0.elapsed_time(e1)
    t = torch.tensor([ms, wall * 1e3], device="cuda")
    if world > 1:
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MAX)
    return float(t[0]) / steps, float(t[1]) / steps


def strong_local_steps(args, device):
    """N=1: the per-GPU step of each strong-scaling point -- the reference's 4096-ray batch
    split over 8 / 4 / 2 GPUs is 512 / 1024 / 2048 rays per GPU -- in the data-parallel step
    shapes at world 1 (serial: gradient -> [all-reduce] -> Adam; sharded: gradient ->
    [reduce-scatter] -> Adam -> [all-gather] -> image rewrite), collectives absent.  The
    strong-scaling projection adds a collective model to these; the
    N > 1 runs measure the real thing (data_parallel.strong)."""
    out = {}
    for bl in [int(x) for x in args.strong_local.split(",") if x]:
        row = {}
        for shape in ("serial", "sharded"):
            try:
                tr = Trainer(args, device, bl, 0, 1, shape=shape, global_batch=args.strong_batch, dp=True)
            except RuntimeError as exc:  # no fused chain at this batch: the shape does not apply
                row[shape] = repr(exc)
                continue
            tr.capture()
            ms, _ = time_steps(tr, max(20, args.steps // 4), 5, 1)
            tr.gather_state()
            row[shape] = ms
            del tr
            torch.cuda.empty_cache()
        out[str(bl)] = {"gpus": args.strong_batch // bl, "ms_per_step": row,
                        "chain3_workgroups": bl // 16}
    return out


def time_allreduce(tr, steps, warmup, world):
    """The flat-gradient all-reduce alone (P fp32, 3.68 MB at config B), issued as the step
    issues it: captured into a graph of GRAPH_STEPS collectives over RCCL (eager over gloo),
    barrier + synchronize around the timed region, max over ranks."""
    dist = torch.distributed
    grads = tr.plan.grads
    graph = None
    if dist.is_initialized() and dist.get_backend() != "gloo":
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            dist.all_reduce(grads)
            graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(graph, stream=s):
                for _ in range(tr.GRAPH_STEPS):
                    dist.all_reduce(grads)
        torch.cuda.current_stream().wait_stream(s)

    def run(n):
        while n > 0:
            if graph is not None and n >= tr.GRAPH_STEPS:
                graph.replay()
                n -= tr.GRAPH_STEPS
            else:
                if dist.is_initialized():
                    dist.all_reduce(grads)
                n -= 1

    run(warmup)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    run(steps)
    e1.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t = torch.tensor([e0.elapsed_time(e1) / steps], device="cuda")
    if world > 1:
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t[0]), {"bytes": grads.numel() * 4, "in_graph": graph is not None}


def time_stage(plan, stage, reps=20, batch=None, layer=0):
    plan.set_batch_index(0)  # stage replays read batch 0 of the epoch
    plan.run_stage(stage, layer, batch)  # warm
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        flops, byts = plan.run_stage(stage, layer, batch)
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps, flops, byts


def _pmc_traffic(key):
    """HBM bytes per launch from the committed rocprofv3 PMC passes (profiles/traffic.json,
    tools/profile_r02.sh: 2 x FETCH_SIZE + WRITE_SIZE), or None."""
    try:
        return json.load(open(os.path.join(ROOT, "profiles", "traffic.json"))).get(key)
    except Exception:
        return None


def flops_per_ray(k, H, L):
    """Training FLOPs per ray: forward, dX chain and dW."""
    return 2 * (2 * (2 * k * H + (L - 2) * H * H + 3 * H) + (L - 2) * H * H + 3 * H)


def step_roofline(k, H, L, B, P, ms, table_bytes=2, weight_bytes=2, dtype="bf16"):
    """Both t_min terms of one training step: FLOPs vs the dense MFMA
    peak, algorithmic HBM bytes (3 table rows + ids/bary/rgb per ray; Adam's 28 B and three
    weight passes per parameter per step) vs 8 TB/s.  frac = t_min / t_measured."""
    k_pad = -(-k // 128) * 128
    flops = B * flops_per_ray(k, H, L)
    byts = B * (3 * k_pad * table_bytes + 36) + P * (28 + 3 * weight_bytes)
    t_mfma = flops / (PEAK[dtype] * 1e12) * 1e3
    t_hbm = byts / (HBM_PEAK * 1e9) * 1e3
    return {"flops": flops, "bytes": byts, "t_mfma_ms": t_mfma, "t_hbm_ms": t_hbm,
            "bound": "mfma" if t_mfma >= t_hbm else "hbm",
            "mfma_frac": t_mfma / ms, "hbm_frac": t_hbm / ms, "frac": max(t_mfma, t_hbm) / ms,
            "achieved_tflops": flops / (ms * 1e-3) / 1e12, "achieved_gbs": byts / (ms * 1e-3) / 1e9}


def config_d_bench(args, device, B=4096, steps=40):
    """Config D (configs/discretization_agnostic/human_dense.yaml):
    k = 4096 eigenfunctions of a ~500k-vertex discretisation, 8 x 256 MLP, skip 4, L2, Adam;
    the bf16 table is 4.1 GB, far beyond the 256 MB MALL, so every row of the gather is a
    random HBM read.  Graph-replayed fused steps (chain3 with a chunked feature tile), the
    per-kernel times, the standalone gather kernel's HBM rate on the same rays, and both
    roofline terms of the step."""
    import copy
    from inf_hip import STAGE_CHAIN, STAGE_DW_GEMM, STAGE_GATHER, STAGE_UPDATE
    a = copy.copy(args)
    a.k, a.verts, a.no_graph = 4096, 500_000, False
    tr = Trainer(a, device, B, 0, 1, nb=epoch_batches(steps))
    tr.capture()
    ms, _ = time_steps(tr, steps, 8, 1)
    path = tr.plan.last_step_path()
    st = {"chain3": time_stage(tr.plan, STAGE_CHAIN, reps=10, batch=tr.batch),
          "dw_gemm": time_stage(tr.plan, STAGE_DW_GEMM, reps=10)}
    if not tr.plan.last_step_fused_update():
        st["update"] = time_stage(tr.plan, STAGE_UPDATE, reps=10, layer=1)
    gms, _, gbytes = time_stage(tr.plan, STAGE_GATHER, reps=10, batch=tr.batch)
    P = tr.plan.info.num_params
    k_pad = tr.plan.in_pad
    row_bytes = B * 3 * k_pad * 2
    # the reference's own product (mesh.py:313-324 with the loader's index select): the
    # B x k feature matrix, row-major only (inf_gather -> gather_rows_kernel), of the same
    # rays from the same packed bf16 table, into bf16 and into fp32 (the reference's dtype)
    from inf_hip import runtime as RT
    Tb = tr.src.table_for(tr.plan)
    ref_gather = {}
    for name, dt in (("bf16", torch.bfloat16), ("fp32", torch.float32)):
        X = torch.empty((B, k_pad), dtype=dt, device=device)
        RT.gather(Tb, tr.src.vids, tr.src.bary, ray_idx=tr.perm, offset=0, batch=B, out=X)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(20):
            RT.gather(Tb, tr.src.vids, tr.src.bary, ray_idx=tr.perm, offset=0, batch=B, out=X)
        e1.record()
        torch.cuda.synchronize()
        ms_g = e0.elapsed_time(e1) / 20
        out_bytes = X.numel() * X.element_size()
        ref_gather[name] = {"ms": ms_g, "table_gbs": row_bytes / (ms_g * 1e-3) / 1e9,
                            "table_hbm_frac": row_bytes / (ms_g * 1e-3) / 1e9 / HBM_PEAK,
                            "hbm_gbs": (row_bytes + out_bytes + B * 32) / (ms_g * 1e-3) / 1e9,
                            "hbm_frac": (row_bytes + out_bytes + B * 32) / (ms_g * 1e-3) / 1e9 / HBM_PEAK}
        del X
    out = {"config": "human_dense D: k=4096 8x256 skip 4, L2, Adam lr 1e-4, V=500000, bf16 table 4.1 GB",
           "rays_per_step": B, "ms_per_step": ms, "value": B / (ms * 1e-3), "unit": "rays/s", "path": path,
           "roofline": step_roofline(4096, a.hidden, a.layers, B, P, ms),
           "traffic_per_launch": ({"zg": _pmc_traffic("zg_bf16_D4096"), "chain3": _pmc_traffic("chain3_zp_bf16_D4096"),
                                   "dw_gemm_update": _pmc_traffic("lgf_bf16_D4096")} if path == "chain3_zg"
                                  else {"chain3": _pmc_traffic("chain3_chunked_bf16_D4096")}),
           "stages": {kk: {"ms": v[0], "tflops": v[1] / (v[0] * 1e-3) / 1e12} for kk, v in st.items()},
           "gather_kernel": {"ms": gms, "table_row_bytes": row_bytes,
                             "table_gbs": row_bytes / (gms * 1e-3) / 1e9,
                             "table_hbm_frac": row_bytes / (gms * 1e-3) / 1e9 / HBM_PEAK,
                             "note": "standalone gather (X and X^T written) of the step's rays; inside the "
                                     "fused chain the rows go straight to LDS"},
           "reference_gather": dict(ref_gather, note="inf_gather of the step's rays: the B x k feature matrix of "
                                                     "mesh.py:313-324, row-major only (table rows read once, one "
                                                     "output write); hbm_gbs counts rows + output + ray records")}
    del tr
    torch.cuda.empty_cache()
    return out


def _secondary_train(args, device, B, steps, **over):
    """Graph-replayed fused steps of another configuration: rays/s, kernel path, step
    roofline (both terms)."""
    import copy
    a = copy.copy(args)
    for kk, v in over.items():
        setattr(a, kk, v)
    a.no_graph = False
    tr = Trainer(a, device, B, 0, 1, nb=epoch_batches(steps))
    tr.capture()
    ms, _ = time_steps(tr, steps, 4, 1)
    P = tr.plan.info.num_params
    out = {"rays_per_step": B, "ms_per_step": ms, "value": B / (ms * 1e-3), "unit": "rays/s",
           "path": tr.plan.last_step_path(), "dtype": a.mode,
           "roofline": step_roofline(a.k, a.hidden, a.layers, B, P, ms, dtype=a.mode,
                                     table_bytes=2 if a.mode == "bf16" else 4,
                                     weight_bytes=2 if a.mode == "bf16" else 4)}
    del tr
    torch.cuda.empty_cache()
    return out


def bf16x3_mode_bench(args, device):
    """The split-bf16 parity mode (fp32 buffers, GEMM products as hi*hi + hi*lo + lo*hi on
    bf16 matrix cores; meets the 1e-4 RGB bar, tests/test_gpu_bf16x3.py) on the headline
    configuration, against a third of the dense bf16 peak."""
    out = _secondary_train(args, device, args.batch, 40, mode="bf16x3")
    out["config"] = (f"cat k={args.k} {args.layers}x{args.hidden} skip {args.skip}, L2, Adam, bf16x3 mode, "
                     f"V={args.verts}")
    return out


def config_a_bench(args, device):
    """Config A (the reference's CPU-runnable cat case, k=64, 4x128, skip 2)
    on the GPU, beside its CPU leg."""
    out = _secondary_train(args, device, 4096, 80, k=64, layers=4, hidden=128, skip=2, verts=20_000)
    out["config"] = "cat k=64 4x128 skip 2, L2, Adam, V=20000"
    return out


def config_r_bench(args, device):
    """Config R -- the reference's own shipped configuration (configs/texture_reconstruction/
    intrinsic_cat.yaml:25-37): k = list(1023) eigenfunction indices (the MLP input is 1023,
    padded to 1024 with zero columns), 6 x 128 MLP, skip 3, L1 loss, batch 4096, Adam."""
    out = _secondary_train(args, device, 4096, 80, k=1023, layers=6, hidden=128, skip=3, loss="L1")
    out["config"] = f"intrinsic_cat.yaml: k=list(1023) 6x128 skip 3, L1, Adam, V={args.verts}"
    return out


def fp32_mode_bench(args, device):
    """The parity mode (exact-fp32 MFMA layered kernels: the mode that meets the 1e-4 RGB
    bar) on the headline configuration, against the 157.3 TFLOP/s fp32 MFMA peak."""
    out = _secondary_train(args, device, args.batch, 40, mode="fp32")
    out["config"] = f"cat k={args.k} {args.layers}x{args.hidden} skip {args.skip}, L2, Adam, fp32 mode, V={args.verts}"
    return out


def render_bench(args, device):
    """Forward-only render slice (renderer.py:112-146) of a 2048x2048 frame at a 50 % hit
    rate over a V=400k table (config E): gather + MLP + placement into the image."""
    from inf_hip import runtime
    H = W = 2048
    V = 400_000
    m = build_model(args, device)
    rt = m.hip_runtime()
    nhit = H * W // 2
    chunk = int(os.environ.get("INF_RENDER_CHUNK", 1 << 18))
    nstreams = int(os.environ.get("INF_RENDER_STREAMS", "1"))
    plans = [runtime.Plan(args.k, args.hidden, args.layers, args.skip, args.mode, "L2", chunk, rt.arena)
             for _ in range(nstreams)]
    plan = plans[0]
    g = torch.Generator(device="cpu").manual_seed(7)
    E = torch.randn((V, args.k), generator=g)
    E = E / (E.max(0, keepdim=True).values - E.min(0, keepdim=True).values)
    vids = torch.randint(0, V, (nhit, 3), generator=g).to(device)
    u = torch.rand((nhit, 3), generator=g).clamp_min(1e-12)
    bary = (-torch.log(u))
    bary = (bary / bary.sum(1, keepdim=True)).to(device)
    src = runtime.RaySource(E.to(device), vids, bary, None)
    del E
    hit = torch.randperm(H * W, device=device)[:nhit]
    img = torch.empty((H * W, 3), device=device)
    offs = list(range(0, nhit, chunk))
    T = src.table_for(plan)
    project = args.mode == "bf16" and plan.can_project() and os.environ.get("INF_RENDER_PROJECT", "1") != "0"
    P = plan.project_table(T) if project else None
    batches = {False: [plans[j % nstreams].make_batch(source=src, offset=o, batch=min(chunk, nhit - o))
                       for j, o in enumerate(offs)]}
    if project:  # no workspace behind a projected batch: the frame's hits in one persistent launch
        batches[True] = [plan.make_batch(source=src, offset=0, batch=nhit, projected=P)]
    streams = [torch.cuda.current_stream()] + [torch.cuda.Stream() for _ in range(nstreams - 1)]

    def frame(pj):
        img.fill_(1.0)
        if pj:  # the vertices' first-layer projections under the current weights, every frame
            plan.project_table(T, out=P)
        cur = torch.cuda.current_stream()
        for st in streams[1:]:
            st.wait_stream(cur)
        # chunks round-robin over the plans/streams: one chunk's gather overlaps another's chain
        for j, (o, b) in enumerate(zip([0] if pj else offs, batches[pj])):
            with torch.cuda.stream(streams[j % nstreams]):
                plans[j % nstreams].render(b, hit[o:o + b.batch], None, img)
        for st in streams[1:]:
            cur.wait_stream(st)

    def timed(fn, reps=10):
        # untimed frames for SETTLE_MS of GPU time first: each variant's inputs are built on the
        # host while the GPU idles (~140 ms), and the frames right after an idle period time a
        # clock transient (round 6 kernel trace of this leg: the pixel-coherent variant's rprojw
        # launches ran 2247 -> 1875 us over its five timed frames, profiles/r06/render/)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        spent = 0.0
        while True:
            e0.record()
            fn()
            e1.record()
            torch.cuda.synchronize()
            spent += e0.elapsed_time(e1)
            if spent >= SETTLE_MS:
                break
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        return e0.elapsed_time(e1) / reps

    ms_gather = timed(lambda: frame(False))
    ms = timed(lambda: frame(True)) if project else ms_gather
    ms_proj = timed(lambda: plan.project_table(T, out=P)) if project else None
    # both t_min terms of the frame: forward FLOPs of the hits vs the
    # dense MFMA peak; table rows + ids / bary / hit index per hit, the image (fill + pixel
    # writes) and one pass of the bf16 weights vs HBM.  Projected frames: the projection
    # GEMM (V x k_pad x 2H) reads the table once and writes the V x 2H projections; each
    # hit then reads three 2H-wide rows and runs the hidden layers and the head only.
    L, Hd, k = args.layers, args.hidden, args.k
    k_pad = -(-k // 128) * 128
    wbytes = 2 * (2 * k_pad * Hd + (L - 2) * Hd * Hd)
    per_hit_io = 12 + 12 + 8 + 12
    if project:
        Vp = -(-V // 128) * 128
        flops = Vp * 2 * k_pad * 2 * Hd + nhit * 2 * ((L - 2) * Hd * Hd + 3 * 2 * Hd + 3 * Hd)
        byts = (V * k_pad * 2 + Vp * 2 * Hd * 2 + nhit * (3 * 2 * Hd * 2 + per_hit_io) + H * W * 12 + wbytes)
    else:
        flops = nhit * 2 * (2 * k * Hd + (L - 2) * Hd * Hd + 3 * Hd)
        byts = nhit * (3 * k_pad * 2 + per_hit_io) + H * W * 12 + wbytes
    t_mfma = flops / (PEAK[args.mode] * 1e12) * 1e3
    t_hbm = byts / (HBM_PEAK * 1e9) * 1e3
    roof = {"flops": flops, "bytes": byts, "t_mfma_ms": t_mfma, "t_hbm_ms": t_hbm,
            "bound": "mfma" if t_mfma >= t_hbm else "hbm", "mfma_frac": t_mfma / ms, "hbm_frac": t_hbm / ms,
            "frac": max(t_mfma, t_hbm) / ms, "achieved_tflops": flops / (ms * 1e-3) / 1e12,
            "achieved_gbs": byts / (ms * 1e-3) / 1e9}
    if project:  # measured HBM bytes (PMC) of the frame's two launches: projection GEMM + rproj
        # (rprojw.hip's 128-ray tiles for the 8 x 256 field with skip 4, else rproj.hip)
        wide = (Hd, L, args.skip) == (256, 8, 4) and os.environ.get("INF_RPROJ_WIDE", "1") != "0"
        kern = "rprojw" if wide else "rproj"
        tr_g, tr_p = _pmc_traffic(f"project_gemm_{args.mode}_render"), _pmc_traffic(f"{kern}_{args.mode}_render")
        if tr_g is not None and tr_p is not None:
            roof["traffic_projection"] = tr_g
            roof["traffic_" + kern] = tr_p
            roof["traffic"] = tr_g + tr_p
    else:
        tr = _pmc_traffic(f"rchain_{args.mode}_render_{chunk}")
        if tr is not None:  # measured HBM bytes of one launch (PMC), over the frame's launches
            roof["traffic_per_launch"] = tr
            roof["traffic"] = tr * len(offs)
    if roof.get("traffic"):
        # the same frame against its MEASURED HBM bytes (PMC, profiles/traffic.json): the
        # random 2H-wide row reads partly hit the MALL, so the model bytes above overstate
        # the HBM term; the binding term of t_min is recomputed from the measured bytes
        t_pmc = roof["traffic"] / (HBM_PEAK * 1e9) * 1e3
        roof["measured"] = {"hbm_bytes": roof["traffic"], "t_hbm_ms": t_pmc, "hbm_frac": t_pmc / ms,
                            "hbm_gbs": roof["traffic"] / (ms * 1e-3) / 1e9, "mfma_frac": t_mfma / ms,
                            "bound": "mfma" if t_mfma >= t_pmc else "hbm", "frac": max(t_mfma, t_pmc) / ms}
    variants = {}
    if project:  # SURVEY.md §8(d)'s second distributions: pixel-coherent ids, a 100 % hit rate
        def variant(n, coherent):
            gv = torch.Generator(device="cpu").manual_seed(11)
            if coherent:  # neighbouring pixels on nearby vertices, hits in pixel order
                base = torch.randint(0, V - 64, (n // 64 + 1,), generator=gv).repeat_interleave(64)[:n]
                vv = (base[:, None] + torch.randint(0, 64, (n, 3), generator=gv)).clamp_max(V - 1)
                hv = torch.randperm(H * W, generator=gv)[:n].sort().values
            else:
                vv = torch.randint(0, V, (n, 3), generator=gv)
                hv = torch.randperm(H * W, generator=gv)[:n]
            uv = -torch.log(torch.rand((n, 3), generator=gv).clamp_min(1e-12))
            sv = runtime.RaySource(src.E, vv.to(device), (uv / uv.sum(1, keepdim=True)).to(device), None,
                                   validate=False)
            sv._tables = src._tables  # the packed table is shared
            bv = plan.make_batch(source=sv, offset=0, batch=n, projected=P)
            hv = hv.to(device)

            def fr():
                img.fill_(1.0)
                plan.project_table(T, out=P)
                plan.render(bv, hv, None, img)
            t = timed(fr)
            return {"hits": n, "ms_per_frame": t, "pixels_per_s": H * W / (t * 1e-3)}
        variants["coherent_ids_50pct"] = variant(nhit, True)
        variants["random_ids_100pct"] = variant(H * W, False)
    return {"value": H * W / (ms * 1e-3), "unit": "pixels/s", "ms_per_frame": ms, "frame": f"{H}x{W}",
            "hits": nhit, "verts": V, "chunk": chunk, "streams": nstreams, "variants": variants,
            "path": ("projected table (inf_project_table per frame + rprojw, 128-ray tiles)" if project and wide else
                     "projected table (inf_project_table per frame + rproj)" if project else "feature gather rchain"),
            "projection_ms": ms_proj, "ms_per_frame_feature_gather": ms_gather,
            "feature_gather_pixels_per_s": H * W / (ms_gather * 1e-3), "roofline": roof}


def torus_mesh(nu=640, nv=320, R=1.0, r=0.4):
    """Synthetic render mesh: a torus grid of nu * nv vertices, 2 nu nv faces."""
    u = np.linspace(0, 2 * np.pi, nu, endpoint=False)
    v = np.linspace(0, 2 * np.pi, nv, endpoint=False)
    uu, vv = np.meshgrid(u, v, indexing="ij")
    V = np.stack([(R + r * np.cos(vv)) * np.cos(uu), (R + r * np.cos(vv)) * np.sin(uu), r * np.sin(vv)], -1)
    i, j = np.meshgrid(np.arange(nu), np.arange(nv), indexing="ij")
    a = i * nv + j
    b = ((i + 1) % nu) * nv + j
    c = ((i + 1) % nu) * nv + (j + 1) % nv
    d = i * nv + (j + 1) % nv
    F = np.concatenate([np.stack([a, b, c], -1).reshape(-1, 3), np.stack([a, c, d], -1).reshape(-1, 3)])
    return V.reshape(-1, 3), F


def render_e2e_bench(args, device):
    """End-to-end render of a 2048x2048 view (renderer.py:64-146 incl. ray casting,
    mesh.py:171-251): camera rays cast against a device BVH of a
    409,600-face mesh, hit compaction, then gather + MLP + placement -- Renderer.render."""
    import mesh as MS
    from renderer import Renderer
    H = W = 2048
    Vn, Fn = torus_mesh()
    g = torch.Generator(device="cpu").manual_seed(11)
    E = torch.randn((Vn.shape[0], args.k), generator=g)
    E = E / (E.max(0, keepdim=True).values - E.min(0, keepdim=True).values)
    m = build_model(args, device)
    t0 = time.perf_counter()
    r = Renderer(m, MS.TriMesh(Vn, Fn), eigenfunctions=E, H=H, W=W, device=device)
    build_s = time.perf_counter() - t0
    th = 0.5
    Rm = np.array([[1, 0, 0], [0, np.cos(th), -np.sin(th)], [0, np.sin(th), np.cos(th)]])
    cam = torch.from_numpy(np.concatenate([Rm, (Rm @ np.array([0.0, 0, -3.2]))[:, None]], 1)).float()
    K = torch.tensor([[1400.0, 0, 1024], [0, 1400, 1024], [0, 0, 1]])
    bvh = r.ray_mesh_intersector
    r.render(cam, K)  # warm (plan, tables)
    torch.cuda.synchronize()
    reps = 5
    t0 = time.perf_counter()
    for _ in range(reps):
        img = r.render(cam, K)
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) / reps * 1e3
    # the cast alone (HIP events; one ray per pixel)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        face, bary, dirs = bvh.cast(cam, K, H, W)
    e1.record()
    torch.cuda.synchronize()
    cast_ms = e0.elapsed_time(e1) / reps
    hits = int((face >= 0).sum().item())
    return {"value": H * W / (ms * 1e-3), "unit": "pixels/s", "ms_per_frame": ms, "frame": f"{H}x{W}",
            "faces": int(Fn.shape[0]), "hits": hits, "raycast_ms": cast_ms,
            "raycast_rays_per_s": H * W / (cast_ms * 1e-3), "bvh_nodes": bvh.num_nodes, "bvh_depth": bvh.depth,
            "bvh_build_s": build_s, "timing": "host wall clock per Renderer.render call (incl. the hit-count readback)",
            "projected_table": "computed on the warm-up frame and kept by the Renderer across the timed frames "
                               "(the weights do not change between them: inf_plan_weight_generation)"}


def rff_bench(args, device, B=4096, reps=6):
    """Secondary line: the extrinsic RFF configuration (configs tf_rff_*: k = 510 RFF
    features -> in_dim 1023, 6 x 128 MLP, skip 3, L1, Adam), fused gather + encode + step,
    graph-replayed like the headline.  Synthetic V x 3 positions in [-1, 1]^3."""
    import model as M
    from inf_hip import runtime
    torch.manual_seed(0)
    m = M.make_model({"feature_strategy": "rff", "k": 510, "embed_std": 8, "num_layers": 6, "mlp_hidden_dim": 128,
                      "skip_layer_idx": 3, "kernels": {"mode": args.mode}}).to(device)
    m.kernel_mode = args.mode
    rt = m.hip_runtime()
    rt.ensure_optimizer_arenas()
    plan = runtime.Plan(m.in_dim, 128, 6, 3, args.mode, "L1", B, rt.arena, rt.grads, rt.exp_avg, rt.exp_avg_sq)
    plan.encoding = m._encoding()
    plan.set_lr(1e-4)
    G = 8
    nb = 4 * G
    N = nb * B
    g = torch.Generator(device="cpu").manual_seed(3)
    P = (torch.rand((args.verts, 3), generator=g) * 2 - 1).to(device)
    vids = torch.randint(0, args.verts, (N, 3), generator=g).to(device)
    bary = -torch.log(torch.rand((N, 3), generator=g).clamp_min(1e-12))
    bary = (bary / bary.sum(1, keepdim=True)).to(device)
    rgb = torch.rand((N, 3), generator=g).to(device)
    src = runtime.RaySource(P, vids, bary, rgb)
    perm = torch.randperm(N, device=device)
    b = plan.make_batch(source=src, ray_idx=perm, offset=0, batch=B, offset_from_ctrl=True, loss="L1")
    plan.set_batch_index(0)
    plan.train_step(b, None, apply_adam=True, advance=True)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        gm = torch.cuda.CUDAGraph()
        with torch.cuda.graph(gm, stream=s):
            for _ in range(G):
                plan.train_step(b, None, apply_adam=True, advance=True)
    torch.cuda.current_stream().wait_stream(s)
    plan.set_batch_index(0)
    for _ in range(2):
        gm.replay()
    plan.set_batch_index(0)
    torch.cuda.synchronize()
    t0, t1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0.record()
    for i in range(reps):
        if (i * G) % nb == 0:
            plan.set_batch_index(0)
        gm.replay()
    t1.record()
    torch.cuda.synchronize()
    ms = t0.elapsed_time(t1) / (reps * G)
    return {"config": "tf_rff: rff k=510 (in_dim 1023), 6x128 skip 3, L1, Adam", "rays_per_step": B,
            "ms_per_step": ms, "value": B / (ms * 1e-3), "unit": "rays/s"}


PSNR_RUNS = {
    # fixture: (workload, model keys, loss)
    "g8_train_curve.npz": ("reference synthetic run G8 (k=64 4x128 skip 2, L1, lr 1e-3, 12 epochs)",
                           {"k": 64, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2}, "L1"),
    "g13_train_curve_B_L2.npz": ("reference synthetic run G13 on config B's MLP (k=1024 8x256 skip 4, L2, lr 1e-4, "
                                 "12 epochs)",
                                 {"k": 1024, "num_layers": 8, "mlp_hidden_dim": 256, "skip_layer_idx": 4}, "L2"),
    # the reference's own shipped configuration (intrinsic_cat.yaml:24-37), k = the fixture's list of 1023 indices
    "g16_train_curve_R.npz": ("reference synthetic run G16 on config R exactly (k=list(1023) 6x128 skip 3, L1, lr 1e-4, "
                              "batch 4096, 12 epochs)",
                              {"k": "k_list", "num_layers": 6, "mlp_hidden_dim": 128, "skip_layer_idx": 3}, "L1"),
}


def psnr_vs_ref(mode, fixture="g8_train_curve.npz"):
    """'PSNR vs ref' of BASELINE.json's metric: the reference's own 12-epoch synthetic
    training runs (tests/golden/g8_train_curve.npz, on the benchmarked MLP
    g13_train_curve_B_L2.npz, and on the reference's own cat configuration
    g16_train_curve_R.npz; produced by importing the reference; no dataset is available
    offline) re-run through this framework's Trainer (trainer.py mirror, fused HIP steps)
    -- validation epoch-PSNR curve against the reference's."""
    import tempfile

    import config
    from ray_dataloader import RayDataLoader
    from trainer import Trainer
    workload, mkeys, loss = PSNR_RUNS[fixture]
    d = np.load(os.path.join(ROOT, "tests", "golden", fixture))
    if mkeys["k"] == "k_list":
        mkeys = dict(mkeys, k=[int(x) for x in d["k_list"]])
    with tempfile.TemporaryDirectory() as out:
        cfg = {"seed": 0, "data": {"img_height": 8, "img_width": 8},
               "model": dict(mkeys, kernels={"mode": mode}),
               "training": {"out_dir": out, "batch_size": int(d["batch"]), "lr": float(d["lr"]), "loss_type": loss,
                            "render_every": 1000, "print_every": 1000, "epochs": len(d["val_psnr"]),
                            "checkpoint_every": 1000}}
        E = torch.from_numpy(d["E"])
        mk = lambda p, drop: RayDataLoader(E, "efuncs", torch.from_numpy(d[f"{p}_vids"]), torch.from_numpy(d[f"{p}_bary"]),
                                           torch.from_numpy(d[f"{p}_rgb"]), None, None, int(d["batch"]), False, drop,
                                           device="cuda")
        torch.manual_seed(0)
        model, optim = config.get_model_and_optim(cfg, None, "cuda")
        model.kernel_mode = mode
        tr = Trainer(model, optim, config.get_loss_fn(cfg), None, {"train": mk("tr", True), "val": mk("va", False)},
                     None, cfg, "cuda")
        tr.train()
        rows = [json.loads(x) for x in open(os.path.join(out, "logs", "scalars.jsonl"))]
    val = np.array([r["value"] for r in rows if r["tag"] == "Val Epoch-PSNR"])
    ref = np.asarray(d["val_psnr"], dtype=np.float64)
    return {"workload": workload, "mode": mode,
            "ref_final_db": float(ref[-1]), "final_db": float(val[-1]), "delta_final_db": float(val[-1] - ref[-1]),
            "max_abs_delta_db": float(np.abs(val - ref).max())}


def _cpu_weights(k, H, L, s):
    import model as M
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s})
    return {n: p.detach().numpy().copy() for n, p in m.named_parameters()}


def _cpu_table(V, k, seed, device):
    """The GPU legs' synthetic table (randn + the reference's column rescale), on the host:
    drawn on the device for the large tables and copied over."""
    if V * k > (1 << 26):
        g = torch.Generator(device=device).manual_seed(seed)
        E = torch.randn((V, k), generator=g, device=device)
        E /= E.max(0, keepdim=True).values - E.min(0, keepdim=True).values
        out = E.cpu()
        del E
        torch.cuda.empty_cache()
        return out
    g = torch.Generator().manual_seed(seed)
    E = torch.randn((V, k), generator=g)
    return E / (E.max(0, keepdim=True).values - E.min(0, keepdim=True).values)


def cpu_leg(kind, k, H, L, s, V, B, seconds, device, max_iters=400):
    """The reference's PyTorch-CPU op sequence (oracle/torch_cpu.py: index + bmm gather,
    F.linear layers with the concatenating skip, mse_loss, autograd, torch.optim.Adam) on
    this host's cores, same configuration and table size as the GPU leg, a bounded sample of
    ~`seconds`.  kind "train": steps of B rays -> rays/s; "render": forward of 2^15-hit
    batches (renderer.py:112-146's batchify size) and the scatter into the image -> hits/s."""
    from oracle import torch_cpu as T
    cores = int(os.environ.get("OMP_NUM_THREADS") or len(os.sched_getaffinity(0)))
    torch.set_num_threads(cores)
    w = _cpu_weights(k, H, L, s)
    E = _cpu_table(V, k, 1, device)
    g = torch.Generator().manual_seed(0)
    tt = T.TorchTrainer(w, L, s, 1e-4, "L2")
    img = torch.ones((2048 * 2048, 3)) if kind == "render" else None

    def rays(n):
        vids = torch.randint(0, V, (n, 3), generator=g)
        u = torch.rand((n, 3), generator=g).clamp_min(1e-12)
        bary = -torch.log(u)
        return vids, bary / bary.sum(1, keepdim=True)

    def one():
        if kind == "train":
            vids, bary = rays(B)
            tt.step(T.gather(E, vids, bary), torch.rand((B, 3), generator=g))
        else:
            vids, bary = rays(B)
            hit = torch.randint(0, img.shape[0], (B,), generator=g)
            with torch.no_grad():
                img[hit] = tt.forward(T.gather(E, vids, bary))

    one()
    t0 = time.perf_counter()
    n = 0
    while time.perf_counter() - t0 < seconds and n < max_iters:
        one()
        n += 1
    dt = time.perf_counter() - t0
    what = "train steps" if kind == "train" else "forward + scatter batches"
    return {"value": n * B / dt, "unit": "rays/s" if kind == "train" else "hits/s", "cores": cores, "kind": "port",
            "sample": f"{n} {what} of the reference's PyTorch-CPU op sequence (oracle/torch_cpu.py, fp32) of {B} "
                      f"rays, k={k} {L}x{H} skip {s}, V={V}, {dt:.1f} s"}


def cpu_baselines(args, device):
    """CPU baselines of SURVEY.md §8(d): configs A, B, D (train) and E (forward + scatter),
    each at the GPU leg's table size.  B (the headline) is `cpu_baseline` proper."""
    sec = args.cpu_seconds
    H, L, s = args.hidden, args.layers, args.skip
    out = {"B": cpu_leg("train", args.k, H, L, s, args.verts, 4096, sec, device)}
    out["A"] = cpu_leg("train", 64, 128, 4, 2, 20_000, 4096, sec / 2, device)
    out["D"] = cpu_leg("train", 4096, H, L, s, 500_000, 4096, sec, device, max_iters=100)
    e = cpu_leg("render", args.k, H, L, s, 400_000, 1 << 15, sec, device)
    e["pixels_per_s"] = e["value"] * 2  # the GPU leg's frame: 50 % of the pixels hit
    out["E"] = e
    return out


def epoch_batches(steps):
    """Batches per epoch of a single-GPU timed leg: the timed window of K steps is one epoch
    of K batches (at least 8), replayed as trainer.py replays an epoch -- one graph."""
    return max(8, int(steps))


def summary_of(line):
    """Compact digest of the line's legs (times in us, rates in M/s or G/s), emitted as the
    line's last key."""
    def us(x):
        return None if x is None else round(x * 1e3, 2)

    def get(d, *path):
        for p in path:
            if not isinstance(d, dict) or p not in d:
                return None
            d = d[p]
        return d

    s = {"B_us": us(line["ms_per_step"]), "B_Mrays": round(line["value"] / 1e6, 2),
         "stages_us": {k: us(v.get("ms")) for k, v in (line.get("stages") or {}).items()},
         "chain3_frac": round(line["roofline"]["frac"], 4)}
    for name, leg in (line.get("secondary") or {}).items():
        s[name + "_us"] = us(leg.get("ms_per_step"))
    s["D_us"] = us(get(line, "config_D", "ms_per_step"))
    s["large_us"] = {k: us(v.get("ms_per_step")) for k, v in (line.get("large_batch") or {}).items()}
    def r4(x):
        return None if x is None else round(x, 4)

    s["render_ms"] = r4(get(line, "render", "ms_per_frame"))
    s["render_Gpix"] = None if s["render_ms"] is None else round(line["render"]["value"] / 1e9, 3)
    s["projection_ms"] = r4(get(line, "render", "projection_ms"))
    s["render_coherent_ms"] = r4(get(line, "render", "variants", "coherent_ids_50pct", "ms_per_frame"))
    s["strong_local_us"] = {k: {sh: us(t) if isinstance(t, float) else t for sh, t in v["ms_per_step"].items()}
                            for k, v in (line.get("strong_scaling_local_steps") or {}).items()}
    dp = line.get("data_parallel")
    if dp:
        s["dp_us"] = {k: us(v["ms_per_step"]) for k, v in dp.items() if isinstance(v, dict) and "ms_per_step" in v}
    s["rff_us"] = us(get(line, "extrinsic_rff", "ms_per_step"))
    s["cpu_rays"] = r4(get(line, "cpu_baseline", "value"))
    return s


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1 or os.environ.get("INF_BENCH_DP"):
        if os.environ.get("INF_DP_BACKEND") == "gloo":
            # rehearsal of the N > 1 code path on a box with fewer GPUs than ranks (RCCL
            # refuses two ranks on one device): ranks share devices, eager all-reduce
            local = local % max(1, torch.cuda.device_count())
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("gloo")
        else:
            torch.cuda.set_device(local)
            torch.distributed.init_process_group("nccl", device_id=torch.device("cuda", local))
    device = torch.device("cuda", local)
    torch.cuda.set_device(device)

    dp_mode = world > 1 or bool(os.environ.get("INF_BENCH_DP"))
    dp_shapes = None
    chosen = None
    if dp_mode:
        # the data-parallel step in each of its shapes (dp.py picks the fastest the same way),
        # and the gradient all-reduce alone; `value` is the fastest shape's
        dp_shapes = {}
        best = None
        for shape in [x for x in os.environ.get("INF_DP_SHAPES", "serial,prefetch,bucketed,sharded").split(",") if x]:
            tr = Trainer(args, device, args.batch, rank, world, shape=shape)
            tr.capture()
            ms_s, wall_s = time_steps(tr, args.steps, args.warmup, world, tag="dp_" + shape)
            tr.gather_state()
            dp_shapes[shape] = {"ms_per_step": ms_s, "value": world * args.batch / (ms_s * 1e-3),
                                "allreduce_in_graph": tr.ar_in_graph, "prefetch_active": bool(tr.prefetch)}
            if best is None or ms_s < best[1]:
                if best is not None:
                    del best[0]
                best = [tr, ms_s, wall_s, shape]
            else:
                del tr
            torch.cuda.empty_cache()
        tr, ms, wall_ms, chosen = best[0], best[1], best[2], best[3]
        ar_ms, ar_info = time_allreduce(tr, args.steps, args.warmup, world)
        dp_shapes["allreduce_alone_ms"] = ar_ms
        dp_shapes["allreduce"] = ar_info
        dp_shapes["chosen"] = chosen
        dp_shapes["note"] = ("serial: fused step -> flat-gradient all-reduce -> Adam in order; prefetch: the next "
                             "batch's gather on a side stream beside the all-reduce; bucketed: the dW GEMM in two "
                             "halves, bucket 1 all-reduced beside the second; sharded: reduce-scatter of the "
                             "gradient -> Adam on 1/N of the parameters -> all-gather of the new bf16 weights; "
                             "value = the fastest shape (dp.py's autotune picks the same way)")
        if world > 1:
            # strong scaling (nn.DataParallel semantics, reference train.py:46-48): the YAML's
            # global batch of 4096 split over the ranks, in the chosen shape (serial if it cannot)
            gb = args.strong_batch
            bl = -(-gb // world)
            st_shape = chosen if chosen != "prefetch" else "serial"
            try:
                trs = Trainer(args, device, bl, rank, world, shape=st_shape, global_batch=gb)
            except RuntimeError:
                st_shape = "serial"
                trs = Trainer(args, device, bl, rank, world, shape=st_shape, global_batch=gb)
            trs.capture()
            ms_st, _ = time_steps(trs, args.steps, args.warmup, world)
            trs.gather_state()
            dp_shapes["strong"] = {"global_batch": gb, "rays_per_gpu": bl, "shape": st_shape, "ms_per_step": ms_st,
                                   "value": gb / (ms_st * 1e-3), "unit": "rays/s",
                                   "note": "the reference's batch of 4096 split over the GPUs (DataParallel "
                                           "semantics); `value` above is weak scaling (4096 rays per GPU)"}
            del trs
            torch.cuda.empty_cache()
    else:
        tr = Trainer(args, device, args.batch, rank, world, nb=epoch_batches(args.steps))
        tr.capture()
        ms, wall_ms = time_steps(tr, args.steps, args.warmup, world, tag="headline")
    tr_ar_in_graph = tr.ar_in_graph
    value = world * args.batch / (ms * 1e-3)

    from inf_hip import STAGE_CHAIN, STAGE_DW_GEMM, STAGE_GATHER, STAGE_UPDATE
    # per-kernel times (HIP events around repeated launches of one stage on its saved inputs)
    stages = {}
    fused_update = tr.plan.last_step_fused_update()
    # the bf16 step's dW GEMM runs the update inside its launch (lgemm GT: split-K 1, each block
    # Adam on its own tile): one stage; otherwise the GEMM and the update launch
    stages["dw_gemm"] = time_stage(tr.plan, STAGE_DW_GEMM)
    if not fused_update:
        stages["update"] = time_stage(tr.plan, STAGE_UPDATE, layer=1)  # Adam + weight images, as in the step
    chain3 = (args.mode == "bf16" and args.batch <= 8192 and args.hidden in (128, 256)
              and not os.environ.get("INF_NO_CHAIN") and not os.environ.get("INF_NO_CHAIN3"))
    if chain3:
        # the gather runs inside the fused chain
        stages["chain3"] = time_stage(tr.plan, STAGE_CHAIN, batch=tr.batch)
    else:
        stages["gather"] = time_stage(tr.plan, STAGE_GATHER, batch=tr.batch)
        if args.mode == "bf16" and not os.environ.get("INF_NO_CHAIN"):
            stages["chain"] = time_stage(tr.plan, STAGE_CHAIN, batch=tr.batch)
    mfma_stages = {k: v for k, v in stages.items() if k in ("dw_gemm", "chain", "chain3")}
    dom = max(mfma_stages, key=lambda k: mfma_stages[k][0])
    dom_ms, dom_flops, _ = stages[dom]
    achieved = dom_flops / (dom_ms * 1e-3) / 1e12
    dw_ms = stages["dw_gemm"][0]
    traffic = None
    # HBM bytes per launch of the dominant kernel from the committed rocprofv3 PMC passes of
    # this same command (tools/profile.sh: 2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md)
    pmc_path = os.path.join(ROOT, "profiles", "traffic.json")
    if os.path.exists(pmc_path):
        try:
            traffic = json.load(open(pmc_path)).get(f"{dom}_{args.mode}_B{args.batch}")
        except Exception:
            traffic = None

    only = {x for x in args.only.split(",") if x}

    def want(section):
        return not only or section in only

    extra = {}
    for eb in [int(x) for x in args.extra_batches.split(",") if x and want("large")]:
        if eb == args.batch:
            continue
        del tr
        torch.cuda.empty_cache()
        tr2 = Trainer(args, device, eb, rank, world)
        tr2.capture()
        ms2, _ = time_steps(tr2, max(10, args.steps // 8), 3, world)
        d_ms, d_fl, _ = time_stage(tr2.plan, STAGE_DW_GEMM, reps=5)
        extra[str(eb)] = {"value": world * eb / (ms2 * 1e-3), "ms_per_step": ms2,
                          "dw_gemm_tflops": d_fl / (d_ms * 1e-3) / 1e12}
        tr = tr2

    del tr
    torch.cuda.empty_cache()
    config_d = None
    if rank == 0 and world == 1 and not args.no_config_d and args.mode == "bf16" and want("configD"):
        config_d = config_d_bench(args, device)

    render = extrinsic = None
    if not args.no_render and rank == 0:
        if want("render"):
            render = render_bench(args, device)
            render["end_to_end"] = render_e2e_bench(args, device)
        if want("rff"):
            extrinsic = rff_bench(args, device)

    psnr = None
    if rank == 0 and world == 1 and not args.no_render and want("psnr"):
        try:
            psnr = [psnr_vs_ref(m, f) for f in PSNR_RUNS for m in ("bf16", "fp32")]
        except Exception as exc:  # reported, never fatal to the throughput line
            psnr = {"error": repr(exc)}

    strong_local = None
    if rank == 0 and world == 1 and want("strong") and args.mode == "bf16":
        strong_local = strong_local_steps(args, device)

    secondary = {}
    if rank == 0 and world == 1 and want("configs"):
        secondary["A"] = config_a_bench(args, device)
        secondary["R"] = config_r_bench(args, device)
        if args.mode == "bf16":
            secondary["fp32_mode_B"] = fp32_mode_bench(args, device)
            secondary["bf16x3_B"] = bf16x3_mode_bench(args, device)

    cpu = cpu_all = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and want("cpu"):
        cpu_all = cpu_baselines(args, device)
        cpu = dict(cpu_all["B"])
        cpu["other_configs"] = {kk: v for kk, v in cpu_all.items() if kk != "B"}

    if rank == 0:
        L, H, k = args.layers, args.hidden, args.k
        k_pad = -(-k // 128) * 128
        flops_ray = flops_per_ray(k, H, L)
        B = args.batch

        def stage_line(name, v):
            ms_, fl, by = v
            d = {"ms": ms_, "tflops": fl / (ms_ * 1e-3) / 1e12 if fl else None}
            if fl:
                d["mfma_frac"] = d["tflops"] / PEAK[args.mode]
            if name == "chain3":
                # run_stage's byte count is the L2 -> CU stream (every workgroup re-reads the
                # weight images) plus HBM rows: reported as such, NOT as an HBM fraction.  The
                # HBM term uses the algorithmic bytes: the table rows and per-ray records, one
                # pass over the weight images, and the X^T / Y^T / dZ^T images + partials the
                # unfused dW GEMM reads back (listed separately as intermediates)
                rows = B * (3 * k_pad * 2 + 36)
                weights = 2 * (2 * k_pad * H + 2 * (L - 2) * H * H)
                inter = B * (k_pad + (2 * L - 3) * H) * 2 + (B // 16) * 4 * ((L - 1) * H + 3 * H)
                d["l2_to_cu_gbs"] = by / (ms_ * 1e-3) / 1e9
                d["hbm_alg_bytes"] = rows + weights
                d["hbm_intermediate_bytes"] = inter
                d["hbm_gbs"] = (rows + weights + inter) / (ms_ * 1e-3) / 1e9
                d["hbm_frac"] = d["hbm_gbs"] / HBM_PEAK
            elif by:
                d["hbm_gbs"] = by / (ms_ * 1e-3) / 1e9
                d["hbm_frac"] = d["hbm_gbs"] / HBM_PEAK
            return d

        stage_lines = {kk: stage_line(kk, v) for kk, v in stages.items()}
        P = sum(x for x in (
            k * H + H, (L - 3) * (H * H + H), H * H + H + k * H + H, 3 * H + 3))
        dom_line = stage_lines[dom]
        line = {
            "metric": "training rays/sec (k=1024, 8x256 MLP)",
            "value": value,
            "unit": "rays/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "clock_settle": {"ms": SETTLE_MS, "steps": SETTLED.get("headline", SETTLED.get("dp_" + str(chosen))),
                             "note": "untimed replays of the same step before the W warmup steps (the GPU's "
                                     "clocks ramp over ~25 ms of load, tools/step_ramp.py), ending so "
                                     "that the timed window starts on an 8-step graph boundary; "
                                     "INF_BENCH_SETTLE_MS=0 disables"},
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": args.mode,
            "data": "synthetic (randn table with reference column rescale, uniform vertex ids, Dirichlet "
                    "barycentrics, U[0,1) colours); seed-0 reference init",
            "config": {"workload": f"cat texture_reconstruction k={k} {L}x{H} MLP skip {args.skip}, L2, Adam "
                                   f"lr 1e-4, fused gather+fwd+bwd+Adam step",
                       "rays_per_gpu_per_step": args.batch, "global_batch": args.batch * world,
                       "verts": args.verts, "parallelism": f"dp{world}", "graph": not args.no_graph,
                       "allreduce_in_graph": tr_ar_in_graph},
            "model_tflops": flops_ray * value / 1e12,
            "roofline": {"bound": "mfma", "kernel": KERNEL_NAMES[dom],
                         "achieved": achieved, "peak": PEAK[args.mode], "unit": "TFLOP/s",
                         "frac": achieved / PEAK[args.mode], "traffic": traffic,
                         "avg_ms": dom_ms, "flops_per_launch": dom_flops,
                         "hbm_term": {"alg_bytes": dom_line.get("hbm_alg_bytes"),
                                      "intermediate_bytes": dom_line.get("hbm_intermediate_bytes"),
                                      "achieved_gbs": dom_line.get("hbm_gbs"), "peak_gbs": HBM_PEAK,
                                      "frac": dom_line.get("hbm_frac")}},
            "step_roofline": step_roofline(k, H, L, B, P, ms, dtype=args.mode,
                                           table_bytes=2 if args.mode == "bf16" else 4,
                                           weight_bytes=2 if args.mode == "bf16" else 4),
            "stages": stage_lines,
            "host_wall_ms_per_step": wall_ms,
            "data_parallel": dp_shapes,
            "strong_scaling_local_steps": strong_local,
            "large_batch": extra,
            "config_D": config_d,
            "secondary": secondary,
            "render": render,
            "extrinsic_rff": extrinsic,
            "psnr_vs_ref": psnr,
            "cpu_baseline": cpu,
        }
        # last key: every leg's headline number in a few hundred bytes, so the tail of the
        # line (a driver keeps the last 8 KB of stdout) carries them all
        line["summary"] = summary_of(line)
        print(json.dumps(line))
    if torch.distributed.is_initialized():
        torch.distributed.destroy_process_group()


if __name__ == "__main__":
    main()
