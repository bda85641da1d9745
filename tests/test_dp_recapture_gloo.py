"""dp.DataParallelEpoch's collective bookkeeping at world 2 on CPU (gloo), with fakes for
the HIP plan: when only rank 0's plan changes between epochs (rank 0 alone renders the
validation views, and a render can grow the model's plan), EVERY rank must re-capture
together, so the all-reduces each rank issues stay matched in number and order.  The
graph replays are stood in for by fake graphs that run the step's all-reduce eagerly,
exactly the collective a captured RCCL graph would replay.  Also: check_replicas raises
when one rank's parameters differ by a single bit."""
import os
import socket

import torch
import torch.distributed as dist
import torch.multiprocessing as mp

P = 37  # parameters of the fake model


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Plan:
    def __init__(self, log):
        self.log = log
        self.params = torch.zeros(P)
        self.exp_avg = torch.zeros(P)
        self.exp_avg_sq = torch.zeros(P)
        self.ctrl = torch.zeros(56, dtype=torch.uint8)

    def make_batch(self, **kw):
        return kw

    def set_batch_index(self, i):
        pass

    def reset_epoch_sums(self):
        pass

    def set_step(self, s):
        pass

    def sync_shadow(self):
        pass

    def train_step(self, batch, pred, apply_adam=False, xslot=None):
        self.log.append("step")

    def adam(self, step=0, lr=0.0, advance=False):
        self.log.append("adam")

    def read_ctrl(self):
        return {"epoch_loss": 1.0, "epoch_sse": 2.0}


class _Rt:
    def __init__(self):
        self.device = torch.device("cpu")
        self.grads = torch.ones(P)
        self.arena = torch.zeros(P)

    def ensure_optimizer_arenas(self):
        pass


class _Model:
    def __init__(self, log):
        self.rt = _Rt()
        self.log = log
        self.plan = _Plan(log)

    def hip_runtime(self):
        return self.rt

    def hip_plan(self, bs, loss):
        return self.plan


class _Optim:
    def fused_group_for(self, model):
        return None

    def sync_runtime_state(self, *a):
        pass

    def after_fused_steps(self, *a):
        pass


class _Loader:
    def __init__(self, N, B):
        self.N, self.B = N, B
        self.source = object()
        self.idxs = torch.arange(N)

    def __iter__(self):
        return self

    def __next__(self):
        raise StopIteration

    def __len__(self):
        return self.N // self.B


class _Graph:
    """A replayed captured step: the all-reduce it holds runs as the RCCL graph would."""

    def __init__(self, epoch, steps):
        self.epoch, self.steps = epoch, steps

    def replay(self):
        for _ in range(self.steps):
            self.epoch._step(self.epoch._rt, self.epoch._plan, None)


def _worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "intrinsic-neural-fields_amd"))
    import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    log = []
    calls = {"capture": 0, "allreduce": 0}
    real_ar = dp.allreduce_grads

    def counting_ar(flat, group=None):
        calls["allreduce"] += 1
        return real_ar(flat, group)

    dp.allreduce_grads = counting_ar

    class Epoch(dp.DataParallelEpoch):
        def graph_collective(self):
            return True  # take the captured-graph branch (RCCL's) on gloo

        def _capture(self, plan, rt, batch, full=2):
            calls["capture"] += 1
            self._plan, self._rt = plan, rt
            self._tail_all_reduce(rt, plan)  # the eager warm-up's collective, as the real one
            self.graph = (_Graph(self, 1), _Graph(self, self.GRAPH_STEPS))

    model = _Model(log)
    trainer = type("T", (), {})()
    trainer.model, trainer.optim = model, _Optim()
    trainer.loss_fn = type("L", (), {"loss_type": "L2"})()
    loader = _Loader(N=20 * 64, B=64)
    ep = Epoch()
    ok = True
    try:
        for epoch in range(3):
            if epoch == 1 and rank == 0:
                model.plan = _Plan(log)  # rank 0 rendered: its model now holds a larger plan
            ep.run(trainer, loader)
    except Exception as exc:  # a mismatched collective surfaces as a gloo error
        ok = repr(exc)
    counts = torch.tensor([calls["capture"], calls["allreduce"]])
    gathered = [torch.zeros_like(counts) for _ in range(world)]
    dist.all_gather(gathered, counts)
    # check_replicas: one bit of rank 1's parameters flipped
    arena = torch.linspace(-1, 1, P)
    dp.check_replicas(arena)
    if rank == 1:
        arena.view(torch.int32)[5] ^= 1
    try:
        dp.check_replicas(arena)
        caught = False
    except RuntimeError as exc:
        caught = "diverged" in str(exc)
    if rank == 0:
        out_q.put((ok, [g.tolist() for g in gathered], caught))
    dist.barrier()
    dist.destroy_process_group()


def test_recapture_is_collective_when_one_rank_changes_plan():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    ok, counts, caught = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert ok is True, ok
    # both ranks captured twice (epoch 0, and epoch 1 where only rank 0's plan changed) and
    # issued the same number of all-reduces
    assert counts[0] == counts[1], counts
    assert counts[0][0] == 2, counts
    assert caught


def _shape_worker(rank, world, port, out_q):
    """The real DataParallelEpoch._capture shape selection with the HIP parts faked: rank 0
    cannot capture the prefetch shape (its plan grew past CHAIN3_MAX_ROWS: no pre-gather
    slots), and each rank's timings favour a different shape."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "intrinsic-neural-fields_amd"))
    import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    os.environ.pop("INF_DP_SHAPE", None)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    timed = []

    class Epoch(dp.DataParallelEpoch):
        def _capture_stream(self):
            return None

        def _capture_shape(self, shape, plan, rt, batch, s):
            if shape == "prefetch" and rank == 0:
                return None
            return (shape, shape, None)

        def _time_graphs(self, g, plan, full):
            timed.append(g[0])
            # rank 1 finds prefetch fastest, rank 0 bucketed; the MAX over ranks decides
            return {"serial": 3.0, "prefetch": 1.0 if rank == 1 else 9.0, "bucketed": 2.0 + rank, "sharded": 4.0}[g[0]]

    log = []
    plan, rt = _Plan(log), _Rt()
    res = {}
    for full in (16, 4):
        ep = Epoch()
        timed.clear()
        ep._capture(plan, rt, None, full=full)
        res[full] = (ep.shape, list(timed), ep.shape_times)
    out = [None] * world
    dist.all_gather_object(out, res)
    if rank == 0:
        out_q.put(out)
    dist.barrier()
    dist.destroy_process_group()


def test_capture_shape_choice_is_collective():
    """every rank must time the same step shapes -- the timing replays
    hold captured all-reduces -- and pick the same one.  With fewer full batches than one
    multi-step graph there is nothing to time: serial, without autotune (ADVICE medium)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_shape_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    out = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    r0, r1 = out
    for full in (16, 4):
        assert r0[full][0] == r1[full][0], (full, r0[full], r1[full])
    # 16 full batches: prefetch dropped on both ranks (rank 0 could not capture it); times
    # serial 3 / bucketed max(2, 3) = 3 -> the first of the tie, serial
    assert r0[16][1] == r1[16][1] == ["serial", "bucketed", "sharded"], (r0[16], r1[16])
    assert r0[16][0] == "serial"
    assert set(r0[16][2]) == set(r1[16][2]) == {"serial", "bucketed", "sharded"}
    # 4 full batches (< GRAPH_STEPS = 8): serial, nothing timed
    assert r0[4][0] == "serial" and r0[4][1] == [] and r1[4][1] == []
