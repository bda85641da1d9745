"""The sharded optimizer step (include/inf_hip.h "Sharded optimizer step"; dp.py shape
"sharded"): reduce-scatter of the item-major gradient, Adam on 1/world of the update's work
items, all-gather of the new weights in the GEMM dtype, every rank rewriting the weight
images.  It replaces nn.DataParallel's reduce to GPU 0 + GPU-0 Adam + re-broadcast
(reference train.py:46-48, config.py:108, trainer.py:80-82), so it must leave exactly the
bytes of the all-reduce step: each parameter is updated by one rank with the same fp32
arithmetic, and the gradient sums are the same sums.

The collectives are emulated in one process on one GPU (the ranks' plans side by side;
reduce-scatter = sum of the ranks' staging buffers, all-gather = concatenation), so the
multi-rank bookkeeping -- uneven item groups, chunk offsets, every rank's images -- is
checked bit for bit on hardware without a process group."""
import numpy as np
import pytest
import torch

from test_gpu_kernels import CFG, golden, make_plan, rt, weights

pytestmark = pytest.mark.gpu


def _rays(name, N, seed):
    k, H, L, s = CFG[name]
    rng = np.random.default_rng(seed)
    V = 3000
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                         torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                         torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
    return src, torch.from_numpy(rng.permutation(N)).cuda()


def _state(plan):
    torch.cuda.synchronize()
    return [t.detach().cpu().numpy().copy() for t in (plan.params, plan.exp_avg, plan.exp_avg_sq, plan.shadow)]


def _assert_same(a, b, what):
    for x, y, n in zip(a, b, ("params", "exp_avg", "exp_avg_sq", "weight images")):
        assert np.array_equal(x, y), (what, n, int((x != y).sum()))


@pytest.mark.parametrize("name,mode,B,lgf", [("B", "bf16", 4096, "0"), ("R", "bf16", 2048, "0"),
                                             ("B", "fp32", 1024, "0"), ("B", "bf16", 4096, "1")])
def test_sharded_step_world1_bitwise(name, mode, B, lgf, monkeypatch):
    """World 1 (chunks alias the staging, no collective): sharded steps == the all-reduce DP
    step shape (gradient -> Adam + advance) bit for bit: masters and Adam state after the
    epoch-end gather, the weight images, the loss sums and the ctrl block's counters.
    lgf "1": the gradient-only step on the fused dW + update path (INF_LGF=1, config D's
    default), whose leading blocks write the bias items into the staging through their own
    copy of the work items (that copy kept pre-shard offsets)."""
    monkeypatch.setenv("INF_LGF", lgf)
    nb = 3
    src, perm = _rays(name, nb * B, seed=33)
    out = {}
    for shape in ("serial", "sharded"):
        plan, params, _ = make_plan(name, mode=mode, max_batch=B, adam=True)
        plan.set_lr(1e-3)
        b = plan.make_batch(source=src, ray_idx=perm, offset=0, batch=B, offset_from_ctrl=True, loss_count=3 * B)
        if shape == "sharded":
            plan.shard(1, 0)
            assert plan.grad_chunk.data_ptr() == plan.grad_staging.data_ptr()
        for _ in range(nb):
            if shape == "serial":
                plan.train_step(b, None, apply_adam=False)
                plan.adam(0, 0.0, advance=True)
            else:
                plan.train_step(b, None, apply_adam=False, shard=True)
                plan.adam_shard(advance=True)
                plan.shard_scatter()
        if shape == "sharded":
            with pytest.raises(RuntimeError, match="sharded"):
                plan.adam(0, 0.0)  # masters / Adam state are not whole yet
            import dp
            dp.gather_sharded_state(plan)
        c = plan.read_ctrl()
        out[shape] = (_state(plan), c["step"], c["batch_index"], c["epoch_loss"])
    s, h = out["serial"], out["sharded"]
    _assert_same(s[0], h[0], "world 1")
    assert s[1:] == h[1:] and s[2] == nb


@pytest.mark.parametrize("world,name,mode,lgf", [(2, "B", "bf16", "0"), (3, "B", "bf16", "0"), (4, "R", "bf16", "0"),
                                                (2, "A", "fp32", "0"), (2, "B", "bf16", "1"), (3, "B", "bf16", "1")])
def test_sharded_step_emulated_ranks_bitwise(world, name, mode, lgf, monkeypatch):
    """`world` ranks emulated on one GPU: rank r trains on its torch.chunk shard of every
    global batch (loss normalised by the global 3 B).  The all-reduce path (sum of the ranks'
    flat gradients -> replicated Adam) and the sharded path (sum of the item-major staging
    buffers -> rank r's chunk -> Adam on its items -> concatenated weight chunks -> every
    rank's images) leave the same bytes on every rank, after three steps and the
    epoch-end gather.  world 3 / 4: uneven item groups.  lgf "1": the fused dW + update
    path (INF_LGF=1) writing the staging."""
    monkeypatch.setenv("INF_LGF", lgf)
    import dp
    nb, B = 3, 2048
    src, perm = _rays(name, nb * B, seed=44)
    spans = [dp.shard_span(B, r, world) for r in range(world)]
    # global batch i, rank r: rows perm[i B + lo : i B + hi], laid out contiguously per rank
    idx = [perm.view(nb, B)[:, lo:hi].reshape(-1).contiguous() for lo, hi in spans]

    def ranks():
        plans = []
        for r, (lo, hi) in enumerate(spans):
            plan, _, _ = make_plan(name, mode=mode, max_batch=hi - lo, adam=True)
            plan.set_lr(1e-3)
            b = plan.make_batch(source=src, ray_idx=idx[r], offset=0, batch=hi - lo, offset_from_ctrl=True,
                                loss_count=3 * B)
            plans.append((plan, b))
        return plans

    # all-reduce reference
    ref = ranks()
    for _ in range(nb):
        for plan, b in ref:
            plan.train_step(b, None, apply_adam=False)
        total = sum(plan.grads for plan, _ in ref)
        for plan, _ in ref:
            plan.grads.copy_(total)
            plan.adam(0, 0.0, advance=True)
    # sharded
    sh = ranks()
    for r, (plan, _) in enumerate(sh):
        plan.shard(world, r)
    Sg, Sw = sh[0][0].shard_g, sh[0][0].shard_w
    assert all((p.shard_g, p.shard_w) == (Sg, Sw) for p, _ in sh)
    for _ in range(nb):
        for plan, b in sh:
            plan.train_step(b, None, apply_adam=False, shard=True)
        total = sum(plan.grad_staging for plan, _ in sh)  # reduce-scatter
        for r, (plan, _) in enumerate(sh):
            plan.grad_chunk.copy_(total[r * Sg:(r + 1) * Sg])
            plan.adam_shard(advance=True)
        gathered = torch.cat([plan.weight_chunk() for plan, _ in sh])  # all-gather
        for plan, _ in sh:
            plan.weight_staging.copy_(gathered)
            plan.shard_scatter()
    for arena in ("params", "exp_avg", "exp_avg_sq"):  # the epoch-end gather
        for plan, _ in sh:
            plan.shard_pack(getattr(plan, arena))
        chunks = torch.cat([plan.grad_chunk for plan, _ in sh])
        for plan, _ in sh:
            plan.grad_staging.copy_(chunks)
            plan.shard_unpack(getattr(plan, arena))
    want = _state(ref[0][0])
    for r in range(world):
        _assert_same(_state(ref[r][0]), want, f"all-reduce rank {r}")
        _assert_same(_state(sh[r][0]), want, f"sharded rank {r}")
        assert sh[r][0].read_ctrl()["batch_index"] == nb


def test_sharded_layout_covers_every_parameter_once():
    """The item-major layout: pack of an arena whose element i holds i, gathered over the
    ranks' chunks, unpacks to the same arena -- every parameter has exactly one slot."""
    for world in (1, 2, 3, 8):
        plans = []
        for r in range(world):
            plan, params, _ = make_plan("B", mode="bf16", max_batch=256, adam=True)
            plan.shard(world, r)
            plans.append(plan)
        P = plans[0].params.numel()
        src = torch.arange(P, dtype=torch.float32, device="cuda")
        for plan in plans:
            plan.shard_pack(src)
        chunks = torch.cat([plan.grad_chunk for plan in plans]) if world > 1 else plans[0].grad_chunk.clone()
        dst = torch.full((P,), -1.0, device="cuda")
        plans[0].grad_staging.copy_(chunks)
        plans[0].shard_unpack(dst)
        assert torch.equal(dst, src), world
        # each chunk is at most 1/world of the gradient plus one item of padding
        assert plans[0].shard_g * world <= P + world * 2048 + 64 * world * 8, (world, plans[0].shard_g)
