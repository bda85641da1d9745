"""Data-parallel training on the GPU (dp.py): the Trainer's data-parallel epochs at world
size 1 are bitwise its single-GPU fused epochs, and `train.py --data_parallel` under
torchrun (an RCCL communicator, the collective captured in the step graphs) writes the
same models and scalars as the single-process run; two ranks sharing the one GPU over gloo
run the HIP step at world 2 against the single-process run.  tests/test_dp_gloo.py covers
the sharding arithmetic on the CPU (no multi-GPU box is available to this suite)."""
import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch
import yaml

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "intrinsic-neural-fields_amd")


def _loaders(B, N, drop_last, k=64, V=500, seed=8):
    from ray_dataloader import RayDataLoader
    rng = np.random.default_rng(seed)
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32))
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    rgb = torch.from_numpy(rng.random((N, 3)).astype(np.float32))
    tr = RayDataLoader(E, "efuncs", vids, bary, rgb, None, None, B, True, drop_last, device="cuda")
    va = RayDataLoader(E, "efuncs", vids[:1000], bary[:1000], rgb[:1000], None, None, B, False, False, device="cuda")
    return tr, va


@pytest.mark.parametrize("mode,drop_last,shape", [("bf16", True, "serial"), ("fp32", False, "serial"),
                                                  ("bf16", True, "sharded"), ("bf16", False, "sharded")])
def test_dp_epochs_world1_bitwise_single_gpu(tmp_path, mode, drop_last, shape, monkeypatch):
    """Trainer(dp=DataParallelEpoch()) without a process group (world 1): the reduce ->
    (identity) all-reduce -> Adam step shape, graph-replayed, leaves exactly the
    parameters, Adam state and epoch metrics of the plain fused epochs.  The sharded shape
    (item-major gradient -> Adam on the rank's items -> weight all-gather -> image rewrite,
    masters gathered at the epoch end, before a partial last batch) too."""
    import config
    import dp
    from trainer import Trainer
    monkeypatch.setenv("INF_DP_SHAPE", shape)
    B, N = 1024, 9 * 1024 + (0 if drop_last else 300)
    outs = {}
    for tag in ("single", "dp"):
        cfg = {"data": {"img_height": 8, "img_width": 8},
               "model": {"k": 64, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2,
                         "kernels": {"mode": mode}},
               "training": {"out_dir": str(tmp_path / tag), "batch_size": B, "lr": 1e-3, "loss_type": "L1",
                            "render_every": 100, "print_every": 100, "epochs": 3}}
        torch.manual_seed(0)
        model, optim = config.get_model_and_optim(cfg, None, "cuda")
        model.kernel_mode = mode
        tr_ld, va_ld = _loaders(B, N, drop_last)
        t = Trainer(model, optim, config.get_loss_fn(cfg), None, {"train": tr_ld, "val": va_ld}, None, cfg, "cuda",
                    dp=dp.DataParallelEpoch() if tag == "dp" else None)
        torch.manual_seed(1)  # the loaders' shuffles
        t.train()
        rows = [json.loads(x) for x in open(tmp_path / tag / "logs" / "scalars.jsonl")]
        st = optim.state_dict()["state"]
        outs[tag] = ([(r["tag"], r["value"]) for r in rows],
                     torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy(),
                     torch.cat([st[i]["exp_avg_sq"].reshape(-1).cpu() for i in sorted(st)]).numpy(),
                     float(st[0]["step"]))
    s, d = outs["single"], outs["dp"]
    assert s[3] == d[3] == 3 * (N // B + (0 if drop_last else 1))
    np.testing.assert_array_equal(s[1], d[1])
    np.testing.assert_array_equal(s[2], d[2])
    assert [t for t, _ in s[0]] == [t for t, _ in d[0]]
    np.testing.assert_allclose([v for _, v in s[0]], [v for _, v in d[0]], rtol=1e-12)


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_train_data_parallel_torchrun_world1(tmp_path):
    """`torchrun --nproc-per-node 1 train.py <cfg> --data_parallel` (RCCL process group,
    all-reduce captured in the step graphs) vs `train.py <cfg>`: the same files, the same
    final weights bit for bit, the same logged scalars."""
    import synthetic_views as S
    S.build(str(tmp_path), views=(4, 1, 1))
    cfg = S.intrinsic_config(epochs=3, batch=512)
    cfg["model"]["kernels"] = {"mode": "bf16"}
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    results = {}
    for tag in ("single", "dp"):
        cfg["training"]["out_dir"] = f"out/{tag}"
        path = tmp_path / f"{tag}.yaml"
        with open(path, "w") as fh:
            yaml.safe_dump(cfg, fh)
        if tag == "single":
            cmd = [sys.executable, os.path.join(PKG, "train.py"), str(path)]
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(PKG, "train.py"),
                   str(path), "--data_parallel"]
        r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
        print(tag, r.stdout[-2000:], r.stderr[-2000:])
        assert r.returncode == 0, tag
        out = tmp_path / "out" / tag
        files = sorted(os.listdir(out))
        sd = torch.load(out / "model_last_epoch.pt", map_location="cpu", weights_only=True)
        rows = [json.loads(x) for x in open(out / "logs" / "scalars.jsonl")]
        results[tag] = (files, sd, rows)
    (fs, ws, rs), (fd, wd, rd) = results["single"], results["dp"]
    assert fs == fd and {"model.pt", "model_last_epoch.pt", "checkpoint.pt", "logs"} <= set(fs)
    for k in ws:
        assert torch.equal(ws[k], wd[k]), k
    assert [(r["tag"], r["step"]) for r in rs] == [(r["tag"], r["step"]) for r in rd]
    np.testing.assert_allclose([r["value"] for r in rs], [r["value"] for r in rd], rtol=1e-9)


@pytest.mark.parametrize("mode,w_rel,loss_rtol", [("fp32", 1e-6, 1e-6)])
def test_train_data_parallel_two_ranks_one_gpu_gloo(tmp_path, mode, w_rel, loss_rtol):
    """`torchrun --nproc-per-node 2 train.py <cfg> --data_parallel` with INF_DP_BACKEND=gloo:
    two ranks share the box's one GPU (RCCL refuses that; gloo all-reduces the flat gradient
    eagerly between the fused steps).  The HIP step at world 2 -- rank-sharded batches, the
    loss normalised by the global batch, the all-reduced gradient, replicated Adam --
    against the single-process run of the same config: the same files, the same logged
    scalars up to the summation order of two half-batch gradients, and weights close in
    relative L2 norm.  fp32 (parity mode) holds tight bounds (seen after two epochs: weights
    4e-8 relative, losses 5e-9).  In bf16 a master-weight difference at rounding level can
    flip a bf16 weight image's rounding, so the runs part faster: bf16 is held to a bar
    derived from a summation-order reordering of the single run instead
    (test_train_data_parallel_two_ranks_within_summation_order_spread)."""
    import synthetic_views as S
    S.build(str(tmp_path), views=(4, 1, 1))
    epochs, batch = 2, 512
    cfg = S.intrinsic_config(epochs=epochs, batch=batch)
    cfg["model"]["kernels"] = {"mode": mode}
    # L2: with L1 a rounding-level change of a residual near zero flips its gradient's sign,
    # and the two runs' trajectories part within a few epochs (seen: 2 % in val loss at 3)
    cfg["training"]["loss_type"] = "L2"
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", INF_DP_BACKEND="gloo")
    results = {}
    for tag in ("single", "dp2"):
        cfg["training"]["out_dir"] = f"out/{tag}"
        path = tmp_path / f"{tag}.yaml"
        with open(path, "w") as fh:
            yaml.safe_dump(cfg, fh)
        if tag == "single":
            cmd = [sys.executable, os.path.join(PKG, "train.py"), str(path)]
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(PKG, "train.py"),
                   str(path), "--data_parallel"]
        r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
        print(tag, r.stdout[-2000:], r.stderr[-3000:])
        assert r.returncode == 0, tag
        out = tmp_path / "out" / tag
        files = sorted(os.listdir(out))
        sd = torch.load(out / "model_last_epoch.pt", map_location="cpu", weights_only=True)
        rows = [json.loads(x) for x in open(out / "logs" / "scalars.jsonl")]
        results[tag] = (files, sd, rows)
    (fs, ws, rs), (fd, wd, rd) = results["single"], results["dp2"]
    assert fs == fd and {"model.pt", "model_last_epoch.pt", "checkpoint.pt", "logs"} <= set(fs)
    lr = float(cfg["training"]["lr"])
    for k in ws:
        a, b = ws[k].float().numpy().reshape(-1), wd[k].float().numpy().reshape(-1)
        # Adam moves every element by ~lr per step whatever its gradient's size, so order-
        # level gradient differences leave element-wise drift of that order; a sharding or
        # normalisation error would move whole tensors (and the logged losses, below)
        d = np.abs(a - b)
        rel = float(np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-12))
        print(k, "max", float(d.max()), "rel", rel)
        assert d.max() <= 2 * lr * 200 and rel <= w_rel, (k, float(d.max()), rel)
    assert [(r["tag"], r["step"]) for r in rs] == [(r["tag"], r["step"]) for r in rd]
    np.testing.assert_allclose([r["value"] for r in rs], [r["value"] for r in rd], rtol=loss_rtol)


def _run_train(tmp_path, cfg, tag, env, nproc):
    cfg["training"]["out_dir"] = f"out/{tag}"
    path = tmp_path / f"{tag}.yaml"
    with open(path, "w") as fh:
        yaml.safe_dump(cfg, fh)
    if nproc == 0:
        cmd = [sys.executable, os.path.join(PKG, "train.py"), str(path)]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(PKG, "train.py"),
               str(path), "--data_parallel"]
    r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
    print(tag, r.stdout[-1500:], r.stderr[-2500:])
    assert r.returncode == 0, tag
    out = tmp_path / "out" / tag
    sd = torch.load(out / "model_last_epoch.pt", map_location="cpu", weights_only=True)
    rows = [json.loads(x) for x in open(out / "logs" / "scalars.jsonl")]
    return sd, rows


@pytest.mark.parametrize("mode,loss", [("fp32", "L1"), ("bf16", "L1"), ("bf16", "L2")])
def test_train_data_parallel_two_ranks_within_summation_order_spread(tmp_path, mode, loss):
    """World 2 (two ranks on the one GPU over gloo, as above) with the reference configs' own
    loss (L1, intrinsic_cat.yaml:34) and, in bf16, L2.  Under L1 a rounding-level change of a
    residual near zero flips its gradient's sign, and in bf16 a rounding-level master
    difference flips a bf16 weight image, so two runs that differ ONLY in summation order
    part over the epochs -- the bar is therefore derived, not chosen: a second single-process
    run whose weight-gradient GEMM sums in another order (fp32: INF_DW_SPLITS=2, split-K 2
    instead of one accumulator; bf16: INF_LGEMM_KS=1, one k group per block instead of two)
    measures how far a pure summation-order change moves this run, and the world-2 run
    (whose only difference is the order of two half-batch gradients) must stay within 10x
    that spread, in weights (relative L2) and in every logged scalar.  A sharding /
    normalisation / all-reduce error moves them by O(1)."""
    import synthetic_views as S
    S.build(str(tmp_path), views=(4, 1, 1))
    cfg = S.intrinsic_config(epochs=2, batch=512)
    cfg["model"]["kernels"] = {"mode": mode}
    cfg["training"]["loss_type"] = loss
    base = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", INF_DP_BACKEND="gloo")
    for key in ("INF_DW_SPLITS", "INF_LGEMM_KS"):
        base.pop(key, None)
    knob = {"INF_DW_SPLITS": "2"} if mode == "fp32" else {"INF_LGEMM_KS": "1"}
    single = _run_train(tmp_path, cfg, "single", base, 0)
    reorder = _run_train(tmp_path, cfg, "single_reordered", dict(base, **knob), 0)
    dp2 = _run_train(tmp_path, cfg, "dp2", base, 2)

    def dist(a, b):
        wa = torch.cat([v.float().reshape(-1) for v in a[0].values()])
        wb = torch.cat([v.float().reshape(-1) for v in b[0].values()])
        w_rel = float((wa - wb).norm() / wa.norm())
        assert [(r["tag"], r["step"]) for r in a[1]] == [(r["tag"], r["step"]) for r in b[1]]
        va, vb = np.array([r["value"] for r in a[1]]), np.array([r["value"] for r in b[1]])
        s_rel = float((np.abs(va - vb) / np.maximum(np.abs(va), 1e-12)).max())
        return w_rel, s_rel

    spread = dist(single, reorder)
    got = dist(single, dp2)
    print(mode, "summation-order spread (weights rel, scalars rel):", spread, "world 2:", got)
    assert spread[0] > 0  # the reordered run did sum differently
    assert got[0] <= 10 * spread[0] + 1e-7, (got, spread)
    assert got[1] <= 10 * spread[1] + 1e-7, (got, spread)


@pytest.mark.parametrize("mode", ["bf16", "fp32"])
def test_sharded_two_ranks_gloo_bitwise_allreduce(tmp_path, mode):
    """`torchrun --nproc-per-node 2 train.py <cfg> --data_parallel` over gloo on the one GPU,
    step shape sharded (reduce-scatter of the item-major gradient, Adam on each rank's half
    of the items, all-gather of the new weights, image rewrite; masters and Adam state
    gathered every epoch) against shape serial (all-reduce, replicated Adam): the same
    files, the same weights BIT FOR BIT and the same scalars -- each element's gradient is
    the same two-term sum and its update the same fp32 arithmetic, on one rank instead of
    both."""
    import synthetic_views as S
    S.build(str(tmp_path), views=(4, 1, 1))
    cfg = S.intrinsic_config(epochs=2, batch=1024)  # 512 rays per rank: chain3 / chainf steps
    cfg["model"]["kernels"] = {"mode": mode}
    results = {}
    for shape in ("serial", "sharded"):
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", INF_DP_BACKEND="gloo", INF_DP_SHAPE=shape)
        cfg["training"]["out_dir"] = f"out/{shape}"
        path = tmp_path / f"{shape}.yaml"
        with open(path, "w") as fh:
            yaml.safe_dump(cfg, fh)
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
               "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(PKG, "train.py"),
               str(path), "--data_parallel"]
        r = subprocess.run(cmd, cwd=tmp_path, env=env, capture_output=True, text=True, timeout=240)
        print(shape, r.stdout[-2000:], r.stderr[-3000:])
        assert r.returncode == 0, shape
        assert f"[dp] world 2: step shape {shape}" in r.stdout, shape  # not a fallback
        out = tmp_path / "out" / shape
        sd = torch.load(out / "model_last_epoch.pt", map_location="cpu", weights_only=True)
        rows = [json.loads(x) for x in open(out / "logs" / "scalars.jsonl")]
        results[shape] = (sorted(os.listdir(out)), sd, rows)
    (fs, ws, rs), (fh_, wh, rh) = results["serial"], results["sharded"]
    assert fs == fh_
    for k in ws:
        assert torch.equal(ws[k], wh[k]), k
    # the epoch's losses come from each rank's own steps, the val metrics from the gathered
    # masters: both bit for bit
    assert [(r["tag"], r["step"], r["value"]) for r in rs] == [(r["tag"], r["step"], r["value"]) for r in rh]


def _bucket_rays(k, V, N, seed):
    rng = np.random.default_rng(seed)
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= E.max(0) - E.min(0)
    return (torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
            torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
            torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())


@pytest.mark.parametrize("graph", [False, True])
def test_bucketed_step_bitwise_unbucketed(monkeypatch, graph):
    """The data-parallel step in two gradient buckets (inf_train_step PART1 / PART2: the dW
    GEMM of Ly and the layers after it, their reduction, then the rest; the caller's
    all-reduce of bucket 1 on a side stream between them) leaves exactly the parameters,
    Adam moments and loss sums of the one-bucket step (fused step, all-reduce, Adam) when
    both sum the same number of split-K partials -- eager and graph-captured, config B's
    MLP at 4096 rays."""
    from inf_hip import runtime
    import model as M
    k, H, L, s, B = 1024, 256, 8, 4, 4096
    N = 3 * B
    E, vids, bary, rgb = _bucket_rays(k, 3000, N, seed=4)
    monkeypatch.setenv("INF_DW_SPLITS", "4")
    monkeypatch.setenv("INF_BUCKET_SPLITS", "4")
    out = {}
    for shape in ("serial", "bucketed"):
        torch.manual_seed(0)
        m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s}).cuda()
        rt = m.hip_runtime()
        rt.ensure_optimizer_arenas()
        plan = runtime.Plan(k, H, L, s, "bf16", "L2", B, rt.arena, rt.grads, rt.exp_avg, rt.exp_avg_sq)
        plan.set_lr(1e-3)
        src = runtime.RaySource(E, vids, bary, rgb)
        perm = torch.randperm(N, generator=torch.Generator().manual_seed(2)).cuda()
        b = plan.make_batch(source=src, ray_idx=perm, offset=0, batch=B, offset_from_ctrl=True)
        side = torch.cuda.Stream()
        split = plan.grad_split()
        assert 0 < split < plan.info.num_params

        def step():
            if shape == "serial":
                plan.train_step(b, None, apply_adam=False)
            else:
                plan.train_step(b, None, apply_adam=False, part=1)
                side.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(side):
                    rt.grads[split:].mul_(1.0)  # stands in for the bucket-1 all-reduce
                plan.train_step(b, None, apply_adam=False, part=2)
                torch.cuda.current_stream().wait_stream(side)
            plan.adam(0, 0.0, advance=True)

        plan.set_batch_index(0)
        if graph:
            step()  # settles the plan's tables
            plan.set_batch_index(0)
            st = torch.cuda.Stream()
            st.wait_stream(torch.cuda.current_stream())
            g = torch.cuda.CUDAGraph()
            saved = [x.clone() for x in (plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl)]
            with torch.cuda.stream(st):
                with torch.cuda.graph(g, stream=st):
                    step()
            torch.cuda.current_stream().wait_stream(st)
            for dst, srcv in zip((plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl), saved):
                dst.copy_(srcv)
            plan.sync_shadow()
            plan.set_batch_index(0)
            for _ in range(3):
                g.replay()
        else:
            for _ in range(3):
                step()
        torch.cuda.synchronize()
        assert plan.last_step_path() == "chain3"
        c = plan.read_ctrl()
        out[shape] = [x.detach().cpu().clone() for x in (plan.params, plan.exp_avg, plan.exp_avg_sq)] + \
            [c["epoch_loss"], c["epoch_sse"], c["batch_index"]]
    a, bb = out["serial"], out["bucketed"]
    for x, y in zip(a[:3], bb[:3]):
        assert torch.equal(x, y)
    assert a[3:] == bb[3:] and a[5] == 3


@pytest.mark.parametrize("mode", ["bf16", "fp32"])
def test_config_c_data_parallel_two_ranks_gloo(tmp_path, mode):
    """Config C -- the human k=1024, 8 x 256 (skip 4), L2, lr 1e-4, batch 4096 MLP of
    configs/texture_reconstruction/intrinsic_human_k1024_8x256.yaml -- through
    `torchrun --nproc-per-node 2 train.py <cfg> --data_parallel` (two ranks on the one GPU
    over gloo, 2048 rays per rank per step) against the single-process run of the same
    YAML on a synthetic dataset in the reference's layout (a torus, 1024 eigenfunction
    columns): same files and logged tags.  The world-2 run differs from the single one only
    in the summation order of the two half-batch gradients, so its distance is held to a bar
    DERIVED from a pure summation-order change (as
    test_train_data_parallel_two_ranks_within_summation_order_spread): a second
    single-process run that sums in another order (bf16: INF_LGEMM_KS=1, one k group per dW
    block instead of two; fp32: INF_NO_CHAINF=1, the layered fp32 kernels instead of the
    fused fp32 chain) measures the spread, and world 2
    must stay within 10 x it per weight tensor (relative L2) and over the logged scalars."""
    import synthetic_views as S
    S.build(str(tmp_path), H=128, W=128, kmax=1024, views=(4, 1, 1))
    with open(os.path.join(ROOT, "configs", "texture_reconstruction", "intrinsic_human_k1024_8x256.yaml")) as fh:
        cfg = yaml.safe_load(fh)
    base = S.intrinsic_config(epochs=2, batch=4096, H=128, W=128)
    cfg["data"] = base["data"]  # the synthetic dataset's paths; the MLP / training keys stay C's
    cfg["model"]["kernels"]["mode"] = mode
    cfg["training"].update(epochs=2, render_every=100)
    assert (cfg["model"]["k"], cfg["model"]["num_layers"], cfg["model"]["mlp_hidden_dim"],
            cfg["model"]["skip_layer_idx"], cfg["training"]["batch_size"]) == (1024, 8, 256, 4, 4096)
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", INF_DP_BACKEND="gloo")
    for key in ("INF_NO_CHAINF", "INF_LGEMM_KS"):
        env.pop(key, None)
    # (fp32: the split count does not change this batch's fused fp32 dW order -- INF_DW_SPLITS=8
    # measured a spread of exactly 0 -- so the reordered run takes the layered fp32 kernels)
    knob = {"INF_NO_CHAINF": "1"} if mode == "fp32" else {"INF_LGEMM_KS": "1"}
    results = {}
    for tag in ("single", "reordered", "dp2"):
        cfg["training"]["out_dir"] = f"out/{tag}"
        path = tmp_path / f"{tag}.yaml"
        with open(path, "w") as fh:
            yaml.safe_dump(cfg, fh)
        if tag != "dp2":
            cmd = [sys.executable, os.path.join(PKG, "train.py"), str(path)]
        else:
            cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
                   "--master-addr", "127.0.0.1", "--master-port", str(_port()), os.path.join(PKG, "train.py"),
                   str(path), "--data_parallel"]
        r = subprocess.run(cmd, cwd=tmp_path, env=dict(env, **knob) if tag == "reordered" else env,
                           capture_output=True, text=True, timeout=300)
        print(tag, r.stdout[-2000:], r.stderr[-3000:])
        assert r.returncode == 0, tag
        out = tmp_path / "out" / tag
        sd = torch.load(out / "model_last_epoch.pt", map_location="cpu", weights_only=True)
        rows = [json.loads(x) for x in open(out / "logs" / "scalars.jsonl")]
        results[tag] = (sorted(os.listdir(out)), sd, rows)
    (fs, ws, rs), (fo, wo, ro), (fd, wd, rd) = results["single"], results["reordered"], results["dp2"]
    assert fs == fd == fo
    assert ws["layers.4.Ly.weight"].shape == (256, 1024)
    assert [(r["tag"], r["step"]) for r in rs] == [(r["tag"], r["step"]) for r in rd] == \
        [(r["tag"], r["step"]) for r in ro]

    def rel(a, b):
        a, b = a.float().numpy().reshape(-1), b.float().numpy().reshape(-1)
        return float(np.linalg.norm(a - b) / max(np.linalg.norm(a), 1e-12))

    spread = {key: rel(ws[key], wo[key]) for key in ws}
    got = {key: rel(ws[key], wd[key]) for key in ws}
    print(mode, "weights rel: world 2", {k: f"{v:.2e}" for k, v in got.items()})
    print(mode, "weights rel: summation-order spread", {k: f"{v:.2e}" for k, v in spread.items()})
    assert max(spread.values()) > 0  # the reordered run did sum differently
    bad = [(key, got[key], spread[key]) for key in ws if got[key] > 10 * spread[key] + 1e-7]
    assert not bad, bad
    vs, vo, vd = (np.array([r["value"] for r in x]) for x in (rs, ro, rd))
    s_spread = float((np.abs(vs - vo) / np.maximum(np.abs(vs), 1e-12)).max())
    s_got = float((np.abs(vs - vd) / np.maximum(np.abs(vs), 1e-12)).max())
    print(mode, "scalars rel: world 2", s_got, "spread", s_spread)
    assert s_got <= 10 * s_spread + 1e-7, (s_got, s_spread)
