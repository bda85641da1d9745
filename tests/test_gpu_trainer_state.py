"""GPU tests of device state that outlives one call: the fused epoch's captured graph
across a plan replacement, and a host-driven Adam step with lr = 0."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

CFG = {"data": {"img_height": 8, "img_width": 8},
       "model": {"k": 64, "num_layers": 4, "mlp_hidden_dim": 128, "skip_layer_idx": 2},
       "training": {"out_dir": "/tmp/unused", "batch_size": 512, "lr": 1e-3, "loss_type": "L2",
                    "render_every": 100, "print_every": 100, "epochs": 1}}


def _data(seed=5, V=400, N=2048, k=64):
    rng = np.random.default_rng(seed)
    E = torch.from_numpy(rng.standard_normal((V, k)).astype(np.float32))
    vids = torch.from_numpy(rng.integers(0, V, (N, 3)))
    bary = torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32))
    rgb = torch.from_numpy(rng.random((N, 3)).astype(np.float32))
    return E, vids, bary, rgb


def test_graph_epoch_survives_plan_replacement(monkeypatch):
    """Fused (graph-replayed) epoch -> the plan is replaced by a larger one (what
    Renderer.render_hits' 2^18-ray chunks or a kernel-mode change do) -> another fused
    epoch: the second epoch must run on the new plan (re-captured graph) and leave the same
    parameters, Adam state and epoch loss as eager epochs (INF_GRAPH=0)."""
    import config
    from ray_dataloader import RayDataLoader
    from trainer import Trainer
    E, vids, bary, rgb = _data()
    B = CFG["training"]["batch_size"]
    outs = {}
    for tag in ("graph", "eager"):
        monkeypatch.setenv("INF_GRAPH", "1" if tag == "graph" else "0")
        torch.manual_seed(0)
        model, optim = config.get_model_and_optim(CFG, None, "cuda")
        model.kernel_mode = "fp32"
        ld = RayDataLoader(E, "efuncs", vids, bary, rgb, None, None, B, False, True, device="cuda")
        tr = Trainer(model, optim, config.get_loss_fn(CFG), None, {"train": ld, "val": ld}, None, CFG, "cuda")
        first = tr._train_epoch()
        old = model._rt.plan
        model.hip_plan(1 << 16)  # regrow: the old plan's workspace goes back to the allocator
        assert model._rt.plan is not old
        del old
        # churn the caching allocator so the freed blocks get new contents
        junk = [torch.full((1 << 20,), 7.0, device="cuda") for _ in range(8)]
        second = tr._train_epoch()
        del junk
        torch.cuda.synchronize()
        st = optim.state_dict()["state"]
        outs[tag] = (first, second, torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy(),
                     torch.cat([st[i]["exp_avg"].reshape(-1).cpu() for i in sorted(st)]).numpy(),
                     float(st[0]["step"]))
    g, e = outs["graph"], outs["eager"]
    assert g[4] == e[4] == 2 * (2048 // B)
    np.testing.assert_allclose(g[0], e[0], rtol=1e-6)
    np.testing.assert_allclose(g[1], e[1], rtol=1e-6)
    np.testing.assert_allclose(g[2], e[2], atol=1e-6)
    np.testing.assert_allclose(g[3], e[3], atol=1e-7)


def test_host_adam_step_with_zero_lr():
    """A host-driven step (optim.step() after loss.backward()) with lr = 0 leaves the
    parameters unchanged and still advances Adam's moments, as torch.optim.Adam does."""
    import config
    E, vids, bary, rgb = _data(seed=9, N=256)
    cfg = {**CFG, "training": {**CFG["training"], "lr": 0.0}}
    torch.manual_seed(0)
    model, optim = config.get_model_and_optim(cfg, None, "cuda")
    model.kernel_mode = "fp32"
    import mesh
    feats = mesh.get_k_eigenfunc_vec_vals(E.cuda(), vids.cuda(), bary.cuda())
    optim.param_groups[0]["lr"] = 1e-3
    loss_fn = config.get_loss_fn(cfg)
    pred = model({"eigenfunctions": feats})
    loss_fn(pred, rgb.cuda()).backward()
    optim.step()
    optim.zero_grad(set_to_none=True)
    model.hip_plan(1).set_lr(1e-3)  # a stale non-zero lr in the device ctrl block (as fused steps leave)
    optim.param_groups[0]["lr"] = 0.0
    before = [p.detach().clone() for p in model.parameters()]
    m_before = [optim.state[p]["exp_avg"].clone() for p in model.parameters()]
    pred = model({"eigenfunctions": feats})
    loss_fn(pred, rgb.cuda()).backward()
    grads = [p.grad.detach().clone() for p in model.parameters()]
    optim.step()
    for p, b, g, mb in zip(model.parameters(), before, grads, m_before):
        assert torch.equal(p.detach(), b)
        torch.testing.assert_close(optim.state[p]["exp_avg"], 0.9 * mb + 0.1 * g, rtol=1e-5, atol=1e-9)


def test_one_shuffle_per_epoch(monkeypatch):
    """The fused epoch draws exactly one permutation per epoch, as the reference's
    `for batch in self.train_data_loader` (trainer.py:248, ray_dataloader.py:103-106):
    eager (INF_GRAPH=0) and graph-replayed epochs use the same batches and leave the same
    global RNG state."""
    import config
    from ray_dataloader import RayDataLoader
    from trainer import Trainer
    E, vids, bary, rgb = _data()
    B = CFG["training"]["batch_size"]
    outs = {}
    for graph in ("1", "0"):
        monkeypatch.setenv("INF_GRAPH", graph)
        torch.manual_seed(0)
        model, optim = config.get_model_and_optim(CFG, None, "cuda")
        model.kernel_mode = "fp32"
        ld = RayDataLoader(E, "efuncs", vids, bary, rgb, None, None, B, True, True, device="cuda")
        tr = Trainer(model, optim, config.get_loss_fn(CFG), None, {"train": ld, "val": ld}, None, CFG, "cuda")
        torch.manual_seed(1)
        calls = []
        orig = RayDataLoader.__iter__
        monkeypatch.setattr(RayDataLoader, "__iter__", lambda self: calls.append(1) or orig(self))
        losses = [tr._train_epoch()[0] for _ in range(3)]
        monkeypatch.setattr(RayDataLoader, "__iter__", orig)
        assert len(calls) == 3
        outs[graph] = (losses, torch.cat([p.detach().reshape(-1) for p in model.parameters()]).cpu().numpy(),
                       torch.cuda.get_rng_state().clone())
    np.testing.assert_allclose(outs["1"][0], outs["0"][0], rtol=1e-6)
    np.testing.assert_allclose(outs["1"][1], outs["0"][1], atol=1e-6)
    assert torch.equal(outs["1"][2], outs["0"][2])
