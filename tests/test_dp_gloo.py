"""World-size-2 data parallelism on CPU (gloo): the sharding, global-mean loss
normalisation and flat-gradient all-reduce of dp.py reproduce the full-batch gradient
(nn.DataParallel semantics, reference train.py:46-48).  The per-shard gradients come
from the CPU oracle (the checker); the code under test is dp.shard_span,
dp.epoch_permutation and dp.allreduce_grads, exactly as the HIP path calls them."""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from oracle import inf_oracle as O

L, S = 4, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _flat(g):
    return np.concatenate([g[n].reshape(-1) for n in O.layer_names(L, S)])


def _worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "intrinsic-neural-fields_amd"))
    sys.path.insert(0, os.path.join(here, ".."))
    import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from conftest import golden
    d = golden("g2_forward_A.npz")
    w = {k[2:]: d[k] for k in d.files if k.startswith("w:")}
    rng = np.random.default_rng(3)
    N, B = 64, 20
    X = rng.standard_normal((N, 64)).astype(np.float32) * 0.3
    Y = rng.random((N, 3)).astype(np.float32)
    perm = dp.epoch_permutation(N, seed=0, epoch=1, device="cpu").numpy()
    perm_all = [torch.zeros(N, dtype=torch.int64) for _ in range(world)]
    dist.all_gather(perm_all, torch.from_numpy(perm))
    same_perm = all(torch.equal(perm_all[0], p) for p in perm_all)
    results = []
    for i in range((N + B - 1) // B):
        b0 = i * B
        gb = min(B, N - b0)
        lo, hi = dp.shard_span(gb, rank, world)
        rows = perm[b0 + lo:b0 + hi]
        if hi > lo:
            pred, cache = O.mlp_forward(w, X[rows], L, S)
            g = O.mlp_backward(w, cache, O.loss_grad(pred, Y[rows], "L2", n_total=3 * gb), L, S)
            flat = torch.from_numpy(_flat(g).astype(np.float64))
        else:
            flat = torch.zeros(sum(w[n].size for n in O.layer_names(L, S)), dtype=torch.float64)
        dp.allreduce_grads(flat)
        results.append(flat.numpy())
    if rank == 0:
        full = []
        for i in range((N + B - 1) // B):
            rows = perm[i * B:min((i + 1) * B, N)]
            pred, cache = O.mlp_forward(w, X[rows], L, S)
            full.append(_flat(O.mlp_backward(w, cache, O.loss_grad(pred, Y[rows], "L2"), L, S)))
        out_q.put((same_perm, max(float(np.abs(a - b).max() / max(np.abs(b).max(), 1e-12))
                                  for a, b in zip(results, full))))
    dist.barrier()
    dist.destroy_process_group()


def test_dp_gloo_world2_matches_full_batch():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    same_perm, err = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert same_perm
    assert err < 1e-5, err


class _FakeRenderer:
    """Stands in for renderer.Renderer on CPU: the shading of pixel p is a fixed function
    of p, background white outside the mask (what render_device returns for a mask)."""

    def __init__(self, H, W):
        self.H, self.W = H, W
        self.calls = []

    def render_device(self, camCv2world, K, obj_mask_1d=None):
        m = torch.ones(self.H * self.W, dtype=torch.bool) if obj_mask_1d is None else obj_mask_1d.reshape(-1)
        self.calls.append(int(m.sum()))
        p = torch.arange(self.H * self.W, dtype=torch.float32)
        img = torch.ones((self.H * self.W, 3))
        shade = torch.stack([torch.sin(p), torch.cos(p), p / (self.H * self.W)], -1)
        img[m] = shade[m]
        return img.reshape(self.H, self.W, 3)


def _render_worker(rank, world, port, out_q):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(here, "..", "intrinsic-neural-fields_amd"))
    import dp
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    H, W = 37, 11  # rows not divisible by the world size
    r = _FakeRenderer(H, W)
    mask = torch.from_numpy(np.random.default_rng(0).random(H * W) < 0.7)
    img = dp.render_distributed(r, None, None, obj_mask_1d=mask)
    full = _FakeRenderer(H, W).render_device(None, None, mask)
    out_q.put((rank, bool(torch.equal(img, full)), r.calls[0], int(mask.sum())))
    dist.barrier()
    dist.destroy_process_group()


def test_render_distributed_gloo_world3():
    """dp.render_distributed: each rank shades only its row shard (no data-path exchange),
    one all_gather assembles the frame, identical to a single-rank render."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    world = 3
    procs = [ctx.Process(target=_render_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(ok for _, ok, _, _ in res)
    assert sum(c for _, _, c, _ in res) == res[0][3]  # the shards partition the masked pixels
