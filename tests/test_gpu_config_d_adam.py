"""Config D's default training step WITH Adam applied.

At k > 1024 the bf16 step fuses the update into the weight-gradient GEMM (lgemm.hip GT,
"LGF": split-K 1, each 64 x 64 block runs Adam on its own dW tile straight from LDS; the
biases and head in the launch's leading blocks).  Its gradient is pinned against the bf16
oracle elsewhere (test_gpu_kernels.py::test_bf16_chunked_chain3_matches_bf16_oracle, a
gradient-only LGF step).  Here the update itself, at config D's own shape (k = 4096,
8 x 256, skip 4, seed-0 reference init, 4096 rays; the chain after zg.hip's gather + input
GEMM, config D's default), over three steps:

* test_config_d_lgf_adam_is_torch_adam_on_its_gradient -- each step's gradient is read
  from a gradient-only replay of the SAME step (same launch, same LDS tile, same sums: the
  bytes the fused Adam consumed), then the oracle's torch Adam (oracle.inf_oracle.adam_step,
  torch 2.10's single-tensor CPU kernel op by op, tools/adam_bits.py) is applied on the host
  and compared with what the fused launch wrote: exp_avg / exp_avg_sq / weights to 1 ulp
  (they are expected bitwise; the ulp allows a libm-vs-device sqrt / pow difference);
* test_config_d_lgf_matches_slab_path -- the fused dW + update against the split-K slabs and
  the separate update launch (INF_LGF=0) on one step: the same chain bit for bit, gradients
  to fp32 summation order, weights with the assert_adam_close bar (a rounding-level
  gradient can take Adam's +-lr step the other way).
"""
import numpy as np
import pytest
import torch

from oracle import inf_oracle as O

pytestmark = pytest.mark.gpu

K, H, L, S = 4096, 256, 8, 4


def rt():
    from inf_hip import runtime
    return runtime


def seed0_weights():
    import model as M
    torch.manual_seed(0)
    m = M.make_model({"k": K, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": S})
    return {n: p.detach().numpy().copy() for n, p in m.named_parameters()}


def to_dict(arena, w):
    a = arena.detach().cpu().numpy()
    out, off = {}, 0
    for n in O.layer_names(L, S):
        out[n] = a[off:off + w[n].size].reshape(w[n].shape).copy()
        off += w[n].size
    return out


def source(B, nb, V=20000, seed=91):
    rng = np.random.default_rng(seed)
    E = rng.standard_normal((V, K)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    N = B * nb
    src = rt().RaySource(torch.from_numpy(E).cuda(), torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                         torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                         torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
    perm = torch.from_numpy(rng.permutation(N)).cuda()
    return src, perm


def make_plan(w, B):
    params = torch.cat([torch.from_numpy(w[n]).reshape(-1) for n in O.layer_names(L, S)]).cuda()
    plan = rt().Plan(K, H, L, S, "bf16", "L2", B, params, grads=torch.zeros_like(params),
                     exp_avg=torch.zeros_like(params), exp_avg_sq=torch.zeros_like(params))
    return plan, params


def max_ulp(a, b):
    """Largest distance in units in the last place between two fp32 arrays."""
    ia = a.astype(np.float32).view(np.int32).astype(np.int64)
    ib = b.astype(np.float32).view(np.int32).astype(np.int64)
    ia = np.where(ia < 0, np.int64(-(2 ** 31)) - ia, ia)  # monotone integer order of floats
    ib = np.where(ib < 0, np.int64(-(2 ** 31)) - ib, ib)
    return int(np.abs(ia - ib).max())


def test_config_d_lgf_adam_is_torch_adam_on_its_gradient(monkeypatch):
    monkeypatch.delenv("INF_LGF", raising=False)
    B, nb, lr = 4096, 3, 1e-4
    w = seed0_weights()
    src, perm = source(B, nb)
    plan, params = make_plan(w, B)
    plan.set_lr(lr)
    names = O.layer_names(L, S)
    W = {n: w[n].astype(np.float32).copy() for n in names}
    M = {n: np.zeros_like(W[n]) for n in names}
    Vv = {n: np.zeros_like(W[n]) for n in names}
    worst = {}
    for t in range(1, nb + 1):
        b = plan.make_batch(source=src, ray_idx=perm, offset=(t - 1) * B, batch=B)
        ctrl0 = plan.ctrl.clone()
        # the gradient this step's fused update will consume: a gradient-only replay of the
        # same launch (LGF writes the reduced gradient from the same LDS tile)
        plan.train_step(b, None, apply_adam=False)
        assert plan.last_step_path() == "chain3_zg" and plan.last_step_fused_update() == 1
        g = to_dict(plan.grads, w)
        plan.ctrl.copy_(ctrl0)  # the replay counted a step and added to the epoch sums
        plan.train_step(b, None, apply_adam=True)
        assert plan.last_step_fused_update() == 1
        assert plan.read_ctrl()["step"] == t
        got_w, got_m, got_v = to_dict(params, w), to_dict(plan.exp_avg, w), to_dict(plan.exp_avg_sq, w)
        for n in names:
            O.adam_step(W[n], g[n], M[n], Vv[n], t, lr)
            worst[n] = (max_ulp(got_m[n], M[n]), max_ulp(got_v[n], Vv[n]), max_ulp(got_w[n], W[n]))
            assert worst[n][0] <= 1 and worst[n][1] <= 1, (t, n, worst[n])
            assert worst[n][2] <= 1, (t, n, worst[n], float(np.abs(got_w[n] - W[n]).max()))
            # next step from the device's own state (what the fused launch wrote)
            W[n], M[n], Vv[n] = got_w[n], got_m[n], got_v[n]
        print("step", t, "max ulp (m, v, w):", {n: worst[n] for n in names})


@pytest.mark.parametrize("apply_adam", [True, False])
def test_config_d_lgf_matches_slab_path(apply_adam, monkeypatch):
    B = 4096
    w = seed0_weights()
    src, perm = source(B, 1, seed=92)
    out = {}
    for tag in ("lgf", "slab"):
        monkeypatch.setenv("INF_LGF", "1" if tag == "lgf" else "0")
        plan, params = make_plan(w, B)
        plan.set_lr(1e-4)
        plan.train_step(plan.make_batch(source=src, ray_idx=perm, offset=0, batch=B), None, apply_adam=apply_adam)
        assert plan.last_step_path() == "chain3_zg"
        assert plan.last_step_fused_update() == (tag == "lgf")
        c = plan.read_ctrl()
        torch.cuda.synchronize()
        out[tag] = (to_dict(params, w), to_dict(plan.grads, w), (c["loss_sum"], c["sse_sum"]))
        del plan
        torch.cuda.empty_cache()
    assert out["lgf"][2] == out["slab"][2]  # the same chain: identical loss sums
    from test_gpu_kernels import assert_adam_close
    for n in O.layer_names(L, S):
        if apply_adam:
            assert_adam_close(out["lgf"][0][n], out["slab"][0][n], lr=1e-4, steps=1, name=n, atol=1e-7, frac=1e-3)
        else:
            ref = out["slab"][1][n]
            err = float(np.abs(out["lgf"][1][n] - ref).max() / max(np.abs(ref).max(), 1e-12))
            assert err < 1e-5, (n, err)
