"""The next batch's gather on a side stream (inf_prefetch_batch + runtime.StepPipeline):
fused steps that read pre-gathered feature rows leave bitwise the state of the plain fused
steps -- parameters, Adam moments, loss sums, step and batch counters -- eager and
graph-captured, at config B (whole feature tile) and at k = 4096 (chunked tile)."""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _setup(k, V, B, nb, seed):
    import model as M
    from inf_hip import runtime
    rng = np.random.default_rng(seed)
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": 8, "mlp_hidden_dim": 256, "skip_layer_idx": 4})
    params = torch.cat([p.detach().reshape(-1) for p in m.parameters()]).cuda()
    g = torch.Generator(device="cuda").manual_seed(seed)
    E = torch.randn((V, k), generator=g, device="cuda")
    N = nb * B
    src = runtime.RaySource(E, torch.from_numpy(rng.integers(0, V, (N, 3))).cuda(),
                            torch.from_numpy(rng.dirichlet([1, 1, 1], N).astype(np.float32)).cuda(),
                            torch.from_numpy(rng.random((N, 3)).astype(np.float32)).cuda())
    perm = torch.from_numpy(rng.permutation(N)).cuda()
    return params, src, perm


def _plan(k, B, params):
    from inf_hip import runtime
    p = params.clone()
    plan = runtime.Plan(k, 256, 8, 4, "bf16", "L2", B, p, grads=torch.zeros_like(p), exp_avg=torch.zeros_like(p),
                        exp_avg_sq=torch.zeros_like(p))
    plan.set_lr(1e-3)
    return plan


@pytest.mark.parametrize("k,V,graph", [(1024, 20000, False), (1024, 20000, True), (4096, 30000, False)])
def test_prefetched_steps_bitwise(k, V, graph, monkeypatch):
    # the chunked chain's schedule on both sides (k = 4096 would otherwise take zg.hip's
    # gather + input GEMM, which the pre-gathered feature rows replace)
    monkeypatch.setenv("INF_ZG", "0")
    from inf_hip import runtime
    B, nb = 4096, 4
    params, src, perm = _setup(k, V, B, nb, seed=k + 1)
    out = {}
    for tag in ("plain", "prefetch"):
        plan = _plan(k, B, params)
        b = plan.make_batch(source=src, ray_idx=perm, offset=0, batch=B, offset_from_ctrl=True, loss_count=3 * B)
        plan.set_batch_index(0)
        if tag == "plain":
            for _ in range(nb):
                plan.train_step(b, None, apply_adam=True, advance=True)
        else:
            pipe = runtime.StepPipeline(plan, b)
            assert pipe.start()
            step = lambda xs: plan.train_step(b, None, apply_adam=True, advance=True, xslot=xs)  # noqa: E731
            if graph:
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                gr = torch.cuda.CUDAGraph()
                saved = [x.clone() for x in (plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl)]
                with torch.cuda.stream(s):
                    with torch.cuda.graph(gr, stream=s):
                        pipe.run(2, step)
                torch.cuda.current_stream().wait_stream(s)
                for dst, src_ in zip((plan.params, plan.exp_avg, plan.exp_avg_sq, plan.ctrl), saved):
                    dst.copy_(src_)
                plan.set_batch_index(0)
                assert pipe.start()
                for _ in range(nb // 2):
                    gr.replay()
            else:
                pipe.run(nb, step)
            assert plan.last_step_path() in ("chain3", "chain3_chunked")
        torch.cuda.synchronize()
        c = plan.read_ctrl()
        out[tag] = (plan.params.cpu().numpy(), plan.exp_avg.cpu().numpy(), plan.exp_avg_sq.cpu().numpy(),
                    c["step"], c["batch_index"], c["epoch_loss"], c["epoch_sse"])
    p, q = out["plain"], out["prefetch"]
    for a, b_ in zip(p[:3], q[:3]):
        np.testing.assert_array_equal(a, b_)
    assert p[3:] == q[3:]
