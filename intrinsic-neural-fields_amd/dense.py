"""Autograd over the generic fp32 dense-layer kernels (csrc/dense.hip) for the layers the
fused plan does not cover: the view-dependent texture field (reference model.py:115-191)
-- a TextureField ending in a ReLU bottleneck, plus the two-layer directional MLP.

`linear(segments, bias, act)` computes act(sum_s x_s @ W_s[:, c_s:c_s + K_s]^T + sum bias)
in one output buffer: a plain nn.Linear (one segment), LinearWithConcatAndActivation
(layers.py:60-62: two weights, two biases) or a Linear over a concatenated input
(model.py:186-191: one weight split by column ranges) without materialising the concat.
Every product, activation, gradient and bias sum runs in libinf_hip.so; torch only
allocates.
"""
from __future__ import annotations

import torch

ACT = {None: 0, "relu": 1, "sigmoid": 2}


def _rt():
    from inf_hip import runtime  # raises if the HIP library is missing: no fallback
    return runtime


def _gemm(M, N, K, A, sam, sak, B, sbn, sbk, bias, act, beta, C, ldc):
    rt = _rt()
    from inf_hip import lib
    rt.check(lib.inf_dense_gemm(M, N, K, rt.ptr(A), sam, sak, rt.ptr(B), sbn, sbk, rt.ptr(bias), act, float(beta),
                                rt.ptr(C), ldc, rt.stream_handle()), "dense_gemm")


class _Linear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec, act, *tensors):
        # spec: per segment (weight index, column offset); tensors: xs..., weights..., biases...
        nseg = len(spec)
        nw = max(w for w, _ in spec) + 1
        xs, ws, bs = tensors[:nseg], tensors[nseg:nseg + nw], tensors[nseg + nw:]
        B = xs[0].shape[0]
        N = ws[0].shape[0]
        y = torch.empty((B, N), dtype=torch.float32, device=xs[0].device)
        for s, (wi, c0) in enumerate(spec):
            x, W = xs[s], ws[wi]
            _gemm(B, N, x.shape[1], x, x.stride(0), x.stride(1), W[:, c0:], W.stride(0), W.stride(1),
                  bs[s] if s < len(bs) else None, act if s == nseg - 1 else 0, 0.0 if s == 0 else 1.0, y, N)
        ctx.spec, ctx.act, ctx.nw, ctx.nb = spec, act, nw, len(bs)
        ctx.save_for_backward(*xs, *ws, y)
        return y

    @staticmethod
    def backward(ctx, dy):
        rt = _rt()
        from inf_hip import lib
        spec, act, nw, nb = ctx.spec, ctx.act, ctx.nw, ctx.nb
        saved = ctx.saved_tensors
        nseg = len(spec)
        xs, ws, y = saved[:nseg], saved[nseg:nseg + nw], saved[-1]
        dy = dy.contiguous().to(torch.float32)
        B, N = y.shape
        if act:
            dz = torch.empty_like(y)
            rt.check(lib.inf_dense_act_bwd(y.numel(), rt.ptr(y), rt.ptr(dy), act, rt.ptr(dz), rt.stream_handle()),
                     "dense_act_bwd")
        else:
            dz = dy
        needs = ctx.needs_input_grad[2:]
        dxs = [None] * nseg
        dws = [None] * nw
        for s, (wi, c0) in enumerate(spec):
            x, W = xs[s], ws[wi]
            K = x.shape[1]
            if needs[s]:
                dx = torch.empty((B, K), dtype=torch.float32, device=y.device)
                # dx[b][k] = sum_n dz[b][n] W[n][c0 + k]
                _gemm(B, K, N, dz, N, 1, W[:, c0:], W.stride(1), W.stride(0), None, 0, 0.0, dx, K)
                dxs[s] = dx
            if needs[nseg + wi]:
                if dws[wi] is None:
                    dws[wi] = torch.empty(W.shape, dtype=torch.float32, device=y.device)
                g = dws[wi]
                # dW[n][c0 + k] = sum_b dz[b][n] x[b][k]
                _gemm(N, K, B, dz, 1, N, x, x.stride(1), x.stride(0), None, 0, 0.0, g[:, c0:], g.stride(0))
        dbs = []
        for i in range(nb):
            if needs[nseg + nw + i]:
                db = torch.empty(N, dtype=torch.float32, device=y.device)
                rt.check(lib.inf_colsum(B, N, rt.ptr(dz), N, rt.ptr(db), 0, rt.stream_handle()), "colsum")
                dbs.append(db)
            else:
                dbs.append(None)
        return (None, None, *dxs, *dws, *dbs)


def linear(segments, weights, biases, act=None):
    """segments: [(x_s, weight index, column offset)]; weights / biases: lists of tensors."""
    for t in [x for x, _, _ in segments] + list(weights) + list(biases):
        if not t.is_cuda:
            raise RuntimeError("the dense layers run on the HIP device only; there is no CPU fallback")
    spec = tuple((wi, c0) for _, wi, c0 in segments)
    xs = [x.to(torch.float32) for x, _, _ in segments]
    return _Linear.apply(spec, ACT[act], *xs, *weights, *biases)


def view_angles(unit_dirs, face_idxs, face_normals):
    """model.py:164-169: acos(cos_sim(-dirs, normals[face])), [B]."""
    rt = _rt()
    from inf_hip import lib
    d = unit_dirs.to(torch.float32).contiguous()
    f = face_idxs.to(torch.int64).contiguous()
    nrm = face_normals.to(torch.float32).contiguous()
    out = torch.empty(d.shape[0], dtype=torch.float32, device=d.device)
    rt.check(lib.inf_view_angle(d.shape[0], rt.ptr(d), rt.ptr(f), rt.ptr(nrm), nrm.shape[0], rt.ptr(out),
                                rt.stream_handle()), "view_angle")
    return out


def ff_encode(x, bands, include_input):
    """FourierFeatEnc.forward (layers.py:21-25) for inputs of any width d: [.., 2dk (+d)]."""
    rt = _rt()
    from inf_hip import lib
    lead, d = x.shape[:-1], x.shape[-1]
    xf = x.reshape(-1, d).to(torch.float32).contiguous()
    k = bands.shape[0]
    w = 2 * d * k + (d if include_input else 0)
    out = torch.empty((xf.shape[0], w), dtype=torch.float32, device=xf.device)
    b = bands.to(torch.float32).contiguous()
    rt.check(lib.inf_ff_encode(xf.shape[0], d, rt.ptr(xf), rt.ptr(b), k, int(include_input), rt.ptr(out), w,
                               rt.stream_handle()), "ff_encode")
    return out.view(*lead, w)


def adam_step(p, grad, exp_avg, exp_avg_sq, step, lr, beta1, beta2, eps):
    rt = _rt()
    from inf_hip import lib
    for t in (p, grad, exp_avg, exp_avg_sq):
        if not (t.is_cuda and t.is_contiguous() and t.dtype == torch.float32):
            raise RuntimeError("HIP Adam needs contiguous fp32 device tensors")
    rt.check(lib.inf_adam_dense(p.numel(), rt.ptr(p), rt.ptr(grad), rt.ptr(exp_avg), rt.ptr(exp_avg_sq), int(step),
                                float(lr), float(beta1), float(beta2), float(eps), rt.stream_handle()), "adam_dense")
