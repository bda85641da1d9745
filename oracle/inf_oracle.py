"""CPU oracle for the intrinsic-neural-fields hot path.

TEST INFRASTRUCTURE ONLY.  This module is the *checker*: only `tests/`,
`__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import it.  The
product path (intrinsic-neural-fields_amd/) never imports it and fails loudly when
the HIP library is missing.

It is a from-scratch numpy restatement of the reference algorithm, one function per
step of the path, each citing the reference file:line it follows
(reference = tum-vision/intrinsic-neural-fields, mounted read-only at /root/reference
in the build container; it is never read at run time).

Parity pinning: every function below is checked against golden vectors produced by
running the reference itself (tests/golden/make_golden.py -> tests/golden/*.npz) in
tests/test_oracle_golden.py.

Arithmetic is done in the dtype of the inputs (fp32 by default, pass fp64 arrays for
an accuracy reference).  Weight layout follows torch.nn.Linear: W[out, in].
"""
from __future__ import annotations

import numpy as np

# ------------------------------------------------------------------------------------
# Table producer and gather
# ------------------------------------------------------------------------------------


def load_first_k_eigenfunctions(table: np.ndarray, k, rescale_strategy: str = "standard") -> np.ndarray:
    """mesh.py:53-108 (column select :60-65, rescale :99-106; embed strategies not used by
    any config on the path).  `table` is the stored V x kmax eigenfunction matrix."""
    if isinstance(k, (list, tuple, np.ndarray)):
        E = table[:, np.asarray(k)]
    else:
        assert k <= table.shape[1]
        E = table[:, :k]
    if rescale_strategy == "standard":
        E = E / (E.max(axis=0, keepdims=True) - E.min(axis=0, keepdims=True))
    elif rescale_strategy == "one-norm":
        E = E / np.linalg.norm(E, ord=2, axis=-1, keepdims=True)
    elif rescale_strategy != "unscaled":
        raise RuntimeError(f"Unknown rescaling strategy: {rescale_strategy}")
    return np.ascontiguousarray(E, dtype=np.float32)


def gather(E: np.ndarray, vids: np.ndarray, bary: np.ndarray) -> np.ndarray:
    """mesh.py:313-324 get_k_eigenfunc_vec_vals: F[b,:] = sum_i bary[b,i] * E[vids[b,i],:]
    (index -> B x 3 x k, then a (B,1,3)x(B,3,k) batched product)."""
    rows = E[vids.reshape(-1)].reshape(vids.shape[0], 3, E.shape[1])
    acc = bary[:, 0:1] * rows[:, 0]
    acc = acc + bary[:, 1:2] * rows[:, 1]
    acc = acc + bary[:, 2:3] * rows[:, 2]
    return acc.astype(E.dtype, copy=False)


def interp_xyz(verts: np.ndarray, vids: np.ndarray, bary: np.ndarray) -> np.ndarray:
    """ray_dataloader.py:134-136 (ff/rff/xyz strategies): the hit position
    bmm(bary[B,1,3], verts[vids] [B,3,3]) -- the same barycentric sum as `gather` over the
    V x 3 vertex table."""
    return gather(verts, vids, bary)


def rff_encode(x: np.ndarray, B: np.ndarray, include_input: bool = True) -> np.ndarray:
    """layers.py:28-39 RandomFourierFeatEnc.forward: e = (2 pi x) @ B (B is 3 x k, drawn as
    randn(3, k) * std at construction), features [cos e | sin e | x]."""
    e = (2 * np.pi * x.astype(np.float64)) @ B.astype(np.float64)
    parts = [np.cos(e), np.sin(e)] + ([x.astype(np.float64)] if include_input else [])
    return np.concatenate(parts, -1).astype(x.dtype)


def ff_bands(k: int, use_logspace: bool = False, max_freq=None) -> np.ndarray:
    """layers.py:11-18 FourierFeatEnc frequency bands (fp32, as the reference's buffer)."""
    if use_logspace:
        return (2.0 ** np.arange(0, k) * np.float32(np.pi)).astype(np.float32)
    assert max_freq is not None
    return (2.0 ** np.linspace(0, max_freq, k + 1, dtype=np.float32)[:-1] * np.float32(np.pi)).astype(np.float32)


def ff_encode(x: np.ndarray, bands: np.ndarray, include_input: bool = True) -> np.ndarray:
    """layers.py:21-25 FourierFeatEnc.forward: e[b, c*k + f] = x[b, c] * bands[f], features
    [cos e | sin e | x]."""
    e = (x.astype(np.float64)[..., None] * bands.astype(np.float64)).reshape(x.shape[0], -1)
    parts = [np.cos(e), np.sin(e)] + ([x.astype(np.float64)] if include_input else [])
    return np.concatenate(parts, -1).astype(x.dtype)


# ------------------------------------------------------------------------------------
# MLP (TextureField) forward / backward
# ------------------------------------------------------------------------------------


def layer_names(num_layers: int, skip: int):
    """Parameter names in model.parameters() order (model.py:43-96, layers.py:50-57)."""
    names = []
    for i in range(num_layers):
        if i == skip:
            names += [f"layers.{i}.Lx.weight", f"layers.{i}.Lx.bias",
                      f"layers.{i}.Ly.weight", f"layers.{i}.Ly.bias"]
        else:
            names += [f"layers.{i}.0.weight", f"layers.{i}.0.bias"]
    return names


def _sigmoid(z):
    return 1.0 / (1.0 + np.exp(-z))


def mlp_forward(w: dict, x: np.ndarray, num_layers: int, skip: int):
    """model.py:98-112 TextureField.forward with layers.py:60-62 at the skip layer.
    Returns (pred[B,3], cache) where cache holds each layer's input, pre-activation and output."""
    cache = {"x": x, "in": [], "z": [], "out": []}
    h = x
    for i in range(num_layers):
        cache["in"].append(h)
        if i == skip:
            z = (h @ w[f"layers.{i}.Lx.weight"].T + w[f"layers.{i}.Lx.bias"]) + \
                (x @ w[f"layers.{i}.Ly.weight"].T + w[f"layers.{i}.Ly.bias"])
            h = np.maximum(z, 0)
        elif i == num_layers - 1:
            z = h @ w[f"layers.{i}.0.weight"].T + w[f"layers.{i}.0.bias"]
            h = _sigmoid(z)
        else:
            z = h @ w[f"layers.{i}.0.weight"].T + w[f"layers.{i}.0.bias"]
            h = np.maximum(z, 0)
        cache["z"].append(z)
        cache["out"].append(h)
    return h.astype(x.dtype, copy=False), cache


CAUCHY_C2 = (20 / 255) * (20 / 255)


def loss_value(pred: np.ndarray, tgt: np.ndarray, loss_type: str) -> float:
    """config.py:113-122 (mean reduction over B*3)."""
    d = pred - tgt
    if loss_type == "L2":
        return float(np.mean(d * d))
    if loss_type == "L1":
        return float(np.mean(np.abs(d)))
    if loss_type == "cauchy":
        return float(np.mean(CAUCHY_C2 * np.log(1 + d * d / CAUCHY_C2)))
    raise RuntimeError(f"Unknown loss function: {loss_type}")


def loss_grad(pred: np.ndarray, tgt: np.ndarray, loss_type: str, n_total: int | None = None) -> np.ndarray:
    """d loss / d pred for the mean losses of config.py:113-122; n_total = number of
    elements of the (global) mean, default pred.size.  sign(0) = 0 as torch's l1 grad."""
    n = pred.size if n_total is None else n_total
    d = pred - tgt
    if loss_type == "L2":
        g = 2.0 * d
    elif loss_type == "L1":
        g = np.sign(d)
    elif loss_type == "cauchy":
        g = 2.0 * d / (1 + d * d / CAUCHY_C2)
    else:
        raise RuntimeError(loss_type)
    return (g / n).astype(pred.dtype, copy=False)


def mlp_backward(w: dict, cache: dict, dpred: np.ndarray, num_layers: int, skip: int) -> dict:
    """Reverse-mode of mlp_forward (what autograd computes at trainer.py:81)."""
    g = {}
    out = cache["out"]
    # sigmoid head
    dz = dpred * out[-1] * (1 - out[-1])
    for i in range(num_layers - 1, -1, -1):
        hin = cache["in"][i]
        if i == skip:
            g[f"layers.{i}.Lx.weight"] = dz.T @ hin
            g[f"layers.{i}.Lx.bias"] = dz.sum(0)
            g[f"layers.{i}.Ly.weight"] = dz.T @ cache["x"]
            g[f"layers.{i}.Ly.bias"] = dz.sum(0)
            wmat = w[f"layers.{i}.Lx.weight"]
        else:
            g[f"layers.{i}.0.weight"] = dz.T @ hin
            g[f"layers.{i}.0.bias"] = dz.sum(0)
            wmat = w[f"layers.{i}.0.weight"]
        if i == 0:
            break
        dh = dz @ wmat
        dz = dh * (out[i - 1] > 0)
    return g


def bf16_round(x) -> np.ndarray:
    """fp32 -> bf16 -> fp32, round to nearest even (the device's bf16 conversions)."""
    u = np.ascontiguousarray(x, dtype=np.float32).view(np.uint32)
    r = ((u >> np.uint32(16)) & np.uint32(1)) + np.uint32(0x7FFF)
    return ((u + r) & np.uint32(0xFFFF0000)).view(np.float32)


def gather_bf16(E: np.ndarray, vids: np.ndarray, bary: np.ndarray) -> np.ndarray:
    """The bf16 mode's feature rows: bf16 table values, fp32 b0 e0 + b1 e1 + b2 e2 in the
    gather's order, one bf16 rounding (chain3.hip gather_cols, gather.hip)."""
    e = bf16_round(E)
    b = bary.astype(np.float32)
    x = b[:, 0:1] * e[vids[:, 0]]
    x = x + b[:, 1:2] * e[vids[:, 1]]
    x = x + b[:, 2:3] * e[vids[:, 2]]
    return bf16_round(x)


def mlp_forward_bf16(w: dict, x_bf: np.ndarray, num_layers: int, skip: int, mm=np.matmul, colsum=None):
    """The bf16 perf mode's arithmetic (chain3.hip epilogues): bf16 weights of the hidden
    / input layers, fp32 accumulation, bias added last, ReLU output rounded to bf16 once;
    the sigmoid head on the bf16 activations with fp32 weights.  x_bf: gather_bf16 rows.
    mm: the fp32 matrix product (another summation order of the same arithmetic for the
    derived test bars, tests/golden/make_bf16_spread.py); colsum: unused here."""
    wb = {n: bf16_round(v) for n, v in w.items() if n.endswith("weight")}
    cache = {"x": x_bf, "in": [], "out": []}
    h = x_bf
    for i in range(num_layers - 1):
        cache["in"].append(h)
        if i == skip:
            z = (mm(h, wb[f"layers.{i}.Lx.weight"].T) + mm(x_bf, wb[f"layers.{i}.Ly.weight"].T)) + \
                w[f"layers.{i}.Lx.bias"] + w[f"layers.{i}.Ly.bias"]
        else:
            z = mm(h, wb[f"layers.{i}.0.weight"].T) + w[f"layers.{i}.0.bias"]
        h = bf16_round(np.maximum(z.astype(np.float32), 0))
        cache["out"].append(h)
    i = num_layers - 1
    cache["in"].append(h)
    z = mm(h, w[f"layers.{i}.0.weight"].T) + w[f"layers.{i}.0.bias"]
    p = _sigmoid(z.astype(np.float32)).astype(np.float32)
    cache["out"].append(p)
    cache["wb"] = wb
    return p, cache


def mlp_forward_bf16_projected(w: dict, E: np.ndarray, vids: np.ndarray, bary: np.ndarray, num_layers: int,
                               skip: int) -> np.ndarray:
    """The render slice over a projected table (csrc/rproj.hip, inf_project_table) in its
    arithmetic: P = bf16(bf16(E) W_0^T), Q = bf16(bf16(E) W_y^T) per vertex (fp32
    accumulation), each hit's pre-activations interpolated in fp32 (b0 r0 + b1 r1 + b2 r2)
    and rounded to bf16 once more, then the hidden layers and the head as in
    mlp_forward_bf16.  The same function as model.py:98-112, reassociated."""
    e = bf16_round(E)
    wb = {n: bf16_round(v) for n, v in w.items() if n.endswith("weight")}
    b = bary.astype(np.float32)

    def interp(T):
        x = b[:, 0:1] * T[vids[:, 0]]
        x = x + b[:, 1:2] * T[vids[:, 1]]
        x = x + b[:, 2:3] * T[vids[:, 2]]
        return bf16_round(x)

    z0 = interp(bf16_round(e @ wb["layers.0.0.weight"].T))
    zy = interp(bf16_round(e @ wb[f"layers.{skip}.Ly.weight"].T))
    h = bf16_round(np.maximum(z0 + w["layers.0.0.bias"], 0))
    for i in range(1, num_layers - 1):
        if i == skip:
            z = h @ wb[f"layers.{i}.Lx.weight"].T + zy + w[f"layers.{i}.Lx.bias"] + w[f"layers.{i}.Ly.bias"]
        else:
            z = h @ wb[f"layers.{i}.0.weight"].T + w[f"layers.{i}.0.bias"]
        h = bf16_round(np.maximum(z.astype(np.float32), 0))
    i = num_layers - 1
    z = h @ w[f"layers.{i}.0.weight"].T + w[f"layers.{i}.0.bias"]
    return _sigmoid(z.astype(np.float32)).astype(np.float32)


def mlp_backward_bf16(w: dict, cache: dict, dpred: np.ndarray, num_layers: int, skip: int, mm=np.matmul,
                      colsum=None) -> dict:
    """Reverse mode in the bf16 perf mode's arithmetic: dZ of every hidden layer rounded to
    bf16 once (the MFMA operand of the dX chain and of the dW GEMM), bias gradients from the
    fp32 dZ before rounding, the head and its backward in fp32 (chain3.hip, lgemm.hip).
    mm / colsum: the fp32 matrix product and column sum (another summation order: see
    mlp_forward_bf16)."""
    if colsum is None:
        colsum = lambda a: a.sum(0)  # noqa: E731
    g = {}
    wb = cache["wb"]
    out, L = cache["out"], num_layers
    p = out[-1]
    dz = (dpred * (1 - p) * p).astype(np.float32)
    h = cache["in"][L - 1]
    g[f"layers.{L - 1}.0.weight"] = mm(dz.T, h)
    g[f"layers.{L - 1}.0.bias"] = colsum(dz)
    v = mm(dz, w[f"layers.{L - 1}.0.weight"]) * (h > 0)
    for i in range(L - 2, -1, -1):
        hin = cache["in"][i]
        v = v.astype(np.float32)
        dzb = bf16_round(v)
        if i == skip:
            g[f"layers.{i}.Lx.weight"] = mm(dzb.T, hin)
            g[f"layers.{i}.Lx.bias"] = colsum(v)
            g[f"layers.{i}.Ly.weight"] = mm(dzb.T, cache["x"])
            g[f"layers.{i}.Ly.bias"] = colsum(v)
            wmat = wb[f"layers.{i}.Lx.weight"]
        else:
            g[f"layers.{i}.0.weight"] = mm(dzb.T, hin)
            g[f"layers.{i}.0.bias"] = colsum(v)
            wmat = wb[f"layers.{i}.0.weight"]
        if i == 0:
            break
        v = mm(dzb, wmat) * (cache["out"][i - 1] > 0)
    return g


# ------------------------------------------------------------------------------------
# Adam (torch.optim.Adam defaults, non-capturable single-tensor formula; config.py:108)
# ------------------------------------------------------------------------------------


def adam_step(p, g, m, v, step: int, lr: float, beta1=0.9, beta2=0.999, eps=1e-8):
    """One Adam update in place; `step` is the post-increment step count.
    m <- lerp(m, g, 1-b1); v <- b2*v + (1-b2)*g*g;
    p <- p - lr/(1-b1^t) * m / (sqrt(v)/sqrt(1-b2^t) + eps).
    torch.optim.Adam's single-tensor CPU kernels op by op (adam.py: lerp_, mul_ + addcmul_,
    sqrt / bc2_sqrt + eps, addcdiv_), whose roundings tools/adam_bits.py pins: lerp_ and
    addcmul_ are fused multiply-adds, addcdiv_ is p + (value * m) / denom.  fp32 arrays take
    the fma as one rounding of the float64 product + sum (exact product, then one rounding)."""
    dt = p.dtype

    def fma(a, b, c):
        if dt == np.float32:
            return (np.float64(a) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)
        return a * b + c

    m[...] = fma(dt.type(1 - beta1), g - m, m)
    vb = v * dt.type(beta2)
    v[...] = fma(dt.type(1 - beta2) * g, g, vb)
    bc1 = 1 - beta1 ** step
    bc2_sqrt = (1 - beta2 ** step) ** 0.5
    step_size = lr / bc1
    denom = np.sqrt(v) / dt.type(bc2_sqrt) + dt.type(eps)
    p += (dt.type(-step_size) * m) / denom


class OracleTrainer:
    """Minimal restatement of Trainer._train_step (trainer.py:71-84) over the oracle
    functions: forward -> loss -> backward -> Adam, with torch-Adam state semantics."""

    def __init__(self, weights: dict, num_layers: int, skip: int, lr: float, loss_type: str):
        self.w = {k: np.array(v, copy=True) for k, v in weights.items()}
        self.L, self.s, self.lr, self.loss_type = num_layers, skip, lr, loss_type
        self.names = layer_names(num_layers, skip)
        self.m = {n: np.zeros_like(self.w[n]) for n in self.names}
        self.v = {n: np.zeros_like(self.w[n]) for n in self.names}
        self.t = 0

    def step(self, x, rgb):
        pred, cache = mlp_forward(self.w, x, self.L, self.s)
        loss = loss_value(pred, rgb, self.loss_type)
        grads = mlp_backward(self.w, cache, loss_grad(pred, rgb, self.loss_type), self.L, self.s)
        self.t += 1
        for n in self.names:
            adam_step(self.w[n], grads[n], self.m[n], self.v[n], self.t, self.lr)
        return loss, pred, grads


# ------------------------------------------------------------------------------------
# Loader batching, metrics, render scatter
# ------------------------------------------------------------------------------------


def loader_batches(N: int, B: int, drop_last: bool, perm: np.ndarray | None = None):
    """ray_dataloader.py:88-113: number of batches and the row indices of each batch."""
    nb = N // B if drop_last else (N + B - 1) // B
    idxs = np.arange(N) if perm is None else np.asarray(perm)
    return [idxs[i * B:min((i + 1) * B, N)] for i in range(nb)]


def psnr(fake, real, obj_mask_1d=None):
    """evaluation_metrics.py:5-22."""
    if obj_mask_1d is not None:
        fake = fake.reshape(-1, 3)[obj_mask_1d]
        real = real.reshape(-1, 3)[obj_mask_1d]
    mse = np.mean((fake - real) ** 2)
    if mse == 0:
        return float("inf")
    return 20 * np.log10(1.0 / np.sqrt(mse))


def structural_similarity(a: np.ndarray, b: np.ndarray, data_range: float = 2.0, win_size: int = 7) -> float:
    """evaluation_metrics.py:33 calls skimage.metrics.structural_similarity(fake, real,
    multichannel=True) with the defaults: per channel, uniform win_size^2 window
    (scipy.ndimage.uniform_filter), K1 = 0.01, K2 = 0.03, sample covariance
    NP / (NP - 1), data_range = the dtype range of the input (2 for float images), S
    averaged over the image cropped by (win_size - 1) // 2; channels averaged.
    scikit-image is not installed here: PARITY UNPINNED beyond known-answer checks."""
    from scipy.ndimage import uniform_filter
    a = np.asarray(a, dtype=np.float64)
    b = np.asarray(b, dtype=np.float64)
    assert a.shape == b.shape and a.ndim == 3
    NP = win_size ** 2
    cov_norm = NP / (NP - 1)
    C1, C2 = (0.01 * data_range) ** 2, (0.03 * data_range) ** 2
    pad = (win_size - 1) // 2
    out = []
    for c in range(a.shape[2]):
        x, y = a[..., c], b[..., c]
        ux, uy = uniform_filter(x, win_size), uniform_filter(y, win_size)
        uxx, uyy, uxy = uniform_filter(x * x, win_size), uniform_filter(y * y, win_size), uniform_filter(x * y, win_size)
        vx, vy, vxy = cov_norm * (uxx - ux * ux), cov_norm * (uyy - uy * uy), cov_norm * (uxy - ux * uy)
        S = ((2 * ux * uy + C1) * (2 * vxy + C2)) / ((ux ** 2 + uy ** 2 + C1) * (vx + vy + C2))
        out.append(S[pad:S.shape[0] - pad, pad:S.shape[1] - pad].mean())
    return float(np.mean(out))


def dssim(fake, real, data_range: float = 2.0) -> float:
    """evaluation_metrics.py:29-34: (1 - SSIM) / 2."""
    return (1 - structural_similarity(fake, real, data_range)) / 2


def epoch_psnr(epoch_mse):
    """evaluation_metrics.py:25-26 (callers divide summed sq. error by rays, trainer.py:263)."""
    return -10 * np.log10(epoch_mse)


def render_scatter(pred, hit_ray_idxs, H, W, obj_mask_1d=None, background="white"):
    """renderer.py:121-146: place predicted colours at hit rays over a constant background,
    then unmask to H*W if an object mask was used."""
    fill = 1.0 if background == "white" else 0.0
    n = H * W if obj_mask_1d is None else int(np.sum(obj_mask_1d))
    img = np.full((n, 3), fill, np.float32)
    img[hit_ray_idxs] = pred
    if obj_mask_1d is not None:
        full = np.full((H * W, 3), fill, np.float32)
        full[np.asarray(obj_mask_1d, bool)] = img
        img = full
    return img.reshape(H, W, 3)
