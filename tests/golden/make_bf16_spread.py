"""Summation-order spread of the bf16 mode's arithmetic at config D's shape (k = 4096,
8 x 256, skip 4, 4096 rays): the bf16 restatement (oracle.inf_oracle.mlp_forward_bf16 /
mlp_backward_bf16) re-run with its fp32 sums in other orders -- every contraction split in
2 or 4 parts, accumulated in 32-deep blocks left to right (an MFMA k-block chain), reversed,
or in float64 -- on the exact inputs of tests/test_gpu_kernels.py
test_bf16_chunked_chain3_matches_bf16_oracle (seed-0 reference init, rng 78).  The bf16
roundings sit at the same points in every variant, so how far the variants land from the
restatement is how far ANY correct implementation of this arithmetic can land from it: the
GPU tests' bars at config D are derived from this spread (tests/golden/bf16_spread_D.npz),
not chosen; likewise for test_chain3_zg_input_layers' k = 4096 cases (two device orders of
the same arithmetic against each other: the spread between two variants).  Test infrastructure (CPU only):

    python tests/golden/make_bf16_spread.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "intrinsic-neural-fields_amd"))
sys.path.insert(0, ROOT)

from oracle import inf_oracle as O  # noqa: E402


def _split(parts):
    def mm(a, b):
        K = a.shape[1]
        if K < 2 * parts or K % parts:
            return a @ b
        c = K // parts
        out = a[:, :c] @ b[:c]
        for i in range(1, parts):
            out = out + a[:, i * c:(i + 1) * c] @ b[i * c:(i + 1) * c]
        return out

    def cs(v):
        n = v.shape[0]
        if n < 2 * parts or n % parts:
            return v.sum(0)
        c = n // parts
        out = v[:c].sum(0)
        for i in range(1, parts):
            out = out + v[i * c:(i + 1) * c].sum(0)
        return out
    return mm, cs


def _blocks32():
    def mm(a, b):
        K = a.shape[1]
        if K % 32:
            return a @ b
        out = a[:, :32] @ b[:32]
        for k0 in range(32, K, 32):
            out = out + a[:, k0:k0 + 32] @ b[k0:k0 + 32]
        return out

    def cs(v):
        n = v.shape[0]
        if n % 16:
            return v.sum(0)
        out = v[:16].sum(0)
        for r in range(16, n, 16):  # one partial per 16-ray chain tile, added in order
            out = out + v[r:r + 16].sum(0)
        return out
    return mm, cs


def _reversed():
    return (lambda a, b: np.ascontiguousarray(a[:, ::-1]) @ np.ascontiguousarray(b[::-1]),
            lambda v: v[::-1].sum(0))


def _f64():
    return (lambda a, b: (a.astype(np.float64) @ b.astype(np.float64)).astype(np.float32),
            lambda v: v.astype(np.float64).sum(0).astype(np.float32))


VARIANTS = {"split2": _split(2), "split4": _split(4), "blocks32": _blocks32(), "reversed": _reversed(),
            "f64": _f64()}


def config_d_inputs():
    """The inputs of test_bf16_chunked_chain3_matches_bf16_oracle (same seeds, same order)."""
    import torch
    import model as M
    rng = np.random.default_rng(78)
    k, H, L, s, B, V = 4096, 256, 8, 4, 4096, 20000
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s})
    w = {n: p.detach().cpu().numpy() for n, p in m.named_parameters()}
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    vids = rng.integers(0, V, (B, 3))
    bary = rng.dirichlet([1, 1, 1], B).astype(np.float32)
    rgb = rng.random((B, 3)).astype(np.float32)
    return w, E, vids, bary, rgb, (L, s)


def zg_inputs(B, V, bad):
    """The inputs of test_chain3_zg_input_layers at k = 4096 (rng 9; the test's ray order is
    a torch.randperm, here the identity -- the statistics of the sums do not depend on which
    rays come first).  bad: every 97th ray's second vertex out of range (a zero table row)
    and every 131st ray index out of range (a zero feature row and a zero target)."""
    import torch
    import model as M
    rng = np.random.default_rng(9)
    k, H, L, s = 4096, 256, 8, 4
    E = rng.standard_normal((V, k)).astype(np.float32)
    E /= (E.max(0) - E.min(0))
    vids = rng.integers(0, V, (B, 3))
    bary = rng.dirichlet([1, 1, 1], B).astype(np.float32)
    rgb = rng.random((B, 3)).astype(np.float32)
    torch.manual_seed(0)
    m = M.make_model({"k": k, "num_layers": L, "mlp_hidden_dim": H, "skip_layer_idx": s})
    w = {n: p.detach().numpy().copy() for n, p in m.named_parameters()}
    dead = np.zeros(B, bool)
    if bad:
        vids[::97, 1] = V + 5
        dead[::131] = True
    return w, E, vids, bary, rgb, dead, (L, s)


def features(E, vids, bary, dead=None):
    """gather_bf16 with the kernels' bounds: an out-of-range vertex reads a zero row, an
    out-of-range ray index a zero feature row."""
    V = E.shape[0]
    Ez = np.concatenate([E, np.zeros((1, E.shape[1]), np.float32)])
    x = O.gather_bf16(Ez, np.where(vids < V, vids, V), bary)
    if dead is not None:
        x[dead] = 0
    return x


def spread(w, x, rgb, L, s):
    """Per tensor (and RGB): the largest distance of a variant from the restatement
    ('vs_ref:') and between two variants ('pair:'), relative to the tensor's max."""
    names = O.layer_names(L, s)
    runs = {}
    for tag, (mm, cs) in [("ref", (np.matmul, None))] + list(VARIANTS.items()):
        p, c = O.mlp_forward_bf16(w, x, L, s, mm=mm)
        runs[tag] = (p, O.mlp_backward_bf16(w, c, O.loss_grad(p, rgb, "L2"), L, s, mm=mm, colsum=cs))
    p_ref, g_ref = runs["ref"]
    out = {}
    tags = list(VARIANTS)
    for n in ["rgb"] + names:
        def d(a, b):
            if n == "rgb":
                return float(np.abs(runs[a][0] - runs[b][0]).max())
            return float(np.abs(runs[a][1][n] - runs[b][1][n]).max() / max(np.abs(g_ref[n]).max(), 1e-12))
        out[f"vs_ref:{n}"] = np.float64(max(d(t, "ref") for t in tags))
        out[f"pair:{n}"] = np.float64(max(d(a, b) for i, a in enumerate(tags) for b in tags[i + 1:]))
    print({kk: round(float(v), 5) for kk, v in out.items()}, flush=True)
    return out


if __name__ == "__main__":
    here = os.path.dirname(os.path.abspath(__file__))
    w, E, vids, bary, rgb, (L, s) = config_d_inputs()
    res = {f"D/{kk}": v for kk, v in spread(w, features(E, vids, bary), rgb, L, s).items()}
    for B, V, bad in ((4096, 20000, False), (1024, 5000, True)):
        w, E, vids, bary, rgb, dead, (L, s) = zg_inputs(B, V, bad)
        rgb = np.where(dead[:, None], 0.0, rgb).astype(np.float32)
        res.update({f"zg_{B}/{kk}": v for kk, v in spread(w, features(E, vids, bary, dead), rgb, L, s).items()})
    np.savez(os.path.join(here, "bf16_spread_D.npz"), **res)
