"""Host mirror of the reference layers.py (the subset on the hot path).

`LinearWithConcatAndActivation` (reference layers.py:50-62) keeps the reference's
module structure (Lx, Ly, actn, batchnorm) so TextureField's parameter names, order
and seeded initialisation are identical.  Inside TextureField its arithmetic,
relu(Lx(h) + Ly(x)), runs fused in the plan's kernels (one accumulator over the two K
segments, csrc/chain3.hip / plan.hip run_forward_layer); called on its own it runs as one
HIP dense-layer launch over both segments (csrc/dense.hip via dense.linear, with
autograd).

The position encoders FourierFeatEnc / RandomFourierFeatEnc (reference layers.py:6-39)
keep the reference's constructor, buffers (`freq_bands` non-persistent, `B` persistent,
drawn from the global torch RNG at construction) and output layout [cos | sin | x].
Their forward is the HIP `inf_encode` kernel (csrc/gather.hip); inside TextureField the
same kernel writes the encoding straight into the MLP's input tiles.  Sine and the
NeuTex MLP (layers.py:42-47,65-125) are outside this build's scope.
"""
import math

import torch
import torch.nn as nn


def _encode(kind, module, x):
    from inf_hip import runtime  # raises if the HIP library is missing: no fallback
    proj = module.B if kind == "rff" else module.freq_bands
    enc = runtime.Encoding(kind, proj.shape[-1], proj.to(torch.float32).contiguous(), module.include_input)
    lead = x.shape[:-1]
    out = runtime.encode(enc, x.reshape(-1, 3).to(torch.float32).contiguous())
    return out.view(*lead, enc.dim)


class FourierFeatEnc(nn.Module):
    """Reference layers.py:6-25: e[..., c*k + f] = x[..., c] * band_f with bands pi*2^i
    (use_logspace, i = 0..k-1) or pi*2^linspace(0, max_freq, k+1)[:-1]."""

    def __init__(self, k, include_input=True, use_logspace=False, max_freq=None):
        super().__init__()
        if use_logspace:
            exps = torch.arange(0, k)
        else:
            assert max_freq is not None
            exps = torch.linspace(0, max_freq, steps=k + 1)[:-1]
        self.register_buffer("freq_bands", torch.pow(2, exps) * math.pi, persistent=False)
        self.include_input = include_input

    def forward(self, x):
        if x.shape[-1] == 3:
            return _encode("ff", self, x)
        import dense  # view directions as angles (model.py:168): any input width
        if not x.is_cuda:
            raise RuntimeError("the encoders run on the HIP device only; there is no CPU fallback")
        return dense.ff_encode(x, self.freq_bands, self.include_input)


class RandomFourierFeatEnc(nn.Module):
    """Reference layers.py:28-39: e = (2 pi x) @ B with B ~ N(0, std^2) of shape [in_dim, k]."""

    def __init__(self, k, std=1., in_dim=3, dtype=torch.float32, include_input=True):
        super().__init__()
        if in_dim != 3:
            raise NotImplementedError("the encoders take 3-D positions (ray_dataloader.py:134-136)")
        self.register_buffer("B", torch.randn((in_dim, k), dtype=dtype) * std, persistent=True)
        self.include_input = include_input

    def forward(self, x):
        return _encode("rff", self, x)


class LinearWithConcatAndActivation(nn.Module):
    """relu(Lx(x) + Ly(y)) -- reference layers.py:50-62."""

    def __init__(self, x_in_dim, y_in_dim, out_dim, batchnorm=False, activation=nn.ReLU):
        super().__init__()
        self.Lx = nn.Linear(x_in_dim, out_dim)
        self.Ly = nn.Linear(y_in_dim, out_dim)
        self.actn = activation()
        self.batchnorm = None
        if batchnorm:
            self.batchnorm = nn.BatchNorm1d(out_dim)

    def forward(self, x, y):
        """actn(Lx(x) + Ly(y)) (layers.py:60-62): both products into one output with the
        ReLU in the epilogue.  BatchNorm (unused by every config) is not implemented."""
        import dense
        if self.batchnorm is not None:
            raise NotImplementedError("batchnorm=True is not used by any intrinsic config and is not implemented")
        if not isinstance(self.actn, nn.ReLU):
            raise NotImplementedError("only the ReLU activation is implemented")
        lead = x.shape[:-1]
        out = dense.linear([(x.reshape(-1, x.shape[-1]), 0, 0), (y.reshape(-1, y.shape[-1]), 1, 0)],
                           [self.Lx.weight, self.Ly.weight], [self.Lx.bias, self.Ly.bias], "relu")
        return out.view(*lead, out.shape[-1])
