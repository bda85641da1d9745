"""Host mirror of the reference layers.py (the subset on the hot path).

`LinearWithConcatAndActivation` (reference layers.py:50-62) keeps the reference's
module structure (Lx, Ly, actn, batchnorm) so TextureField's parameter names, order
and seeded initialisation are identical.  Its arithmetic, relu(Lx(h) + Ly(x)), runs
fused inside TextureField's HIP forward as ONE GEMM over the concatenated K = H + k
(csrc/plan.hip run_forward_layer); it has no standalone CPU implementation.

The baseline encoders (FourierFeatEnc, RandomFourierFeatEnc, Sine, MLP; reference
layers.py:6-47,65-125) feed the xyz/ff/rff configurations, which are outside this
build's scope.
"""
import torch.nn as nn


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
        raise RuntimeError("LinearWithConcatAndActivation runs fused inside TextureField's HIP forward "
                           "(one GEMM over [h | x]); it is not callable on its own in this build")
