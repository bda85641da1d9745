"""PyTorch-CPU restatement of the reference's training step (the CPU baseline's second leg).

TEST INFRASTRUCTURE ONLY: imported by `tests/` and by `bench.py`'s `cpu_baseline` leg,
never by the product path.  Written from scratch with the same torch op sequence the
reference runs on a CPU device, so its timing stands for "the reference's own PyTorch-CPU
path" on the GPU box (where /root/reference does not exist):

  gather   E[vids.reshape(-1)] -> B x 3 x k, torch.bmm with the barycentrics
           (mesh.py:313-324)
  forward  Linear+ReLU layers, the skip layer relu(Lx(h) + Ly(x)), Linear+Sigmoid head
           (model.py:89-112, layers.py:60-62)
  loss     F.mse_loss / F.l1_loss (config.py:113-122)
  step     zero_grad(set_to_none=True), backward, torch.optim.Adam defaults
           (trainer.py:71-84, config.py:108)

Pinned against the reference's one-step goldens (tests/golden/g3_step_*.npz) in
tests/test_oracle_golden.py.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def gather(E: torch.Tensor, vids: torch.Tensor, bary: torch.Tensor) -> torch.Tensor:
    """mesh.py:313-324: B x k features, sum_i bary[b, i] * E[vids[b, i]]."""
    rows = E[vids.reshape(-1)].reshape(vids.shape[0], 3, E.shape[1])
    return torch.bmm(bary[:, None, :], rows).squeeze(1)


class TorchTrainer:
    """Weights dict (reference state-dict names, W[out, in]) -> one Adam step per call."""

    def __init__(self, w: dict, L: int, s: int, lr: float, loss: str = "L2"):
        self.L, self.s, self.loss = L, s, loss
        self.p = {n: torch.tensor(v, dtype=torch.float32).requires_grad_(True) for n, v in w.items()}
        self.opt = torch.optim.Adam(list(self.p.values()), lr=lr)

    def forward(self, x: torch.Tensor) -> torch.Tensor:
        p, L, s = self.p, self.L, self.s
        h = x
        for i in range(L):
            if i == s:
                h = F.relu(F.linear(h, p[f"layers.{i}.Lx.weight"], p[f"layers.{i}.Lx.bias"])
                           + F.linear(x, p[f"layers.{i}.Ly.weight"], p[f"layers.{i}.Ly.bias"]))
            elif i == L - 1:
                h = torch.sigmoid(F.linear(h, p[f"layers.{i}.0.weight"], p[f"layers.{i}.0.bias"]))
            else:
                h = F.relu(F.linear(h, p[f"layers.{i}.0.weight"], p[f"layers.{i}.0.bias"]))
        return h

    def step(self, features: torch.Tensor, rgb: torch.Tensor):
        self.opt.zero_grad(set_to_none=True)
        pred = self.forward(features)
        if self.loss == "L2":
            loss = F.mse_loss(pred, rgb)
        elif self.loss == "L1":
            loss = F.l1_loss(pred, rgb)
        else:
            c2 = (20.0 / 255.0) ** 2
            loss = (c2 * torch.log(1 + (pred - rgb) ** 2 / c2)).mean()
        loss.backward()
        grads = {n: t.grad.detach().clone() for n, t in self.p.items()}
        self.opt.step()
        return float(loss.detach()), pred.detach(), grads
