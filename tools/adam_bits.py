"""Which fp32 formulation of Adam's element update reproduces torch's CPU optimizer bit for
bit (torch.optim.Adam, single-tensor path, as the reference steps it at trainer.py:82)?
Emulates the candidate roundings in numpy (fma: float64 product + sum, one rounding) and
counts exact matches on 2^20 random elements; csrc/adam_dev.hpp adam_elem follows the winner."""
import numpy as np
import torch


def main():
    torch.manual_seed(0)
    n = 1 << 20
    p, g = torch.randn(n) * 0.1, torch.randn(n) * 1e-3
    m, v = torch.randn(n) * 1e-3, torch.rand(n) * 1e-6
    par = torch.nn.Parameter(p.clone())
    opt = torch.optim.Adam([par], lr=1e-3)
    par.grad = g.clone()
    st = opt.state[par]
    st["step"], st["exp_avg"], st["exp_avg_sq"] = torch.tensor(5.0), m.clone(), v.clone()
    opt.step()
    tm, tv, tp = st["exp_avg"].numpy(), st["exp_avg_sq"].numpy(), par.detach().numpy()
    f = np.float32

    def fma(a, b, c):
        return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(f)

    G, M, V, P = g.numpy(), m.numpy(), v.numpy(), p.numpy()
    b1, b2, lr, eps, t = 0.9, 0.999, 1e-3, 1e-8, 6
    print("m fma(1-b1, g-m, m):", (fma(f(1 - b1), G - M, M) == tm).mean(), " m + (1-b1)(g-m):", (M + f(1 - b1) * (G - M) == tm).mean())
    vb = V * f(b2)
    print("v fma((1-b2)g, g, v b2):", (fma(f(1 - b2) * G, G, vb) == tv).mean(), " v b2 + ((1-b2)g)g:", (vb + (f(1 - b2) * G) * G == tv).mean())
    step, bc2s = lr / (1 - b1 ** t), (1 - b2 ** t) ** 0.5
    den = np.sqrt(tv) / f(bc2s) + f(eps)
    print("p + (-step m)/den:", (P + (f(-step) * tm) / den == tp).mean(), " p + -step (m/den):", (P + f(-step) * (tm / den) == tp).mean())
    print("torch sqrt == IEEE sqrt:", (torch.from_numpy(tv).sqrt().numpy() == np.sqrt(tv)).mean())


if __name__ == "__main__":
    main()
