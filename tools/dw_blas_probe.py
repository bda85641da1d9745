"""Probe: what a library GEMM takes for the step's weight gradients if the fused chain
wrote row-major [ray][feature] activations instead of fragment images -- dW_0 / dW_y as one
512 x 1024 x 4096 GEMM (shared X) and the six hidden dW as a batched 256 x 256 x 4096 GEMM
(torch.matmul -> hipBLASLt / rocBLAS), bf16 in, bf16 and fp32 out."""
import torch

B, k, H = 4096, 1024, 256
dev = "cuda"
X = torch.randn(B, k, device=dev, dtype=torch.bfloat16)
dZin = torch.randn(B, 2 * H, device=dev, dtype=torch.bfloat16)
Y = torch.randn(6, B, H, device=dev, dtype=torch.bfloat16)
dZ = torch.randn(6, B, H, device=dev, dtype=torch.bfloat16)


def timeit(f, n=200):
    for _ in range(10):
        f()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(10):
            f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    g.replay()
    e0.record()
    for _ in range(n // 10):
        g.replay()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e3


t_in = timeit(lambda: dZin.t() @ X)
t_h = timeit(lambda: torch.bmm(dZ.transpose(1, 2), Y))
t_in32 = timeit(lambda: torch.matmul(dZin.t().float(), X.float()))
print(f"input dW (512x1024x4096) bf16 out: {t_in:.1f} us; hidden dW batched 6x(256x256x4096): {t_h:.1f} us; "
      f"sum {t_in + t_h:.1f} us (fused lgemm: ~15.7 us)")
print(f"fp32 input GEMM (tf32-free fp32 math) {t_in32:.1f} us")
