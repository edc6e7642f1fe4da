"""Library GEMM rate at the 5x512 BLSTM shapes (torch.matmul -> hipBLASLt /
rocBLAS on ROCm), for comparison with tools/gemm_bench.py's native kernels.
Diagnostic only: the product path never calls torch.matmul."""
import torch

dev = torch.device('cuda:0')
M, H = 32000, 512
D = 2 * H
bf = dict(dtype=torch.bfloat16, device=dev)
x = torch.randn(M, D, **bf)
w = torch.randn(8 * H, D, **bf) * 0.05
dg = torch.randn(M, 8 * H, **bf)
cases = {
    'fwd  M=32000 N=4096 K=1024': (lambda: x @ w.t(), 2.0 * M * 8 * H * D),
    'dX   M=32000 N=1024 K=4096': (lambda: dg @ w, 2.0 * M * D * 8 * H),
    'dW   M=4096 N=1024 K=32000': (lambda: dg.t() @ x, 2.0 * 8 * H * D * M),
}
for name, (fn, fl) in cases.items():
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    n = 20
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n):
        fn()
    b.record()
    torch.cuda.synchronize()
    us = a.elapsed_time(b) * 1000 / n
    print('%-30s %8.1f us  %7.1f TF/s (bf16 out)' % (name, us, fl / us / 1e6))
