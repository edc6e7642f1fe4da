"""bf16 GEMM throughput at the BLSTM layer shapes of the 5x512 bench (B*T =
32000, H = 512): forward gx (R x R), input gradient (R x K), weight gradient
(K x K, split-K), each timed with HIP events over n launches."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

dev = torch.device('cuda:0')
ops.set_compute_dtype('bf16')
M, H = 32000, 512
D = 2 * H
bf = dict(dtype=torch.bfloat16, device=dev)
x = torch.randn(M, D, **bf)
w = torch.randn(8 * H, D, **bf) * 0.05
dg = torch.randn(M, 8 * H, **bf)
gx = torch.empty(M, 8 * H, device=dev)
dx = torch.empty(M, D, device=dev)
dw = torch.zeros(8 * H, D, device=dev)
R = ops.rowmap
x80 = torch.randn(M, 80, **bf)
w80 = torch.randn(8 * H, 80, **bf) * 0.05
shapes = {
    'fwd  M=32000 N=4096 K=1024 (RR)': [ops.gemm_problem(ops.operand(x, 0, R(D)), ops.operand(w, 0, R(D)),
                                                         gx, R(8 * H), M, 8 * H, D)],
    'fwdb M=32000 N=4096 K=1024 (RR) +bias pair': [
        ops.gemm_problem(ops.operand(x, 0, R(D)), ops.operand(w, 0, R(D)), gx, R(8 * H), M, 8 * H,
                         D, bias=torch.zeros(8 * H, device=dev), bias2=torch.zeros(8 * H, device=dev))],
    'fw80 M=32000 N=4096 K=80 (RR) +bias pair': [
        ops.gemm_problem(ops.operand(x80, 0, R(80)), ops.operand(w80, 0, R(80)), gx, R(8 * H), M,
                         8 * H, 80, bias=torch.zeros(8 * H, device=dev),
                         bias2=torch.zeros(8 * H, device=dev))],
    'dX   M=32000 N=1024 K=4096 (RK)': [ops.gemm_problem(ops.operand(dg, 0, R(8 * H)),
                                                         ops.operand(w, 1, R(D)), dx, R(D), M, D,
                                                         8 * H)],
    'dW   M=4096 N=1024 K=32000 (KK)': [ops.gemm_problem(ops.operand(dg, 1, R(8 * H)),
                                                         ops.operand(x, 1, R(D)), dw, R(D), 8 * H,
                                                         D, M, beta=1.0)],
    'dWhh 2x M=2048 N=512 K=32000 (KK)': [
        ops.gemm_problem(ops.operand(dg, 1, R(8 * H)), ops.operand(x, 1, R(D)), dw, R(H),
                         4 * H, H, M, beta=1.0),
        ops.gemm_problem(ops.operand(dg, 1, R(8 * H), offset=4 * H),
                         ops.operand(x, 1, R(D), offset=H), dw, R(H), 4 * H, H, M, beta=1.0,
                         c_offset=4 * H * H)],
}
tag = ' '.join('%s=%s' % (k, os.environ[k]) for k in ('ASR_GEMM_8W', 'ASR_GEMM_8R')
               if k in os.environ)
print('--', tag or 'defaults')
only = os.environ.get('GEMM_BENCH_ONLY')
for name, probs in shapes.items():
    if only and not name.startswith(only):
        continue
    for _ in range(3):
        ops.run_gemm(probs, dev)
    torch.cuda.synchronize()
    n = 20
    gap = int(os.environ.get('GEMM_BENCH_GAP', '0'))   # idle cycles before each launch
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(n)]
    fresh = os.environ.get('GEMM_BENCH_FRESH') == '1'   # a new C buffer per launch
    keep = []
    for i in range(n):
        if gap:
            torch.cuda._sleep(gap)
        if fresh:
            c = torch.empty(probs[0].M * probs[0].N + 64, device=dev)
            keep.append(c)
            if len(keep) > 3:
                keep.pop(0)
            for p in probs:
                p.c = c.data_ptr()
        ev[i][0].record()
        ops.run_gemm(probs, dev)
        ev[i][1].record()
    torch.cuda.synchronize()
    us = sum(a.elapsed_time(b) for a, b in ev) * 1000 / n
    fl = sum(2.0 * p.M * p.N * p.K for p in probs)
    print('%s  %8.1f us  %6.0f TF/s' % (name, us, fl / us / 1e6))
