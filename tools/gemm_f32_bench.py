"""fp32 (reference-precision) GEMM throughput at the shapes of the fp32 bench
lines: the 4x320 BLSTM layers of att4x320 (B*T = 32000 rows, forward gx,
input gradient, weight gradient), the V = 10001 word CTC head of vgg_hier and
the VGG 3x3 convolutions as tap-addressed GEMMs (forward, input gradient,
weight gradient).  HIP-event time per launch and TF/s (f32 MFMA peak 157)."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

dev = torch.device('cuda:0')
ops.set_compute_dtype('fp32')
R = ops.rowmap


def timeit(fn, n=10):
    for _ in range(2):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


def f(*s, scale=1.0):
    return torch.randn(*s, device=dev) * scale


cases = []
M, H = 32000, 320
D = 2 * H
x, w, dg = f(M, D), f(8 * H, D, scale=0.05), f(M, 8 * H)
gx, dx, dw = torch.empty(M, 8 * H, device=dev), torch.empty(M, D, device=dev), torch.zeros(8 * H, D, device=dev)
cases += [
    ('lstm fwd M=32000 N=2560 K=640 (RR)', 2.0 * M * 8 * H * D,
     [ops.gemm_problem(ops.operand(x, 0, R(D)), ops.operand(w, 0, R(D)), gx, R(8 * H), M, 8 * H, D)]),
    ('lstm dX  M=32000 N=640 K=2560 (RK)', 2.0 * M * 8 * H * D,
     [ops.gemm_problem(ops.operand(dg, 0, R(8 * H)), ops.operand(w, 1, R(D)), dx, R(D), M, D, 8 * H)]),
    ('lstm dW  M=2560 N=640 K=32000 (KK)', 2.0 * M * 8 * H * D,
     [ops.gemm_problem(ops.operand(dg, 1, R(8 * H)), ops.operand(x, 1, R(D)), dw, R(D), 8 * H, D, M,
                       beta=1.0)]),
]
Mh, V = 8000, 10001
Vp = (V + 3) // 4 * 4   # the fp32 CTC head's logits pitch (native_ops.LinearCTC32Fn)
xh, wh, lg = f(Mh, D), f(V, D, scale=0.05), torch.empty(Mh, Vp, device=dev)
dlg, dxh, dwh = f(Mh, Vp), torch.empty(Mh, D, device=dev), torch.zeros(V, D, device=dev)
cases += [
    ('head fwd M=8000 N=10001 K=640 (RR)', 2.0 * Mh * V * D,
     [ops.gemm_problem(ops.operand(xh, 0, R(D)), ops.operand(wh, 0, R(D)), lg, R(Vp), Mh, V, D)]),
    ('head dX  M=8000 N=640 K=10001 (RK)', 2.0 * Mh * V * D,
     [ops.gemm_problem(ops.operand(dlg, 0, R(Vp)), ops.operand(wh, 1, R(D)), dxh, R(D), Mh, D, V)]),
    ('head dW  M=10001 N=640 K=8000 (KK)', 2.0 * Mh * V * D,
     [ops.gemm_problem(ops.operand(dlg, 1, R(Vp)), ops.operand(xh, 1, R(D)), dwh, R(D), V, D, Mh,
                       beta=1.0)]),
]
B = 32
for name, T, F, ci, co, sign in [('conv L1 fwd 64->64 F80', 1000, 80, 64, 64, 1),
                                  ('conv L1 dX 64->64 F80', 1000, 80, 64, 64, -1),
                                  ('conv L3 fwd 128->128 F40', 500, 40, 128, 128, 1)]:
    P = B * (T + 2) * (F + 2)
    xc, wc, out = f(P, ci), f(co, 9 * ci, scale=0.05), torch.empty(P, co, device=dev)
    cases.append(('%s P=%d' % (name, P), 2.0 * P * co * 9 * ci,
                  [ops.gemm_problem(ops._tap_operand(xc, 0, ci, ci, F + 2, sign),
                                    ops.operand(wc, 0, R(9 * ci)), out, R(co), P, co, 9 * ci)]))
for name, T, F, ci, co in [('conv L1 dW 64x64 F80', 1000, 80, 64, 64),
                           ('conv L3 dW 128x128 F40', 500, 40, 128, 128)]:
    P = B * (T + 2) * (F + 2)
    xc, dz, packed = f(P, ci), f(P, co, scale=0.1), torch.empty(co, 9 * ci, device=dev)
    cases.append(('%s P=%d' % (name, P), 2.0 * P * co * 9 * ci,
                  [ops.gemm_problem(ops.operand(dz, 1, R(co)), ops._tap_operand(xc, 1, ci, ci, F + 2, 1),
                                    packed, R(9 * ci), co, 9 * ci, P)]))

only = os.environ.get('GEMM_BENCH_ONLY')
print('-- fp32', ' '.join('%s=%s' % (k, v) for k, v in os.environ.items() if k.startswith('ASR_GEMM')))
for name, fl, probs in cases:
    if only and only not in name:
        continue
    t = timeit(lambda: ops.run_gemm(probs, dev))
    print('%-44s %9.1f us %6.1f TF/s' % (name, t, fl / t / 1e6), flush=True)
