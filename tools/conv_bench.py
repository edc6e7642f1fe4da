"""VGG 3x3 convolutions of the vgg_hier bench (B = 32, T = 1000, F = 80,
channels [64, 64, 128, 128], pools after layers 1 and 3): the tap-resident
kernel (asr_conv3x3_tr) against the tap-addressed GEMM, HIP-event time per
call and TF/s, forward (sign +1) and input-gradient (sign -1) geometries."""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

dev = torch.device('cuda:0')
ONLY_TR = os.environ.get('CONV_BENCH_ONLY_TR') == '1'   # profiling: the tap-resident kernels only
ops.set_compute_dtype('bf16')
B = 32
cases = [  # name, T, F, Cin, Cout, sign, out dtype
    ('L1 fwd 64->64   F80', 1000, 80, 64, 64, 1, torch.bfloat16),
    ('L1 dX  64->64   F80', 1000, 80, 64, 64, -1, torch.float32),
    ('L2 fwd 64->128  F40', 500, 40, 64, 128, 1, torch.bfloat16),
    ('L2 dX 128->64   F40', 500, 40, 128, 64, -1, torch.float32),
    ('L3 fwd 128->128 F40', 500, 40, 128, 128, 1, torch.bfloat16),
    ('L3 dX 128->128  F40', 500, 40, 128, 128, -1, torch.float32),
]


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) * 1000.0 / n


for name, T, F, ci, co, sign, odt in cases:
    P = B * (T + 2) * (F + 2)
    x = torch.randn(P, ci, device=dev).to(torch.bfloat16)
    w = (torch.randn(co, 9 * ci, device=dev) * 0.05).to(torch.bfloat16)
    b = torch.randn(co, device=dev) if sign == 1 else None
    out = torch.empty(P, co, dtype=odt, device=dev)
    fl = 2.0 * P * co * 9 * ci
    t_tr = timeit(lambda: ops.conv3x3_tr(x, P, ci, F + 2, sign, w, co, b, out))
    t_g = 1e9 if ONLY_TR else timeit(lambda: ops.run_gemm([ops.gemm_problem(
        ops._tap_operand(x, 0, ci, ci, F + 2, sign), ops.operand(w, 0, ops.rowmap(9 * ci)), out,
        ops.rowmap(co), P, co, 9 * ci, bias=b)], dev))
    print('%s  P=%d  tr %8.1f us %6.0f TF/s | tap GEMM %8.1f us %6.0f TF/s' % (
        name, P, t_tr, fl / t_tr / 1e6, t_g, fl / t_g / 1e6), flush=True)

# weight gradients (dz^T X over the pixels)
for name, T, F, ci, co in [('L1 dW 64x64 F80', 1000, 80, 64, 64), ('L2 dW 64->128 F40', 500, 40, 64, 128),
                           ('L3 dW 128x128 F40', 500, 40, 128, 128)]:
    P = B * (T + 2) * (F + 2)
    x = torch.randn(P, ci, device=dev).to(torch.bfloat16)
    dz = (torch.randn(P, co, device=dev) * 0.1).to(torch.bfloat16)
    packed = torch.empty(co, 9 * ci, device=dev)
    fl = 2.0 * P * co * 9 * ci
    t_tr = timeit(lambda: ops.conv3x3_tr_wgrad(x, dz, P, ci, F + 2, co, packed))
    t_g = 1e9 if ONLY_TR else timeit(lambda: ops.run_gemm([ops.gemm_problem(
        ops.operand(dz, 1, ops.rowmap(co)), ops._tap_operand(x, 1, ci, ci, F + 2, 1), packed,
        ops.rowmap(9 * ci), co, 9 * ci, P)], dev))
    print('%s  P=%d  tr %8.1f us %6.0f TF/s | tap GEMM %8.1f us %6.0f TF/s' % (
        name, P, t_tr, fl / t_tr / 1e6, t_g, fl / t_g / 1e6), flush=True)
