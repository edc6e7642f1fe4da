"""The fused CTC output layer of vgg_hier's word head (B 32 x T' 250 frames,
640 -> V = 10001) as the step runs it: linear_ctc_loss forward + backward in
bf16 mode (LinearCTCFn) and fp32 mode (LinearCTC32Fn), 20 iterations each --
run under rocprofv3 --kernel-trace --stats for the per-kernel times of the
CTC op (ctc_lse_from_parts / ctc_emit_gather / ctc_lattice / ctc_grad*) and
the head GEMMs.  Prints the HIP-event time per iteration of each mode."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

dev = torch.device('cuda:0')
B, T, K, V = 32, 250, 640, 10001
rng = np.random.RandomState(0)
y_lens = rng.randint(10, 26, B).astype(np.int32)
labels = np.concatenate([rng.randint(1, V, l) for l in y_lens]).astype(np.int32)
lab, yl = torch.from_numpy(labels).to(dev), torch.from_numpy(y_lens).to(dev)
al = torch.full((B,), T, dtype=torch.int32, device=dev)
x = (torch.randn(B, T, K, device=dev) * 0.5).requires_grad_(True)
w = (torch.randn(V, K, device=dev) * 0.05).requires_grad_(True)
b = torch.zeros(V, device=dev, requires_grad=True)
for mode in os.environ.get('HEAD_MODES', 'bf16,fp32').split(','):
    ops.set_compute_dtype(mode)

    def it():
        x.grad = w.grad = b.grad = None
        loss, _ = ops.linear_ctc_loss(x, w, b, lab, yl, al, int(y_lens.max()), 1.0 / B)
        loss.backward()
    for _ in range(3):
        it()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        it()
    e1.record()
    torch.cuda.synchronize()
    print('%s head fwd+bwd %.1f us / iteration' % (mode, e0.elapsed_time(e1) * 1000.0 / 20),
          flush=True)
ops.set_compute_dtype('fp32')
