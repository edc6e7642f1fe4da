"""CTC forward-backward alone (the warp-ctc replacement, asr_ctc_*) at the
bench shapes: HIP-event time per call and the algorithmic HBM rate
(activations read + gradient written = 8 V bytes per output frame;
the lattice state is not counted).  Writes one JSON line per shape."""
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops  # noqa: E402

dev = torch.device('cuda:0')
out = []
for (B, T, V, Lmin, Lmax) in [(32, 250, 10001, 10, 25), (32, 1000, 29, 60, 125),
                              (32, 250, 29, 60, 125)]:
    rng = np.random.RandomState(0)
    acts = torch.randn(B, T, V, device=dev, dtype=torch.float32).requires_grad_(True)
    y_lens = rng.randint(Lmin, Lmax + 1, B).astype(np.int32)
    labels = np.concatenate([rng.randint(1, V, l) for l in y_lens]).astype(np.int32)
    act_lens = np.full(B, T, np.int32)
    lab_d, yl_d, al_d = [torch.from_numpy(a).to(dev) for a in (labels, y_lens, act_lens)]
    for _ in range(3):
        acts.grad = None
        loss, _ = native_ops.ctc_loss(acts, lab_d, yl_d, al_d, int(y_lens.max()), 1.0 / B)
        loss.backward()
    torch.cuda.synchronize()
    n = 20
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        acts.grad = None
        loss, _ = native_ops.ctc_loss(acts, lab_d, yl_d, al_d, int(y_lens.max()), 1.0 / B)
        loss.backward()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / n
    nbytes = 8.0 * V * B * T
    rec = dict(kernel='ctc_fwd_bwd', B=B, T=T, V=V, us_per_call=round(us, 1),
               algorithmic_bytes=int(nbytes), achieved_GBs=round(nbytes / us / 1e3, 1),
               peak_GBs=8000.0, frac=round(nbytes / us / 1e3 / 8000.0, 4),
               note='whole ctc_loss forward + backward incl. allocation of grads; '
                    'lattice is sequential over T (latency-bound at small V)')
    out.append(rec)
    print(json.dumps(rec))
    # the fused CTC head's form: forward + the gradient written as the bf16,
    # column-padded dY operand of the output layer's GEMMs (asr_ctc_backward_bf16)
    N = native_ops.N
    Np = (V + 7) // 8 * 8
    nb = N.query('asr_ctc_workspace_bytes', T, B, V, int(y_lens.max()))
    ws = torch.empty(nb, dtype=torch.uint8, device=dev)
    costs = torch.empty(B, device=dev)
    lossb = torch.empty(1, device=dev)
    dyo = torch.empty(B * T, Np, dtype=torch.bfloat16, device=dev)
    st = N.stream_handle(dev)

    def call():
        N.call('asr_ctc_forward', N.ptr(acts), V, T * V, T, B, V, N.ptr(lab_d), N.ptr(yl_d),
               N.ptr(al_d), int(y_lens.max()), 0, 1, N.ptr(costs), N.ptr(lossb), 1.0 / B,
               N.ptr(ws), nb, st)
        N.call('asr_ctc_backward_bf16', N.ptr(acts), V, T * V, T, B, V, N.ptr(lab_d),
               N.ptr(yl_d), N.ptr(al_d), int(y_lens.max()), 0, None, 1.0 / B, N.ptr(dyo), Np,
               T * Np, Np, N.ptr(ws), nb, st)
    for _ in range(3):
        call()
    torch.cuda.synchronize()
    e0.record()
    for _ in range(n):
        call()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1000.0 / n
    actual = (4.0 * V + 4.0 * V + 2.0 * Np) * B * T
    rec = dict(kernel='ctc_fwd_bwd_bf16dy', B=B, T=T, V=V, us_per_call=round(us, 1),
               algorithmic_bytes=int(nbytes), achieved_GBs=round(nbytes / us / 1e3, 1),
               peak_GBs=8000.0, frac=round(nbytes / us / 1e3 / 8000.0, 4),
               bytes_moved_min=int(actual), moved_GBs=round(actual / us / 1e3, 1),
               note='forward (emission + lattice) + gradient as the bf16 padded GEMM '
                    'operand (the fused CTC head); algorithmic = SURVEY 8 V per frame, '
                    'bytes_moved_min = 4 V (emit) + 4 V + 2 Np (grad) per frame')
    out.append(rec)
    print(json.dumps(rec))
