"""CTC forward + backward at the ctc5x512 shape (B 32 x T 1000, V 29, labels
60-125) for the lattice variants: run under rocprofv3 --kernel-trace --stats
with ASR_CTC_LATTICE_W=1|2|4 to read the lattice kernel's own duration."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from pytorch_end2end_speech_recognition_amd import native_ops  # noqa: E402

dev = torch.device('cuda:0')
B, T, V, Lmin, Lmax = 32, 1000, 29, 60, 125
rng = np.random.RandomState(0)
acts = torch.randn(B, T, V, device=dev, dtype=torch.float32).requires_grad_(True)
y_lens = rng.randint(Lmin, Lmax + 1, B).astype(np.int32)
labels = np.concatenate([rng.randint(1, V, l) for l in y_lens]).astype(np.int32)
act_lens = np.full(B, T, np.int32)
lab_d, yl_d, al_d = [torch.from_numpy(a).to(dev) for a in (labels, y_lens, act_lens)]
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for it in range(25):
    if it == 5:
        torch.cuda.synchronize()
        e0.record()
    loss, _ = native_ops.ctc_loss(acts, lab_d, yl_d, al_d, int(y_lens.max()), 1.0 / B)
e1.record()
torch.cuda.synchronize()
print('ASR_CTC_LATTICE_W=%s: ctc forward %.1f us / call, waves %d, loss %.6f' % (
    os.environ.get('ASR_CTC_LATTICE_W', 'default'), e0.elapsed_time(e1) * 1000.0 / 20,
    native_ops.N.lib().asr_ctc_last_lattice_waves(), float(loss)))
