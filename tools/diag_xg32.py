"""f32 persistent recurrence (lstm_fwd_xg<F32>) vs per-step f32 kernels vs a
float64 oracle: forward output error growth over T at H = 320."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from oracle import asr_ref  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

dev = torch.device('cuda:0')
ops.set_compute_dtype('fp32')
B, T, H, Din = int(os.environ.get('B', 32)), int(os.environ.get('T', 250)), 320, int(os.environ.get('DIN', 640))
rng = np.random.RandomState(5)
lens = np.full(B, T, np.int32)
if os.environ.get('RAGGED'):
    lens = np.sort(rng.randint(T * 4 // 5, T + 1, B))[::-1].astype(np.int32)
    lens[0] = T
x = torch.from_numpy(rng.randn(B, T, Din).astype(np.float32) * float(os.environ.get('XS', '0.5')))
sc = float(os.environ.get('WS', '0.1'))
ws = [torch.from_numpy(rng.uniform(-sc, sc, s).astype(np.float32))
      for s in ((8 * H, Din), (8 * H, H), (8 * H,), (8 * H,))]
if os.environ.get('FORGET1'):   # the reference init: gate biases 0, forget-gate biases 1
    for b in ws[2:]:
        b.zero_()
        for d in range(2):
            b[d * 4 * H + H:d * 4 * H + 2 * H] = 1.0
H4 = 4 * H
xd64 = x.double()
w64 = [w.double() for w in ws]
ref = torch.cat([asr_ref.lstm_direction(xd64, lens, w64[0][:H4], w64[1][:H4], w64[2][:H4], w64[3][:H4], False),
                 asr_ref.lstm_direction(xd64, lens, w64[0][H4:], w64[1][H4:], w64[2][H4:], w64[3][H4:], True)],
                dim=2).numpy()
for name, env in (('xg32', {}), ('step', {'ASR_LSTM_XG32': '0'})):
    os.environ.pop('ASR_LSTM_XG32', None)
    os.environ.update(env)
    y = ops.blstm_layer(x.to(dev), torch.from_numpy(lens).to(dev), T, *[w.to(dev) for w in ws])
    y = y.detach().cpu().numpy().astype(np.float64)
    e = np.abs(y - ref)
    fw = [float(e[:, t, :H].max()) for t in range(T)]
    eb = [float(e[b].max()) for b in range(B)]
    print('%-5s max |y - y64| %.2e  fwd dir at t=0,10,50,100,%d: %s' % (
        name, e.max(), T - 1, ' '.join('%.1e' % fw[t] for t in (0, 10, 50, 100, T - 1) if t < T)),
        flush=True)
    print('      per utterance: %s  lens %s' % (' '.join('%.1e' % v for v in eb), lens.tolist()), flush=True)

# determinism: the persistent f32 kernels twice on identical inputs
os.environ.pop('ASR_LSTM_XG32', None)
ys = [ops.blstm_layer(x.to(dev), torch.from_numpy(lens).to(dev), T, *[w.to(dev) for w in ws]).detach().cpu()
      for _ in range(3)]
print('xg32 repeat: max |y1 - y0| %.2e  |y2 - y0| %.2e' % (float((ys[1] - ys[0]).abs().max()),
                                                          float((ys[2] - ys[0]).abs().max())), flush=True)
