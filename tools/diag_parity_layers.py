"""vgg_hier parity sample: each BLSTM layer's output with the f32 persistent
recurrence vs the per-step kernels (ASR_LSTM_XG32=0), same process."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

cfg = bench.CONFIGS['vgg_hier']
p = cfg['params']
batch = bench.synthetic_hier_batch(32, 1000, bench.input_dim(p), p['num_classes'],
                                   p['num_classes_sub'], seed=0)
torch.manual_seed(1623)
model = bench.load(cfg['model_type'], dict(p), 'pytorch')
sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
sub = bench._sample(batch, 6)

rec = []
_orig = ops.blstm_layer


def blstm_layer(x, lens, T, *a, **kw):
    y = _orig(x, lens, T, *a, **kw)
    rec.append((x.detach().clone(), lens.detach().cpu().numpy().copy(), int(T), kw.get('perm'),
                y.detach().clone()))
    return y


ops.blstm_layer = blstm_layer
out = {}
for name in ('xg32', 'step'):
    os.environ.pop('ASR_LSTM_XG32', None)
    if name == 'step':
        os.environ['ASR_LSTM_XG32'] = '0'
    del rec[:]
    loss = bench._gpu_loss(cfg, sd, sub, 'fp32')
    out[name] = (loss, list(rec))
    print(name, 'loss', loss, 'layers', len(rec), flush=True)
for l, (a, b) in enumerate(zip(out['xg32'][1], out['step'][1])):
    xa, lens, T, perm, ya = a
    xb, _, _, _, yb = b
    dx = float((xa - xb).abs().max())
    d = (ya - yb).abs()
    print('layer %d T=%d lens %s perm %s x shape %s |dx| %.2e |dy| %.2e of %.2e; per utt %s' % (
        l, T, lens.tolist(), None if perm is None else perm.tolist() if hasattr(perm, 'tolist') else perm,
        tuple(xa.shape), dx, float(d.max()), float(yb.abs().max()),
        ' '.join('%.1e' % float(d[i].max()) for i in range(d.shape[0]))), flush=True)
    # where in time the first large difference appears, utterance 0
    dt = d.amax(dim=2)
    for i in range(d.shape[0]):
        bad = (dt[i] > 1e-4).nonzero()
        if len(bad):
            print('    utt %d first t with |dy| > 1e-4: %d (fwd %.2e bwd %.2e at that t)' % (
                i, int(bad[0]), float(d[i, int(bad[0]), :d.shape[2] // 2].max()),
                float(d[i, int(bad[0]), d.shape[2] // 2:].max())))
