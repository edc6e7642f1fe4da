"""Isolate the fp32 persistent recurrence's reverse-direction gap on vgg_hier's
layer 0: replay the recorded layer input through ops.blstm_layer with the
persistent f32 kernels and the per-step ones, then vary one thing at a time."""
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
    if not rec:
        rec.append((x.detach().clone(), lens.detach().clone(), int(T), [t.detach().clone() for t in a], dict(kw)))
    return y


ops.blstm_layer = blstm_layer
dev = torch.device('cuda:0')
ops.recurrence_status(dev)
bench._gpu_loss(cfg, sd, sub, 'fp32')
print('status after the model forward', ops.recurrence_status(dev).tolist(), flush=True)
ops.blstm_layer = _orig
x, lens, T, ws, kw = rec[0]
print('x', tuple(x.shape), 'abs max %.3f std %.3f' % (float(x.abs().max()), float(x.std())),
      'lens', lens.tolist(), 'kw', {k: (v if not torch.is_tensor(v) else v.tolist()) for k, v in kw.items()
                                     if k in ('perm', 't_mul', 't_add', 'concat', 'drop', 'next_rec')},
      'w shapes', [tuple(w.shape) for w in ws[:4]], flush=True)
ops.set_compute_dtype('fp32')


def run(xx, ll, env, **k):
    os.environ.pop('ASR_LSTM_XG32', None)
    os.environ.update(env)
    with torch.no_grad():
        return _orig(xx, ll, T, *ws[:4], **k).detach().clone()


def cmp(tag, xx, ll, **k):
    a = run(xx, ll, {}, **k)
    st = ops.recurrence_status(dev).tolist()
    b = run(xx, ll, {'ASR_LSTM_XG32': '0'}, **k)
    print('   status', st, end=' ')
    H = a.shape[2] // 2
    d = (a - b).abs()
    print('%-34s fwd %.2e bwd %.2e' % (tag, float(d[..., :H].max()), float(d[..., H:].max())), flush=True)


cmp('replay (no perm)', x, lens)
if kw.get('perm') is not None:
    cmp('replay (perm)', x, lens, perm=kw['perm'])
cmp('all lens = T', x, torch.full_like(lens, T))
g = torch.Generator(device=x.device).manual_seed(3)
xr = torch.randn(x.shape, device=x.device, generator=g) * float(x.std())
cmp('random x same std', xr, lens)
cmp('x / 10', x / 10, lens)
cmp('B = 1 (utt 0)', x[:1].contiguous(), lens[:1].contiguous())
cmp('B = 2', x[:2].contiguous(), lens[:2].contiguous())
torch.save({'x': x.cpu(), 'lens': lens.cpu(), 'ws': [w.cpu() for w in ws[:4]]},
           os.path.join(ROOT, 'gpurun_out', 'l0_inputs.pt'))
