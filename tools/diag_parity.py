"""vgg_hier fp32 parity ('full' sample of bench.parity_report) under one set
of switches (taken from the environment): GPU fp32 eval loss vs the float64
reference (cached in gpurun_out/diag_parity_ref.json)."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

cfg = bench.CONFIGS[os.environ.get('DIAG_CONFIG', 'vgg_hier')]
p = cfg['params']
batch = bench.synthetic_hier_batch(32, 1000, bench.input_dim(p), p['num_classes'],
                                   p['num_classes_sub'], seed=0)
torch.manual_seed(1623)
model = bench.load(cfg['model_type'], dict(p), 'pytorch')
sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
sub = bench._sample(batch, 6)
T = int(os.environ.get('DIAG_T', '0'))
if T:
    sub = bench._truncate(sub, T)
cache = os.path.join(ROOT, 'gpurun_out', 'diag_parity_ref_%d.json' % T)
if os.path.exists(cache):
    ref = json.load(open(cache))
else:
    torch.set_num_threads(16)
    ref = bench._ref_losses(cfg, sd, sub)
    json.dump(ref, open(cache, 'w'))
got = bench._gpu_loss(cfg, sd, sub, 'fp32')
sw = ' '.join('%s=%s' % (k, v) for k, v in sorted(os.environ.items()) if k.startswith('ASR_'))
print('%-40s T=%d fp32 %.6f ref64 %.6f rel %.3e (ref f32 rel %.1e)' % (
    sw or 'default', T, got, ref['f64'], abs(got - ref['f64']) / abs(ref['f64']),
    abs(ref['f32'] - ref['f64']) / abs(ref['f64'])), flush=True)
