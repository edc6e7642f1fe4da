"""Loss trajectory of the bench workload for A/B runs (env toggles)."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step  # noqa

steps = int(sys.argv[1]) if len(sys.argv) > 1 else 8
cfg = bench.CONFIGS['ctc5x512']
p = dict(cfg['params'])
if os.environ.get('NO_DROPOUT'):
    p['dropout_encoder'] = 0.0
torch.manual_seed(1623)
native_ops.manual_seed(1623)
model = load(cfg['model_type'], p, 'pytorch')
model.set_cuda()
model.set_precision(os.environ.get('PREC', 'bf16'))
model.set_optimizer(p['optimizer'], p['learning_rate'], weight_decay=p['weight_decay'],
                    lr_schedule=False)
batch = bench.synthetic_batch(32, 1000, 80, 28, seed=0)
out = []
for i in range(steps):
    model, lv = train_step(model, batch, p['clip_grad_norm'])
    out.append(lv)
print(' '.join('%.4f' % v for v in out))
