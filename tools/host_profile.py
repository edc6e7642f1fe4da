"""Host-side (Python) profile of train_step at a bench config: where the
per-step host time goes (cProfile over N steps after warmup)."""
import cProfile
import os
import pstats
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step  # noqa

cfg = bench.CONFIGS[os.environ.get('CONFIG', 'ctc5x512')]
p = dict(cfg['params'])
torch.manual_seed(1623)
model = load(cfg['model_type'], p, 'pytorch')
model.set_cuda()
model.set_precision('bf16')
model.set_optimizer(p['optimizer'], p['learning_rate'], weight_decay=p['weight_decay'],
                    lr_schedule=False)
batch = bench.synthetic_batch(32, 1000, bench.input_dim(p), p['num_classes'], seed=0)
batch['xs'] = torch.from_numpy(np.ascontiguousarray(batch['xs'])).cuda()
for _ in range(3):
    train_step(model, batch, p['clip_grad_norm'])
torch.cuda.synchronize()
pr = cProfile.Profile()
pr.enable()
for _ in range(10):
    train_step(model, batch, p['clip_grad_norm'])
pr.disable()
st = pstats.Stats(pr)
st.sort_stats('tottime').print_stats(25)
