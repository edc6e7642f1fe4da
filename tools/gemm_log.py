"""Which host ops launch which GEMMs in one training step of a bench config:
every run_gemm call of the last of three steps with its caller chain, the
problems' M x N x K, operand dtypes / layouts and row maps, and the GEMM
kernel family the library ran (asr_gemm_last_family), so the generic-kernel
products and the small ops on the critical path can be named.

usage: python tools/gemm_log.py [config]      (GPU; bench.py's configs)
"""
import os
import sys
import traceback

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402
from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL  # noqa: E402

cfg = bench.CONFIGS[sys.argv[1] if len(sys.argv) > 1 else 'att4x320']
p = dict(cfg['params'])
model = load(cfg['model_type'], p, 'pytorch')
model.set_cuda()
model.set_precision('bf16')
model.set_optimizer(p['optimizer'], p['learning_rate'], weight_decay=p['weight_decay'],
                    lr_schedule=False)
F = bench.input_dim(p)
batch = bench.synthetic_batch(32, 1000, F, p['num_classes'], 0)
log = []
orig = ops.run_gemm


def logged(problems, device, lse=None):
    orig(problems, device, lse=lse)
    fam = N.lib().asr_gemm_last_family()
    st = [f for f in traceback.extract_stack()[:-1]
          if 'native_ops' in f.filename or 'models' in f.filename]
    where = ' < '.join('%s:%d' % (f.name, f.lineno) for f in reversed(st[-3:]))
    desc = []
    for pr in problems:
        desc.append('%dx%dx%d a%s%d b%s%d' % (pr.M, pr.N, pr.K, 'h' if pr.a.dtype else 'f',
                                              pr.a.trans, 'h' if pr.b.dtype else 'f', pr.b.trans))
    log.append((where, ' | '.join(desc), fam))


for step in range(3):
    if step == 2:
        ops.run_gemm = logged
    model, lv = TL.train_step(model, batch, clip_grad_norm=p['clip_grad_norm'])
torch.cuda.synchronize()
ops.run_gemm = orig
for i, (w, d, fam) in enumerate(log):
    print('%3d fam %2d  %-60s  %s' % (i, fam, d, w))
