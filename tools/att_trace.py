"""Phase stamps of the per-step attention kernels (work-group (0, 0), decoder
step 10; csrc/decoder.hip ATT_TR) after one hybrid4x320 training step."""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from pytorch_end2end_speech_recognition_amd import _native as N  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step  # noqa

cfg = bench.CONFIGS[os.environ.get('CONFIG', 'hybrid4x320')]
p = dict(cfg['params'])
torch.manual_seed(1623)
model = load(cfg['model_type'], p, 'pytorch')
model.set_cuda()
model.set_precision('bf16')
model.set_optimizer(p['optimizer'], p['learning_rate'], weight_decay=p['weight_decay'],
                    lr_schedule=False)
batch = bench.synthetic_batch(32, 1000, bench.input_dim(p), p['num_classes'], seed=0)
for _ in range(2):
    model, _ = train_step(model, batch, p['clip_grad_norm'])
torch.cuda.synchronize()
buf = (ctypes.c_ulonglong * 64)()
N.call('asr_att_trace_read', ctypes.cast(buf, ctypes.c_void_p))
tr = np.frombuffer(buf, dtype=np.uint64).astype(np.int64)


def ph(name, ks):
    parts = ['%s %.2f' % ('%d->%d' % (a, b), (tr[b] - tr[a]) / 100.0) for a, b in zip(ks, ks[1:])]
    print('%-16s total %.2f us | %s' % (name, (tr[ks[-1]] - tr[ks[0]]) / 100.0, '  '.join(parts)))


ph('att_energy', [0, 1, 2, 3, 4])
ph('att_bwd_energy', [10, 11, 12, 13, 15, 16, 17])
ph('att_bwd_conv', [20, 21, 22, 24, 23, 26])
ph('persist_fwd C', [32, 33, 34, 35, 36, 37])
ph('persist_fwd E', [37, 38, 39, 40, 41, 42])
ph('persist_fwd X', [42, 43, 44, 45, 46])
ph('persist_fwd step', [32, 37, 42, 46])
ph('persist_bwd H', [48, 49, 50, 51])
ph('persist_bwd E', [51, 52, 53, 54])
ph('persist_bwd F', [54, 55, 56, 57])
ph('persist_bwd G', [57, 58, 59, 60, 61])
ph('persist_bwd step', [48, 51, 54, 57, 61])
ph('persist_bwd F in', [55, 0, 1, 2, 3, 4, 56])
ph('persist_bwd G in', [59, 10, 11, 12, 13, 14, 60])
ph('persist_bwd E in', [51, 18, 10, 19, 27, 28, 29, 52])
