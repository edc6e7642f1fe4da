"""Diagnostic: bf16 gradient error of the production-shape attention model
(tests/golden/model_att_prod*.npz) per recurrence implementation, to tell
bf16 rounding amplification from a kernel defect.  Usage (GPU box):
    ASR_LSTM_PERSIST=0 python tools/att_prod_bf16_diag.py"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'tests')]
import torch  # noqa: E402
import test_attention_prod as T  # noqa: E402

dev = torch.device('cuda', 0)
for name in T.NAMES:
    for prec in ('fp32', 'bf16'):
        d, loss, grads, launch = T._gpu_run(name, prec, dev)
        errs = T._norm_errors(d, grads)
        worst = sorted(errs.items(), key=lambda kv: -kv[1])[:5]
        print(name, prec, 'env PERSIST=%s XG=%s' % (os.environ.get('ASR_LSTM_PERSIST', '1'),
                                                   os.environ.get('ASR_LSTM_XG', '1')),
              'loss err %.2e' % (abs(loss - float(d['loss'][0])) / abs(float(d['loss'][0]))),
              ' '.join('%s=%.3f' % kv for kv in worst), flush=True)
