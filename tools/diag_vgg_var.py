"""Diagnose test_vgg_fused_bn_variance_matches_two_pass[fp32]: each of
(f32 fast GEMM on/off) x (fused BN variance on/off) against the float64
oracle."""
import os
import sys

import numpy as np
import torch

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
sys.path.insert(0, os.path.join(root, 'tests'))
import test_parity_pins_gpu as t  # noqa: E402

kw = dict(t.VGG_PROD, input_size=40)
model = t._ctc(kw)
model.set_cuda()   # as the test: the running means drawn on the device
with torch.no_grad():
    for k, v in model.state_dict().items():
        if k.endswith('running_mean'):
            v.uniform_(0.0, 0.5)
sd0 = {k: v.clone() for k, v in model.state_dict().items()}
batch = t._vgg_batch(40, seed=12)
ref_loss, ref_g = t._oracle({k: v.cpu() for k, v in sd0.items()}, t._vgg_cfg(kw), batch,
                            dtype=torch.float64)
variants = [{}, {'ASR_GEMM_F32FAST': '0'}, {'ASR_GEMM_F32FAST_NOTAP': '1'},
            {'ASR_GEMM_F32FAST_MASK': '1'}, {'ASR_GEMM_F32FAST_MASK': '2'},
            {'ASR_GEMM_F32FAST_MASK': '4'}, {'ASR_GEMM_F32FAST_MASK': '8'},
            {'ASR_GEMM_NOSPLIT': '1'}, {'ASR_VGG_WGRAD_SIDE': '0', 'ASR_OVERLAP_WGRAD': '0'}]
for var in variants:
    for k in ('ASR_GEMM_F32FAST', 'ASR_GEMM_F32FAST_NOTAP', 'ASR_GEMM_F32FAST_MASK', 'ASR_GEMM_NOSPLIT',
              'ASR_VGG_WGRAD_SIDE', 'ASR_OVERLAP_WGRAD'):
        os.environ.pop(k, None)
    os.environ.update(var)
    os.environ['ASR_VGG_FUSED_VAR'] = '1'
    model.load_state_dict(sd0)
    loss, g = t._gpu_grads(model, batch, 'fp32')
    errs = sorted(((t._rel_l2(g[k], ga), k) for k, ga in ref_g.items()), reverse=True)[:2]
    print('%-70s loss %.2e  worst %s' % (
        var, abs(loss - ref_loss) / abs(ref_loss),
        ', '.join('%s %.2e' % (k.replace('encoder.conv.layers.', 'conv'), e) for e, k in errs)),
        flush=True)
