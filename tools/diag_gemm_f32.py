"""Find fp32-mode products whose f32 fast kernel result differs from the
generic kernel's inside the VGG production model step (the failing
test_vgg_fused_bn_variance_matches_two_pass[fp32] setup): every run_gemm call
is run twice (fast, then generic from the same C) and compared."""
import os
import sys

import numpy as np
import torch

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
sys.path.insert(0, os.path.join(root, 'tests'))
import test_parity_pins_gpu as t  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402

_c = {}
_orig_problem = ops.gemm_problem
_orig_run = ops.run_gemm


def gemm_problem(a, b, c, c_map, M, N_, K, *args, **kw):
    p = _orig_problem(a, b, c, c_map, M, N_, K, *args, **kw)
    _c[id(p)] = (c, int(M), int(N_), int(K), a.trans, b.trans, a.tap_group, b.tap_group)
    return p


calls = [0]


def run_gemm(problems, device, lse=None):
    if ops.compute_dtype() != ops.F32 or lse is not None:
        return _orig_run(problems, device, lse=lse)
    cs = [_c.get(id(p)) for p in problems]
    torch.cuda.synchronize()
    before = [c[0].clone() for c in cs]
    _orig_run(problems, device)
    torch.cuda.synchronize()
    fast = [c[0].clone() for c in cs]
    for c, b0 in zip(cs, before):
        c[0].copy_(b0)
    os.environ['ASR_GEMM_F32FAST'] = '0'
    _orig_run(problems, device)
    torch.cuda.synchronize()
    os.environ.pop('ASR_GEMM_F32FAST')
    calls[0] += 1
    for c, f in zip(cs, fast):
        g = c[0]
        d = float((f - g).abs().max())
        s = float(g.abs().max()) + 1e-30
        tag = 'MISMATCH' if d > 1e-4 * s else 'ok'
        if tag != 'ok' or os.environ.get('DIAG_ALL'):
            bad = (f - g).abs() > 1e-4 * s
            idx = bad.nonzero()[:4].tolist() if tag != 'ok' else []
            print('%s call %d M=%d N=%d K=%d trans=(%d,%d) taps=(%d,%d) max|d| %.3e of %.3e first bad %s'
                  ' C shape %s' % (tag, calls[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], d, s, idx,
                                   tuple(g.shape)), flush=True)
        g.copy_(f)   # continue with the fast result, as the step would


ops.gemm_problem = gemm_problem
ops.run_gemm = run_gemm
ops._tap_operand.__globals__['gemm_problem'] = gemm_problem
ops._tap_operand.__globals__['run_gemm'] = run_gemm

kw = dict(t.VGG_PROD, input_size=40)
model = t._ctc(kw)
model.set_cuda()
with torch.no_grad():
    for k, v in model.state_dict().items():
        if k.endswith('running_mean'):
            v.uniform_(0.0, 0.5)
sd0 = {k: v.clone() for k, v in model.state_dict().items()}
batch = t._vgg_batch(40, seed=12)
ref_loss, ref_g = t._oracle({k: v.cpu() for k, v in sd0.items()}, t._vgg_cfg(kw), batch,
                            dtype=torch.float64)
os.environ['ASR_VGG_FUSED_VAR'] = '1'
os.environ['ASR_VGG_WGRAD_SIDE'] = '0'
for check in (True, False):
    model.load_state_dict(sd0)
    if not check:
        ops.run_gemm = _orig_run
        ops._tap_operand.__globals__['run_gemm'] = _orig_run
    loss, g = t._gpu_grads(model, batch, 'fp32')
    errs = sorted(((t._rel_l2(g[k], ga), k) for k, ga in ref_g.items()), reverse=True)[:2]
    print('checked' if check else 'plain', 'calls', calls[0], 'loss', loss, errs, flush=True)
