"""Diagnostic: run-to-run determinism of the 5x512 backward with side-stream
weight gradients (ASR_OVERLAP_WGRAD=2), with and without the recording
bucket shim of tests/test_grad_buckets_gpu.py.  Prints per-parameter max
gradient differences."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from test_grad_buckets_gpu import _batch, _kw, _Work  # noqa: E402
from test_model_ctc import _build  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops  # noqa: E402
from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL  # noqa: E402


def main():
    os.environ['ASR_OVERLAP_WGRAD'] = sys.argv[1] if len(sys.argv) > 1 else '2'
    dev = torch.device('cuda', 0)
    batch = _batch()
    native_ops.set_compute_dtype('bf16')
    torch.manual_seed(1623)
    sd = {k: v.clone() for k, v in _build(_kw()).state_dict().items()}

    def run(shim):
        m = _build(_kw())
        m.load_state_dict(sd)
        m.set_cuda()
        m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
        native_ops.recurrence_status(dev)
        if shim:
            TL._world, old_w = (lambda: 2), TL._world
            old_ar = dist.all_reduce
            dist.all_reduce = lambda t, op=None, async_op=False, **kw: (t.clone(), _Work())[1]
        try:
            m, lv = TL.train_step(m, batch, clip_grad_norm=5.0)
        finally:
            if shim:
                TL._world, dist.all_reduce = old_w, old_ar
        torch.cuda.synchronize()
        g = {k: p.grad.detach().clone() for k, p in m.named_parameters()}
        return lv, g, m._flat_param.clone()

    r1 = run(False)
    r2 = run(False)
    r3 = run(True)
    for name, r in (('ref2', r2), ('shim', r3)):
        print(name, 'loss', r[0], r1[0], 'param maxdiff', float((r[2] - r1[2]).abs().max()))
        for k in r1[1]:
            d = float((r[1][k] - r1[1][k]).abs().max())
            if d:
                print('   ', k, d, float(r1[1][k].abs().max()))


if __name__ == '__main__' and not (len(sys.argv) > 1 and sys.argv[1] == 'trace'):
    main()


def layer_trace():
    """Per-layer backward input dy of two identical runs (ASR_OVERLAP_WGRAD from
    argv[2]): where do the runs first differ?"""
    from pytorch_end2end_speech_recognition_amd import native_ops as no
    os.environ['ASR_OVERLAP_WGRAD'] = sys.argv[2] if len(sys.argv) > 2 else '2'
    H, L = int(os.environ.get('DIAG_H', 512)), int(os.environ.get('DIAG_L', 5))
    batch = _batch()
    no.set_compute_dtype('bf16')
    torch.manual_seed(1623)
    sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}
    if os.environ.get('DIAG_WHH'):     # contracting recurrence: no chaotic amplification
        sc = float(os.environ['DIAG_WHH'])
        for k in sd:
            if 'weight_hh' in k:
                sd[k] = sd[k] * (sc / 0.1)
    orig = no.BLSTMLayerFn.backward

    extras = []

    def run():
        rec = []
        extra = []
        extras.append(extra)

        def bwd(ctx, dy):
            saved = ctx.saved_tensors
            rec.append(dy.detach().clone())
            out = orig(ctx, dy)
            rec.append(out[0].detach().clone() if out[0] is not None else None)
            if os.environ.get('DIAG_INPUTS'):
                torch.cuda.synchronize()
                # the recurrence's inputs, read back after it ran: x_op, act, cst, y_op, dy
                extra.append([t.detach().clone() for t in (saved[0], saved[6], saved[7],
                                                          saved[8], dy)])
            return out

        no.BLSTMLayerFn.backward = staticmethod(bwd)
        try:
            m = _build(_kw(H, L))
            m.load_state_dict(sd)
            m.set_cuda()
            m.zero_grad()
            loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
            loss.backward()
            torch.cuda.synchronize()
        finally:
            no.BLSTMLayerFn.backward = orig
        return rec

    a, b = run(), run()
    if extras[0]:
        for i, (x, y) in enumerate(zip(extras[0], extras[1])):
            print('call %d after-run inputs maxdiff x_op %.3e act %.3e cst %.3e y_op %.3e dy %.3e' % (
                (i,) + tuple(float((u.float() - v.float()).abs().max()) for u, v in zip(x, y))))
    for i, (x, y) in enumerate(zip(a, b)):
        if x is None:
            continue
        print('layer-backward call %d %s maxdiff %.3e (max %.3e)' % (
            i // 2, 'dy ' if i % 2 == 0 else 'dx ', float((x - y).abs().max()),
            float(x.abs().max())))


if __name__ == '__main__' and len(sys.argv) > 1 and sys.argv[1] == 'trace':
    layer_trace()
