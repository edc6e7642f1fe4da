"""bf16 parameter shadow (round 6, native_ops.param_shadow).

In bf16 mode the fused optimizer step also writes a bf16 copy of every
parameter it updates, and the next forward's BLSTM layers take their staged
W_ih from it instead of converting W_ih again.  Both roundings are the same
f2bf (csrc/common.h), so training with the shadow must be BITWISE the
training without it; a parameter written by anything but the optimizer step
voids the shadow for its layer.
"""
import numpy as np
import pytest
import torch

from test_grad_buckets_gpu import _batch, _kw
from test_model_ctc import _build


def _train(sd, batch, H, L, steps, poke, monkeypatch, shadow, fc=()):
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL
    monkeypatch.setenv('ASR_PARAM_SHADOW', '1' if shadow else '0')
    m = _build(dict(_kw(H, L), fc_list=list(fc)))
    m.load_state_dict(sd)
    m.set_cuda()
    m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
    native_ops.SHADOW_STATS['hits'] = 0
    native_ops.SHADOW_STATS['linear_hits'] = 0
    losses = []
    for i in range(steps):
        m, lv = TL.train_step(m, batch, clip_grad_norm=5.0)
        losses.append(float(lv))
        if poke and i == steps - 2:
            # an in-place write outside the optimizer step (a schedule that
            # rescales weights, a manual re-init): the shadow must not be used
            name, p = next((n, p) for n, p in m.named_parameters() if 'weight_ih' in n)
            with torch.no_grad():
                p.mul_(0.5)
    torch.cuda.synchronize()
    return (losses, m._flat_param.clone(), native_ops.SHADOW_STATS['hits'],
            native_ops.SHADOW_STATS['linear_hits'])


@pytest.mark.gpu
@pytest.mark.parametrize('poke', [False, True])
def test_shadow_training_bitwise_equals_conversion(poke, cuda_dev, monkeypatch):
    """With a dense staged fc layer (512 -> 640: the linear path reads its
    bf16 weight from the shadow too) between the encoder and the CTC head."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    H, L, steps, fc = 256, 3, 3, (640,)
    native_ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(1623)
        sd = {k: v.clone()
              for k, v in _build(dict(_kw(H, L), fc_list=list(fc))).state_dict().items()}
        batch = _batch(T=160)
        l0, p0, h0, q0 = _train(sd, batch, H, L, steps, poke, monkeypatch, False, fc)
        l1, p1, h1, q1 = _train(sd, batch, H, L, steps, poke, monkeypatch, True, fc)
    finally:
        native_ops.set_compute_dtype('fp32')
    assert h0 == 0 and q0 == 0
    # every layer of every forward after the first step reads the shadow,
    # except the poked layer's forward right after the poke; the fc layer too
    assert h1 == L * (steps - 1) - (1 if poke else 0), h1
    assert q1 == steps - 1, q1
    assert l0 == l1, (l0, l1)
    assert torch.equal(p0, p1), int((p0 != p1).sum())
    assert np.isfinite(l1).all()
