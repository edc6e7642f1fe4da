"""The row-blocked bf16 VGG element-wise passes (csrc/cnn.hip rw_apply /
rw_post_fwd / rw_bn_moments / rw_post_bwd) against the grid-stride passes they
replace (ASR_VGG_ROWS=0), through the C entry points asr_vgg_block_forward_zp /
asr_vgg_block_backward_zdp on the same inputs.

Per element the arithmetic is the same, so P, the pool argmax slots, the
next-layer input in eval mode and the input gradient given the same batch
statistics are bitwise equal; the per-channel sums (batch mean / variance, the
BN-backward moments, the conv-bias gradient) are the same values summed in a
different fixed order, compared at f32 rounding.  Shapes: the 64- and
128-channel vgg_hier layers, 2 x 2 pooling with an odd time extent (ceil-mode
partial windows), padded bf16 and flat f32 neighbours.
Reference: models/pytorch_v3/encoders/cnn.py:92-111, 124-165 (ReLU, MaxPool2d,
BatchNorm2d of the VGG blocks)."""
import ctypes

import numpy as np
import pytest
import torch

BF16, F32 = 1, 0


def _N():
    from pytorch_end2end_speech_recognition_amd import _native as N
    return N


def _pool_dims(T, F, pt, ceil):
    N = _N()
    To, Fo = ctypes.c_int(), ctypes.c_int()
    if not pt:
        return T, F
    N.call('asr_vgg_pool_dims', T, F, pt, pt, ceil, ctypes.byref(To), ctypes.byref(Fo))
    return To.value, Fo.value


def _case(B, T, F, C, pt, seed):
    g = torch.Generator().manual_seed(seed)
    z = torch.zeros(B, T + 2, F + 2, C)
    z[:, 1:-1, 1:-1] = torch.randn(B, T, F, C, generator=g)
    To, Fo = _pool_dims(T, F, pt, 1)
    return dict(z=z.reshape(-1, C), To=To, Fo=Fo,
                gamma=torch.rand(C, generator=g) + 0.5, beta=torch.randn(C, generator=g) * 0.1,
                run_mean=torch.randn(C, generator=g) * 0.1, run_var=torch.rand(C, generator=g) + 0.5,
                dnext_pad=torch.randn(B, To + 2, Fo + 2, C, generator=g),
                dnext_flat=torch.randn(B, To, Fo, C, generator=g))


def _fwd(c, B, T, F, C, pt, training, flat, dev, rows, monkeypatch):
    N = _N()
    monkeypatch.setenv('ASR_VGG_ROWS', '1' if rows else '0')
    To, Fo = c['To'], c['Fo']
    z = c['z'].to(dev).to(torch.bfloat16)
    P = torch.empty(B * To * Fo, C, dtype=torch.bfloat16, device=dev)
    slot = torch.zeros(B * To * Fo * C, dtype=torch.uint8, device=dev) if pt else None
    rm, rv = c['run_mean'].clone().to(dev), c['run_var'].clone().to(dev)
    mean, rstd = torch.empty(C, device=dev), torch.empty(C, device=dev)
    if flat:
        out = torch.zeros(B, To, Fo * C, device=dev)
        odt = F32
    else:
        out = torch.zeros(B * (To + 2) * (Fo + 2), C, dtype=torch.bfloat16, device=dev)
        odt = BF16
    nb = N.query('asr_vgg_block_workspace_bytes', B, To, Fo, C)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    N.call('asr_vgg_block_forward_zp', N.ptr(z), BF16, B, T, F, C, pt, pt, 1, N.ptr(P), BF16,
           N.ptr(slot), N.ptr(c['gamma'].to(dev)), N.ptr(c['beta'].to(dev)), N.ptr(rm), N.ptr(rv),
           int(training), 0.1, 1e-5, N.ptr(mean), N.ptr(rstd), 0.0, 0, N.ptr(out), odt, int(flat),
           N.ptr(ws), nb, N.stream_handle(dev))
    torch.cuda.synchronize()
    return dict(P=P, slot=slot, out=out, mean=mean, rstd=rstd, rm=rm, rv=rv, z=z)


def _bwd(c, f, B, T, F, C, pt, flat, dnext_bf16, dev, rows, monkeypatch):
    N = _N()
    monkeypatch.setenv('ASR_VGG_ROWS', '1' if rows else '0')
    To, Fo = c['To'], c['Fo']
    if flat:
        dn = c['dnext_flat'].to(dev).contiguous()
        ddt = F32
    else:
        dn = c['dnext_pad'].to(dev)
        dn = (dn.to(torch.bfloat16) if dnext_bf16 else dn).reshape(-1, C).contiguous()
        ddt = BF16 if dnext_bf16 else F32
    dz = torch.zeros(B * (T + 2) * (F + 2), C, dtype=torch.bfloat16, device=dev)
    dgamma, dbeta, dbias = (torch.zeros(C, device=dev) for _ in range(3))
    nb = N.query('asr_vgg_block_workspace_bytes', B, To, Fo, C)
    ws = torch.empty(max(nb, 1), dtype=torch.uint8, device=dev)
    N.call('asr_vgg_block_backward_zdp', N.ptr(dn), ddt, int(flat), N.ptr(f['z']), BF16, B, T, F,
           C, pt, pt, 1, N.ptr(f['P']), BF16, N.ptr(f['slot']), N.ptr(c['gamma'].to(dev)),
           N.ptr(f['mean']), N.ptr(f['rstd']), N.ptr(dgamma), N.ptr(dbeta), 0.0, 0, N.ptr(dz), BF16,
           N.ptr(dbias), N.ptr(ws), nb, N.stream_handle(dev))
    torch.cuda.synchronize()
    return dict(dz=dz, dgamma=dgamma, dbeta=dbeta, dbias=dbias)


def _rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.gpu
@pytest.mark.parametrize('B,T,F,C,pt,flat', [(4, 37, 40, 64, 2, False), (3, 20, 16, 128, 0, False),
                                             (2, 25, 20, 64, 0, False), (3, 17, 10, 128, 2, True)])
def test_row_passes_match_grid_stride(B, T, F, C, pt, flat, cuda_dev, monkeypatch):
    c = _case(B, T, F, C, pt, seed=B * 100 + C)
    # eval mode: the running statistics, so every output is elementwise arithmetic
    fe = {r: _fwd(c, B, T, F, C, pt, False, flat, cuda_dev, r, monkeypatch) for r in (True, False)}
    for k in ('P', 'out'):
        assert torch.equal(fe[True][k], fe[False][k]), k
    if pt:
        assert torch.equal(fe[True]['slot'], fe[False]['slot'])
    # training: batch statistics summed in another fixed order
    ft = {r: _fwd(c, B, T, F, C, pt, True, flat, cuda_dev, r, monkeypatch) for r in (True, False)}
    assert torch.equal(ft[True]['P'], ft[False]['P'])
    for k in ('mean', 'rstd', 'rm', 'rv'):
        assert _rel(ft[True][k], ft[False][k]) <= 1e-5, (k, _rel(ft[True][k], ft[False][k]))
    assert _rel(ft[True]['out'].float(), ft[False]['out'].float()) <= 1e-3
    # backward from the same saved tensors and statistics
    for dnb in ((False,) if flat else (True, False)):
        bw = {r: _bwd(c, ft[False], B, T, F, C, pt, flat, dnb, cuda_dev, r, monkeypatch)
              for r in (True, False)}
        for k in ('dgamma', 'dbeta', 'dbias'):
            assert _rel(bw[True][k], bw[False][k]) <= 1e-5, (k, dnb, _rel(bw[True][k], bw[False][k]))
        d1, d0 = bw[True]['dz'].float(), bw[False]['dz'].float()
        # the BN-backward sums differ in their last bits: dz within bf16 rounding
        assert _rel(d1, d0) <= 2e-3, (dnb, _rel(d1, d0))
        assert float((d1 - d0).abs().max()) <= 8e-3 * float(d0.abs().max()), dnb
        assert float(d0.abs().sum()) > 0


@pytest.mark.gpu
def test_first_layer_relu_p_matches_separate_pass(cuda_dev, monkeypatch):
    """The first VGG layer's stencil writing P = max(0, bf16 z) and the batch-norm
    moment partials itself (asr_vgg_c1_forward_relu_p, no z) against the stencil
    + ReLU pass (ASR_VGG_C1_RELU_P=0), production channel plan, bf16: eval-mode
    losses (running statistics: elementwise arithmetic only) bitwise equal; in
    training the moments are summed in another fixed order, so the loss agrees
    to f32 rounding moved through bf16 roundings and the gradients to the
    bf16-flip level of the batch-norm backward."""
    from test_parity_pins_gpu import VGG_PROD, _ctc, _vgg_batch, _with_env
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(VGG_PROD, input_size=40)
    model = _ctc(kw)
    model.set_cuda()
    batch = _vgg_batch(40, seed=21)
    xs, ys, x_lens, y_lens = batch
    native_ops.set_compute_dtype('bf16')
    try:
        ev = {}
        for v in ('1', '0'):
            monkeypatch.setenv('ASR_VGG_C1_RELU_P', v)
            model.eval()
            with torch.no_grad():
                ev[v] = float(model(xs, ys, x_lens, y_lens, is_eval=True))
        model.train()
    finally:
        monkeypatch.delenv('ASR_VGG_C1_RELU_P', raising=False)
        native_ops.set_compute_dtype('fp32')
    assert ev['1'] == ev['0'], ev
    l1, g1 = _with_env(monkeypatch, 'ASR_VGG_C1_RELU_P', '1', model, batch, 'bf16')
    l0, g0 = _with_env(monkeypatch, 'ASR_VGG_C1_RELU_P', '0', model, batch, 'bf16')
    np.testing.assert_allclose(l1, l0, rtol=5e-5)
    for k in g0:
        d = float(np.linalg.norm(g1[k] - g0[k]) / max(np.linalg.norm(g0[k]), 1e-30))
        assert d <= 5e-2, (k, d)


@pytest.mark.gpu
def test_conv_weight_gradients_on_side_stream_bitwise(cuda_dev, monkeypatch):
    """The VGG convolutions' weight gradients on a side stream beside the input
    gradient and the layer below's passes (ASR_VGG_WGRAD_SIDE, default on)
    against the same kernels on the compute stream: loss and every gradient
    bit for bit (production channel plan, bf16, training-mode BN)."""
    from test_parity_pins_gpu import VGG_PROD, _ctc, _vgg_batch, _with_env
    kw = dict(VGG_PROD, input_size=40)
    model = _ctc(kw)
    model.set_cuda()
    batch = _vgg_batch(40, seed=5)
    l1, g1 = _with_env(monkeypatch, 'ASR_VGG_WGRAD_SIDE', '1', model, batch, 'bf16')
    l0, g0 = _with_env(monkeypatch, 'ASR_VGG_WGRAD_SIDE', '0', model, batch, 'bf16')
    assert l1 == l0, (l1, l0)
    for k in g0:
        np.testing.assert_array_equal(g1[k], g0[k], err_msg=k)
