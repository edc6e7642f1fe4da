"""VGG front-end (CNNEncoder, models/pytorch_v3/encoders/cnn.py) before the
BLSTM, inside the drop-in CTC model, vs golden vectors recorded from the
reference (tests/golden/make_golden.py case_vgg_model: batch norm with ceil-mode
pooling over an odd length, and conv bias without batch norm).

CPU: bit-identical initial state_dict under the reference's seed (same
nn.Sequential module indices), the oracle restatement vs the golden loss and
gradients.  GPU: loss, every gradient and the updated BatchNorm running
statistics through the HIP path (tap-addressed implicit-GEMM convolutions);
bf16 fast path (C_in multiple of 64) vs the oracle at a larger shape."""
import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_params
from oracle import asr_ref

NAMES = ['model_vgg_bn', 'model_vgg_nobn']


def _build(kw):
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.ctc.ctc import CTC
    torch.manual_seed(1623)
    return CTC(**kw)


def _cfg(kw):
    return dict(num_layers=kw['encoder_num_layers'], subsample_list=kw['subsample_list'],
                fc_list=kw['fc_list'], conv_channels=kw['conv_channels'],
                poolings=kw['poolings'], batch_norm=kw['batch_norm'])


def _float_params(p):
    return {k: v for k, v in p.items() if v.is_floating_point() and 'running' not in k}


@pytest.mark.parametrize('name', NAMES)
def test_vgg_init_matches_reference_state_dict(name):
    d = golden(name)
    model = _build(json.loads(str(d['kwargs'])))
    sd = model.state_dict()
    ref = {k[3:]: d[k] for k in d.files if k.startswith('sd/')}
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


@pytest.mark.parametrize('name', NAMES)
def test_vgg_conv_lens_quirk(name):
    """ConvOutSize floors every pool, so the ceil-mode pool's extra frame is not
    counted (cnn_utils.py:34-37)."""
    d = golden(name)
    model = _build(json.loads(str(d['kwargs'])))
    lens = [model.encoder.conv.conv_out_len(int(x)) for x in d['x_lens']]
    np.testing.assert_array_equal(lens, d['conv_lens'])


@pytest.mark.parametrize('name', NAMES)
def test_vgg_oracle_matches_golden(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    p, g = golden_params(d)
    for v in _float_params(p).values():
        v.requires_grad_(True)
    loss, _, _, _ = asr_ref.ctc_model_loss(p, _cfg(kw), d['xs'], d['ys'], d['x_lens'],
                                           d['y_lens'])
    np.testing.assert_allclose(float(loss), float(d['loss'][0]), rtol=1e-5)
    loss.backward()
    for k, v in _float_params(p).items():
        np.testing.assert_allclose(v.grad.numpy(), g[k], rtol=1e-4, atol=1e-6, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize('name', NAMES)
def test_vgg_model_matches_golden(name, cuda_dev):
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('fp32')
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    sd, g = golden_params(d)
    model = _build(kw)
    model.load_state_dict(sd)
    model.set_cuda()
    model.zero_grad()
    loss = model(d['xs'], d['ys'], d['x_lens'], d['y_lens'])
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.item(), float(d['loss'][0]), rtol=1e-4)
    for k, p in model.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g[k], rtol=2e-3, atol=2e-5, err_msg=k)
    after = model.state_dict()
    for k in d.files:
        if k.startswith('after/'):
            np.testing.assert_allclose(after[k[6:]].cpu().numpy(), d[k], rtol=1e-4, atol=1e-6,
                                       err_msg=k)


@pytest.mark.gpu
def test_vgg_bf16_fast_path_vs_oracle(cuda_dev):
    """Reference VGG channel plan (64, 64, 128, 128; pools after layers 2 and 4)
    so layers 2-4 take the bf16 buffer->LDS GEMM with tap addressing."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=16, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=32, encoder_num_proj=0, encoder_num_layers=2, fc_list=[],
              dropout_input=0, dropout_encoder=0, num_classes=6, parameter_init=0.1,
              subsample_list=[], subsample_type='drop', conv_channels=[64, 64, 128, 128],
              conv_kernel_sizes=[[3, 3]] * 4, conv_strides=[[1, 1]] * 4,
              poolings=[[], [2, 2], [], [2, 2]], activation='relu', batch_norm=True)
    model = _build(kw)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    rng = np.random.RandomState(9)
    B, T = 3, 41
    x_lens = np.array([41, 30, 22], np.int32)
    y_lens = np.array([4, 3, 2], np.int32)
    xs = rng.randn(B, T, 16).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 4), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 6, y_lens[b])
    p = {k: v.clone() for k, v in sd.items()}
    for v in _float_params(p).values():
        v.requires_grad_(True)
    ref, _, _, _ = asr_ref.ctc_model_loss(p, _cfg(kw), xs, ys, x_lens, y_lens)
    ref.backward()
    native_ops.set_compute_dtype('bf16')
    try:
        model.set_cuda()
        model.zero_grad()
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        native_ops.set_compute_dtype('fp32')
    # bf16 operands (activations, dZ, weights) with f32 accumulation: the batch-norm
    # backward subtracts per-channel means, so the weight-gradient sums over the
    # pixels cancel heavily and carry ~1e-1 of max |g| (tools/vgg_diag.py: fp32
    # mode at this shape is ~1e-5).  Exactness of the tap-addressed GEMMs
    # themselves: test_tap_gemm_conv_exact.
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 2e-2
    for k, prm in model.named_parameters():
        if 'conv' not in k:
            continue
        ga = p[k].grad.numpy()
        gw = prm.grad.cpu().numpy()
        scale = np.abs(ga).max() + 1e-6
        assert np.abs(gw - ga).max() / scale < 0.25, (k, np.abs(gw - ga).max(), scale)
        # the tensor as a whole: relative Frobenius error and direction
        fro = np.linalg.norm(gw - ga) / (np.linalg.norm(ga) + 1e-12)
        cos = float((gw * ga).sum() / (np.linalg.norm(gw) * np.linalg.norm(ga) + 1e-30))
        # measured on MI355X: fro 0.003-0.18, cos >= 0.984 (BN's cancellation at B = 3)
        assert fro < 0.3 and cos > 0.97, (k, fro, cos)


@pytest.mark.gpu
@pytest.mark.parametrize('fast,n64st', [('1', '2'), ('1', '3'), ('0', '2')])
@pytest.mark.parametrize('Ci,Co', [(64, 64), (64, 128), (128, 128)])
def test_tap_gemm_conv_exact(fast, n64st, Ci, Co, cuda_dev, monkeypatch):
    """The three tap-addressed GEMMs of a 3x3 conv layer (forward, input
    gradient, weight gradient incl. split-K over the pixels) on small-integer
    bf16 operands, where bf16 MFMA with f32 accumulation is exact: bit-equal to
    torch's conv2d in float64 on the host, for the buffer->LDS fast path and
    the generic kernel."""
    from pytorch_end2end_speech_recognition_amd import native_ops as ops
    monkeypatch.setenv('ASR_GEMM_FAST', fast)
    monkeypatch.setenv('ASR_GEMM_N64_STAGES', n64st)   # 256 x 64 kernel: double buffer / ring
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(Ci + Co)
        B, T, F = 2, 101, 30   # M = B (T+2)(F+2) >= 4096: the 256 x 64 kernel takes N = 64
        Fn = torch.nn.functional
        x = rng.randint(-3, 4, (B, Ci, F, T)).astype(np.float64)          # NCHW, H = F, W = T
        w = rng.randint(-2, 3, (Co, Ci, 3, 3)).astype(np.float64)
        dz_valid = rng.randint(-3, 4, (B, Co, F, T)).astype(np.float64)
        xt, wt, gt = torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(dz_valid)
        z_ref = Fn.conv2d(xt, wt, padding=1)
        dx_ref = Fn.conv_transpose2d(gt, wt, padding=1)
        dw_ref = Fn.conv2d(xt.transpose(0, 1), gt.transpose(0, 1), padding=1).transpose(0, 1)

        def padded(a):   # NCHW -> [B][T+2][F+2][C]
            Bc, C = a.shape[:2]
            out = np.zeros((Bc, T + 2, F + 2, C))
            out[:, 1:T + 1, 1:F + 1] = a.transpose(0, 3, 2, 1)
            return torch.from_numpy(out.reshape(-1, C)).to(cuda_dev)

        def valid(a, C):  # [B][T+2][F+2][C] -> NCHW
            a = a.cpu().double().numpy().reshape(B, T + 2, F + 2, C)[:, 1:T + 1, 1:F + 1]
            return a.transpose(0, 3, 2, 1)

        npad = B * (T + 2) * (F + 2)
        xb = padded(x).to(torch.bfloat16)
        dzb = padded(dz_valid).to(torch.bfloat16)
        w_d = torch.from_numpy(w.astype(np.float32)).to(cuda_dev)
        wg = torch.empty(Co, 9 * Ci, dtype=torch.bfloat16, device=cuda_dev)
        wtp = torch.empty(Ci, 9 * Co, dtype=torch.bfloat16, device=cuda_dev)
        from pytorch_end2end_speech_recognition_amd import _native as N
        N.call('asr_conv_weight_pack', N.ptr(w_d), Co, Ci, 0, N.ASR_DT_BF16, N.ptr(wg),
               N.stream_handle(cuda_dev))
        N.call('asr_conv_weight_pack', N.ptr(w_d), Co, Ci, 1, N.ASR_DT_BF16, N.ptr(wtp),
               N.stream_handle(cuda_dev))
        z = torch.empty(npad, Co, device=cuda_dev)
        ops.run_gemm([ops.gemm_problem(ops._tap_operand(xb, 0, Ci, Ci, F + 2, 1),
                                       ops.operand(wg, 0, ops.rowmap(9 * Ci)), z,
                                       ops.rowmap(Co), npad, Co, 9 * Ci)], cuda_dev)
        dx = torch.empty(npad, Ci, device=cuda_dev)
        ops.run_gemm([ops.gemm_problem(ops._tap_operand(dzb, 0, Co, Co, F + 2, -1),
                                       ops.operand(wtp, 0, ops.rowmap(9 * Co)), dx,
                                       ops.rowmap(Ci), npad, Ci, 9 * Co)], cuda_dev)
        packed = torch.empty(Co, 9 * Ci, device=cuda_dev)
        ops.run_gemm([ops.gemm_problem(ops.operand(dzb, 1, ops.rowmap(Co)),
                                       ops._tap_operand(xb, 1, Ci, Ci, F + 2, 1), packed,
                                       ops.rowmap(9 * Ci), Co, 9 * Ci, npad)], cuda_dev)
        dw = torch.zeros(Co, Ci, 3, 3, device=cuda_dev)
        N.call('asr_conv_weight_unpack_acc', N.ptr(packed), Co, Ci, N.ptr(dw),
               N.stream_handle(cuda_dev))
        torch.cuda.synchronize()
        np.testing.assert_array_equal(valid(z, Co), z_ref.numpy())
        np.testing.assert_array_equal(valid(dx, Ci), dx_ref.numpy())
        np.testing.assert_array_equal(dw.cpu().double().numpy(), dw_ref.numpy())
    finally:
        ops.set_compute_dtype('fp32')


def test_oracle_vgg_decision_replay_is_exact():
    """asr_ref.vgg_front's `decisions` (the bf16 pins replay the GPU's ReLU /
    max-pool choices): replaying the oracle's own choices reproduces its
    output and gradients exactly (float64), ceil-mode windows included."""
    import torch
    from oracle import asr_ref
    torch.manual_seed(3)
    cfg = dict(conv_channels=[4, 6, 8], poolings=[[], [2, 2], [2, 2]], batch_norm=True)
    p = {}
    cin, idx = 1, 0
    for l, C in enumerate(cfg['conv_channels']):
        p['conv.layers.%d.weight' % idx] = torch.randn(C, cin, 3, 3, dtype=torch.float64) * 0.3
        p['conv.layers.%d.bias' % idx] = torch.randn(C, dtype=torch.float64) * 0.1
        idx += 2 + (1 if cfg['poolings'][l] else 0)
        p['conv.layers.%d.weight' % idx] = 1 + 0.1 * torch.randn(C, dtype=torch.float64)
        p['conv.layers.%d.bias' % idx] = 0.1 * torch.randn(C, dtype=torch.float64)
        p['conv.layers.%d.running_mean' % idx] = torch.zeros(C, dtype=torch.float64)
        p['conv.layers.%d.running_var' % idx] = torch.ones(C, dtype=torch.float64)
        idx += 2
        cin = C
    xs = torch.randn(2, 13, 9, dtype=torch.float64)          # odd T, F: ceil windows
    dec = asr_ref.vgg_decisions(p, '', cfg, xs)
    outs = []
    for d in (None, dec):
        q = {k: v.clone().requires_grad_('running' not in k) for k, v in p.items()}
        out, _, _ = asr_ref.vgg_front(q, '', cfg, xs, [13, 11], decisions=d)
        (out * torch.linspace(-1, 1, out.numel(), dtype=torch.float64).view(out.shape)).sum().backward()
        outs.append((out.detach(), {k: v.grad for k, v in q.items() if v.grad is not None}))
    assert torch.equal(outs[0][0], outs[1][0])
    for k in outs[0][1]:
        assert torch.equal(outs[0][1][k], outs[1][1][k]), k
