"""Tap-resident 3x3 convolution (csrc/conv.hip, asr_conv3x3_tr) against the
tap-addressed GEMM it replaces in the VGG front-end (encoders/cnn.py:124-165)
and against float64 torch convolutions: small-integer bf16 operands (exact in
bf16 MFMA with f32 accumulation) bit-equal to conv2d / conv_transpose2d, and
random bf16 operands equal to the tap GEMM (same k order), for every channel
pair, both tap directions, f32 and bf16 outputs, with long chains of tiles per
work-group (ASR_CONV_TR_GRID) and the full grid."""
import numpy as np
import pytest
import torch

from pytorch_end2end_speech_recognition_amd import _native as N
from pytorch_end2end_speech_recognition_amd import native_ops as ops

pytestmark = pytest.mark.gpu


def _padded(a, T, F, dev):   # NCHW (H = F, W = T) -> [B][T+2][F+2][C]
    Bc, C = a.shape[:2]
    out = np.zeros((Bc, T + 2, F + 2, C))
    out[:, 1:T + 1, 1:F + 1] = a.transpose(0, 3, 2, 1)
    return torch.from_numpy(out.reshape(-1, C)).to(dev)


def _valid(a, B, T, F, C):   # [B][T+2][F+2][C] -> NCHW
    a = a.cpu().double().numpy().reshape(B, T + 2, F + 2, C)[:, 1:T + 1, 1:F + 1]
    return a.transpose(0, 3, 2, 1)


def _packs(w, Co, Ci, dev):
    w_d = torch.from_numpy(w.astype(np.float32)).to(dev)
    wg = torch.empty(Co, 9 * Ci, dtype=torch.bfloat16, device=dev)
    wtp = torch.empty(Ci, 9 * Co, dtype=torch.bfloat16, device=dev)
    N.call('asr_conv_weight_pack', N.ptr(w_d), Co, Ci, 0, N.ASR_DT_BF16, N.ptr(wg),
           N.stream_handle(dev))
    N.call('asr_conv_weight_pack', N.ptr(w_d), Co, Ci, 1, N.ASR_DT_BF16, N.ptr(wtp),
           N.stream_handle(dev))
    return wg, wtp


def _gemm_conv(inp, cin, fp, sign, wimg, cout, bias, out):
    npad = inp.shape[0]
    ops.run_gemm([ops.gemm_problem(ops._tap_operand(inp, 0, cin, cin, fp, sign),
                                   ops.operand(wimg, 0, ops.rowmap(9 * cin)), out,
                                   ops.rowmap(cout), npad, cout, 9 * cin, bias=bias)],
                 inp.device)


@pytest.mark.parametrize('grid', ['3', '0'])
@pytest.mark.parametrize('Ci,Co,wres', [(64, 64, '1'), (64, 64, '0'), (64, 128, '1'),
                                        (128, 64, '1'), (128, 128, '1')])
def test_conv_tr_integer_exact(Ci, Co, wres, grid, cuda_dev, monkeypatch):
    """wres '0': the 64 -> 64 layers on the weight ring instead of the resident
    weight image."""
    if grid != '0':
        monkeypatch.setenv('ASR_CONV_TR_GRID', grid)
    monkeypatch.setenv('ASR_CONV_TR_WRES', wres)
    ops.set_compute_dtype('bf16')
    try:
        assert N.query('asr_conv3x3_tr_supported', Ci, Co, 32) == 1
        rng = np.random.RandomState(Ci * 3 + Co)
        B, T, F = 2, 61, 30
        Fn = torch.nn.functional
        x = rng.randint(-3, 4, (B, Ci, F, T)).astype(np.float64)
        w = rng.randint(-2, 3, (Co, Ci, 3, 3)).astype(np.float64)
        g = rng.randint(-3, 4, (B, Co, F, T)).astype(np.float64)
        bias = rng.randint(-4, 5, Co).astype(np.float64)
        xt, wt, gt = torch.from_numpy(x), torch.from_numpy(w), torch.from_numpy(g)
        z_ref = Fn.conv2d(xt, wt, bias=torch.from_numpy(bias), padding=1).numpy()
        dx_ref = Fn.conv_transpose2d(gt, wt, padding=1).numpy()
        xb = _padded(x, T, F, cuda_dev).to(torch.bfloat16)
        gb = _padded(g, T, F, cuda_dev).to(torch.bfloat16)
        wg, wtp = _packs(w, Co, Ci, cuda_dev)
        b_d = torch.from_numpy(bias.astype(np.float32)).to(cuda_dev)
        npad = B * (T + 2) * (F + 2)
        for odt in (torch.float32, torch.bfloat16):
            z = torch.full((npad, Co), 7.0, dtype=odt, device=cuda_dev)
            ops.conv3x3_tr(xb, npad, Ci, F + 2, 1, wg, Co, b_d, z)
            dx = torch.full((npad, Ci), 7.0, dtype=odt, device=cuda_dev)
            ops.conv3x3_tr(gb, npad, Co, F + 2, -1, wtp, Ci, None, dx)
            # every padded row (halo pixels included) equals the tap GEMM's
            zg = torch.empty(npad, Co, dtype=odt, device=cuda_dev)
            _gemm_conv(xb, Ci, F + 2, 1, wg, Co, b_d, zg)
            dxg = torch.empty(npad, Ci, dtype=odt, device=cuda_dev)
            _gemm_conv(gb, Co, F + 2, -1, wtp, Ci, None, dxg)
            torch.cuda.synchronize()
            if odt == torch.float32:   # exact integers; bf16 outputs round large values
                np.testing.assert_array_equal(_valid(z, B, T, F, Co), z_ref)
                np.testing.assert_array_equal(_valid(dx, B, T, F, Ci), dx_ref)
            assert torch.equal(z, zg)
            assert torch.equal(dx, dxg)
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('Ci,Co,F', [(64, 64, 80), (64, 128, 40), (128, 64, 40), (128, 128, 40)])
def test_conv_tr_random_equals_tap_gemm(Ci, Co, F, cuda_dev):
    """The VGG geometries (F = 80 / 40 padded to 82 / 42), several tiles per
    work-group on the full grid: random bf16 operands, equal to the tap GEMM."""
    ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(Ci + Co + F)
        B, T = 4, 300 if F == 80 else 160
        npad = B * (T + 2) * (F + 2)
        xb = torch.randn(npad, Ci, device=cuda_dev).to(torch.bfloat16)
        wg = (torch.randn(Co, 9 * Ci, device=cuda_dev) * 0.05).to(torch.bfloat16)
        b_d = torch.randn(Co, device=cuda_dev)
        for sign in (1, -1):
            z = torch.empty(npad, Co, device=cuda_dev)
            ops.conv3x3_tr(xb, npad, Ci, F + 2, sign, wg, Co, b_d, z)
            zg = torch.empty(npad, Co, device=cuda_dev)
            _gemm_conv(xb, Ci, F + 2, sign, wg, Co, b_d, zg)
            torch.cuda.synchronize()
            d = (z - zg).abs().max().item()
            assert d <= 1e-5 * zg.abs().max().item(), (sign, d)
    finally:
        ops.set_compute_dtype('fp32')


def _gemm_wgrad(x, dz, cin, fp, cout):
    npad = x.shape[0]
    packed = torch.empty(cout, 9 * cin, device=x.device)
    ops.run_gemm([ops.gemm_problem(ops.operand(dz, 1, ops.rowmap(cout)),
                                   ops._tap_operand(x, 1, cin, cin, fp, 1), packed,
                                   ops.rowmap(9 * cin), cout, 9 * cin, npad)], x.device)
    return packed


@pytest.mark.parametrize('splits', ['5', '0'])
@pytest.mark.parametrize('Ci,Co', [(64, 64), (64, 128), (128, 64), (128, 128)])
def test_conv_tr_wgrad_integer_exact(Ci, Co, splits, cuda_dev, monkeypatch):
    """Weight-gradient image on small-integer operands: bit-equal to float64
    torch (conv2d of x with dz as the kernel) and to the tap GEMM's image,
    with few long pixel chunks and with the full grid."""
    if splits != '0':
        monkeypatch.setenv('ASR_CONV_TR_SPLITS', splits)
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(Ci * 7 + Co)
        B, T, F = 2, 61, 30
        Fn = torch.nn.functional
        x = rng.randint(-3, 4, (B, Ci, F, T)).astype(np.float64)
        g = rng.randint(-3, 4, (B, Co, F, T)).astype(np.float64)
        dw_ref = Fn.conv2d(torch.from_numpy(x).transpose(0, 1), torch.from_numpy(g).transpose(0, 1),
                           padding=1).transpose(0, 1).numpy()       # [Co][Ci][3][3]
        xb = _padded(x, T, F, cuda_dev).to(torch.bfloat16)
        gb = _padded(g, T, F, cuda_dev).to(torch.bfloat16)
        npad = xb.shape[0]
        packed = torch.full((Co, 9 * Ci), 7.0, device=cuda_dev)
        assert ops.conv3x3_tr_wgrad(xb, gb, npad, Ci, F + 2, Co, packed)
        dw = torch.zeros(Co, Ci, 3, 3, device=cuda_dev)
        N.call('asr_conv_weight_unpack_acc', N.ptr(packed), Co, Ci, N.ptr(dw),
               N.stream_handle(cuda_dev))
        pg = _gemm_wgrad(xb, gb, Ci, F + 2, Co)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(dw.cpu().double().numpy(), dw_ref)
        assert torch.equal(packed, pg)
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('Ci,Co,F', [(64, 64, 80), (64, 128, 40), (128, 128, 40)])
def test_conv_tr_wgrad_random_vs_tap_gemm(Ci, Co, F, cuda_dev):
    """The VGG geometries on random bf16 operands: the image agrees with the
    tap GEMM's up to f32 summation order (different pixel chunks)."""
    ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(Ci + 3 * Co + F)
        B, T = 4, 300 if F == 80 else 160
        npad = B * (T + 2) * (F + 2)
        xb = torch.randn(npad, Ci, device=cuda_dev).to(torch.bfloat16)
        gb = (torch.randn(npad, Co, device=cuda_dev) * 0.1).to(torch.bfloat16)
        packed = torch.empty(Co, 9 * Ci, device=cuda_dev)
        assert ops.conv3x3_tr_wgrad(xb, gb, npad, Ci, F + 2, Co, packed)
        pg = _gemm_wgrad(xb, gb, Ci, F + 2, Co)
        torch.cuda.synchronize()
        rel = ((packed - pg).norm() / pg.norm()).item()
        assert rel < 1e-5, rel
    finally:
        ops.set_compute_dtype('fp32')


@pytest.mark.parametrize('T,F', [(61, 30), (203, 80)])
def test_conv_c1_wgrad_xs_integer_exact(T, F, cuda_dev):
    """First-layer weight-gradient image straight from the raw features equals
    the tap GEMM's image over the 16-channel padded operand, bit for bit on
    small-integer values (channel 0 = xs, the others zero)."""
    ops.set_compute_dtype('bf16')
    try:
        rng = np.random.RandomState(T + F)
        B, Co, Cip = 3, 64, 16
        xs = rng.randint(-3, 4, (B, T, F)).astype(np.float32)
        g = rng.randint(-3, 4, (B, Co, F, T)).astype(np.float64)
        xs_d = torch.from_numpy(xs).to(cuda_dev)
        gb = _padded(g, T, F, cuda_dev).to(torch.bfloat16)
        npad = gb.shape[0]
        x_op = torch.empty(npad, Cip, dtype=torch.bfloat16, device=cuda_dev)
        N.call('asr_vgg_pad_input_ch', N.ptr(xs_d), B, T, F, Cip, N.ASR_DT_BF16, N.ptr(x_op),
               N.stream_handle(cuda_dev))
        ref = _gemm_wgrad(x_op, gb, Cip, F + 2, Co)
        packed = torch.full((Co, 9 * Cip), 7.0, device=cuda_dev)
        nb = N.query('asr_conv3x3_c1_wgrad_workspace_bytes', Co)
        ws = torch.empty(nb, dtype=torch.uint8, device=cuda_dev)
        N.call('asr_conv3x3_c1_wgrad_xs', N.ptr(xs_d), 1, B, T, F, Co, N.ptr(gb), Cip,
               N.ptr(packed), N.ptr(ws), nb, N.stream_handle(cuda_dev))
        torch.cuda.synchronize()
        assert torch.equal(packed, ref)
    finally:
        ops.set_compute_dtype('fp32')
