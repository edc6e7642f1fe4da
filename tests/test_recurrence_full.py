"""The bench's BLSTM layer op at the FULL bench shape (B = 32, H = 512,
T = 1000, ragged lengths U[800, 1000], Din = 1024 as in layers 1-4 of
ctc5x512) against the float64 oracle, for every output and gradient: y, dx,
dW_ih, dW_hh, db.  In bf16 mode this is the persistent tagged-granule
recurrence (lstm_xg.hip: lstm_fwd_xg / lstm_bwd_xg, one launch per pass, the
one-bit step tag in the LSB of one bf16 in four) plus the bf16 GEMMs.  In fp32
mode the forward is the f32 tagged-granule recurrence (lstm_fwd_xg<..., F32>,
f32 granules, H <= 512) and the backward the exact-f32 per-step kernels (the
f32 persistent backward takes H <= 384); asr_lstm_last_path records which ran,
and the test asserts it.

Why two weight regimes.  With the reference's initialisation (uniform +-0.1,
H = 512) the recurrence is chaotic: a 1e-7 perturbation grows ~x65 per 100
steps (measured on CPU: float32 vs float64 of the SAME oracle differ by 1e-7
at t = 0, 7e-6 at t = 100, 1e-2 at t = 500 and O(1) at t = 999), so no
float32 or bf16 implementation -- the reference's own CPU path included --
can match a float64 trajectory over 1000 steps.  Hence:
  * contracting recurrent weights (W_hh uniform +-0.03): errors stay bounded,
    and every output / gradient at every one of the 1000 steps is compared
    with tight bounds (this pins the kernels' indexing, every step's
    hand-off, the reverse direction's start at each utterance's own length,
    the bias-gradient sums and the weight-gradient GEMMs);
  * the reference's initialisation: the outputs of the first 48 steps of each
    direction (before the chaotic growth) against float64.
Bounds (max error / max |reference|): fp32 1e-4; bf16 2e-2 (bf16 operands of
every product, the tag bit included; measured values are printed).
"""
import numpy as np
import pytest
import torch

from oracle import asr_ref

B, T, H, DIN = 32, 1000, 512, 1024


def _case(whh_scale, seed=0):
    rng = np.random.RandomState(seed)
    lens = np.sort(rng.randint(800, T + 1, B))[::-1].astype(np.int32)
    lens[0] = T
    x = (rng.randn(B, T, DIN) * 0.5).astype(np.float32)
    for b in range(B):
        x[b, lens[b]:] = 0
    g = torch.Generator().manual_seed(seed + 1)
    w_ih = torch.rand(8 * H, DIN, generator=g) * 0.2 - 0.1
    w_hh = (torch.rand(8 * H, H, generator=g) * 2 - 1) * whh_scale
    b_ih = torch.rand(8 * H, generator=g) * 0.2 - 0.1
    b_hh = torch.rand(8 * H, generator=g) * 0.2 - 0.1
    dy = torch.from_numpy(rng.randn(B, T, 2 * H).astype(np.float32))
    for b in range(B):
        dy[b, lens[b]:] = 0
    return lens, torch.from_numpy(x), w_ih, w_hh, b_ih, b_hh, dy


def _oracle(lens, x, w_ih, w_hh, b_ih, b_hh, dy):
    """Both directions in float64 (forward rows [0, 4H), reverse [4H, 8H))."""
    torch.set_num_threads(max(1, min(16, len(__import__('os').sched_getaffinity(0)))))
    d = torch.float64
    outs = []
    for r, sl in ((False, slice(0, 4 * H)), (True, slice(4 * H, 8 * H))):
        hs = slice(0, H) if not r else slice(H, 2 * H)
        outs.append(asr_ref.lstm_direction_bptt(x.to(d), lens, w_ih[sl].to(d), w_hh[sl].to(d),
                                                b_ih[sl].to(d), b_hh[sl].to(d), r,
                                                dy[:, :, hs].to(d)))
    y = torch.cat([outs[0][0], outs[1][0]], dim=2)
    dx = outs[0][1] + outs[1][1]
    return y, dx, torch.cat([outs[0][2], outs[1][2]]), torch.cat([outs[0][3], outs[1][3]]), \
        torch.cat([outs[0][4], outs[1][4]])


def test_bptt_oracle_matches_autograd():
    rng = np.random.RandomState(1)
    Bs, Ts, Ds, Hs = 3, 17, 5, 4
    lens = np.array([17, 12, 6])
    x = torch.from_numpy(rng.randn(Bs, Ts, Ds)).requires_grad_(True)
    for b in range(Bs):
        x.data[b, lens[b]:] = 0
    ws = [torch.from_numpy(rng.randn(*s) * 0.4).requires_grad_(True)
          for s in ((4 * Hs, Ds), (4 * Hs, Hs), (4 * Hs,), (4 * Hs,))]
    dy = torch.from_numpy(rng.randn(Bs, Ts, Hs))
    for rev in (False, True):
        for t in [x] + ws:
            t.grad = None
        y = asr_ref.lstm_direction(x, lens, *ws, reverse=rev)
        (y * dy).sum().backward()
        y2, dx, dwi, dwh, db = asr_ref.lstm_direction_bptt(x.detach(), lens,
                                                           *[w.detach() for w in ws], rev, dy)
        for a, b_ in ((y2, y), (dx, x.grad), (dwi, ws[0].grad), (dwh, ws[1].grad),
                      (db, ws[2].grad), (db, ws[3].grad)):
            np.testing.assert_allclose(a.numpy(), b_.detach().numpy(), rtol=1e-10, atol=1e-12)


def _gpu(prec, lens, x, w_ih, w_hh, b_ih, b_hh, dy, dev):
    from pytorch_end2end_speech_recognition_amd import native_ops as ops
    ops.set_compute_dtype(prec)
    try:
        ws = [t.clone().to(dev).requires_grad_(True) for t in (w_ih, w_hh, b_ih, b_hh)]
        for w in ws:
            w.grad = torch.zeros_like(w)
        xd = x.to(dev).requires_grad_(True)
        lens_d = torch.from_numpy(lens).to(dev)
        y = ops.blstm_layer(xd, lens_d, T, *ws)
        y.backward(dy.to(dev))
        torch.cuda.synchronize()
        return [t.double().cpu() for t in (y.detach(), xd.grad, ws[0].grad, ws[1].grad,
                                           ws[2].grad, ws[3].grad)]
    finally:
        ops.set_compute_dtype('fp32')


def _last_path():
    import ctypes
    from pytorch_end2end_speech_recognition_amd import _native as N
    out = (ctypes.c_int * 2)()
    N.call('asr_lstm_last_path', ctypes.cast(out, ctypes.c_void_p))
    return list(out)


def _rel(a, ref):
    return float((a - ref).abs().max() / ref.abs().max())


@pytest.mark.gpu
@pytest.mark.parametrize('prec,bound,xu', [('bf16', 2e-2, '16'), ('bf16', 2e-2, '32'),
                                           ('fp32', 1e-4, '16')])
def test_full_shape_layer_vs_float64_oracle(prec, bound, xu, cuda_dev, monkeypatch):
    """xu: hidden units per work-group of the backward recurrence (32: half the
    work-groups, the default of the ctc5x512 layer's mode-3 overlap)."""
    from test_encoder_gpu import _xg_mode
    monkeypatch.setenv('ASR_XG_BWD_XU', xu)
    case = _case(0.03)
    ref = _oracle(*case)
    _xg_mode()                                   # clear
    got = _gpu(prec, *case, cuda_dev)
    path = _last_path()
    if prec == 'bf16':
        assert _xg_mode() != 0, 'the persistent tagged-granule recurrence did not run'
        # tagged-granule bf16 both passes (the forward with or without the fused
        # input projection)
        assert path[0] in (1, 3) and path[1] == 1, path
    else:
        # f32 tagged-granule forward; per-step exact-f32 backward (H = 512 > 384)
        assert path == [2, 0], path
    names = ['y', 'dx', 'dW_ih', 'dW_hh', 'db_ih', 'db_hh']
    refs = list(ref[:4]) + [ref[4], ref[4]]
    errs = {n: _rel(g, r) for n, g, r in zip(names, got, refs)}
    print('\n%s xu=%s full-shape max error / max|ref|: %s' % (
        prec, xu, ', '.join('%s %.2e' % kv for kv in errs.items())))
    for n, e in errs.items():
        assert e <= bound, (prec, n, e, bound)


@pytest.mark.gpu
def test_reference_init_early_steps_vs_float64(cuda_dev):
    """Reference initialisation (chaotic at H = 512): the first 48 outputs of
    each direction (forward t < 48; reverse the last 48 frames of each
    utterance) against float64, bf16 mode."""
    lens, x, w_ih, w_hh, b_ih, b_hh, dy = _case(0.1, seed=3)
    ref = _oracle(lens, x, w_ih, w_hh, b_ih, b_hh, dy)[0]
    y = _gpu('bf16', lens, x, w_ih, w_hh, b_ih, b_hh, dy, cuda_dev)[0]
    W = 48
    fwd = _rel(y[:, :W, :H], ref[:, :W, :H])
    rev = max(_rel(y[b, lens[b] - W:lens[b], H:], ref[b, lens[b] - W:lens[b], H:])
              for b in range(B))
    print('\nreference-init first %d steps: fwd %.2e, rev %.2e' % (W, fwd, rev))
    assert fwd <= 2e-2 and rev <= 2e-2, (fwd, rev)


def _sat_case(seed=5, Bs=16, Ts=160, Hs=256, Ds=256):
    """Saturated gates: every gate row's bias drawn +-U[3, 8] (random sign), so
    sigmoid gates sit at 0.95-0.9997 or 3e-4-0.05 and the tanh gate near +-1,
    where fp16 storage of s itself would make 1 - s coarse or zero; every 16th
    row +-25, where the f32 gate is exactly 1 / 0 / +-1."""
    rng = np.random.RandomState(seed)
    lens = np.sort(rng.randint(120, Ts + 1, Bs))[::-1].astype(np.int32)
    lens[0] = Ts
    x = (rng.randn(Bs, Ts, Ds) * 0.5).astype(np.float32)
    for b in range(Bs):
        x[b, lens[b]:] = 0
    g = torch.Generator().manual_seed(seed + 1)
    w_ih = torch.rand(8 * Hs, Ds, generator=g) * 0.2 - 0.1
    w_hh = (torch.rand(8 * Hs, Hs, generator=g) * 2 - 1) * 0.03
    mag = torch.rand(8 * Hs, generator=g) * 5 + 3
    mag[::16] = 25.0          # sigmoid == 1 / tanh == +-1 exactly in f32 (the -0 encoding)
    sign = torch.where(torch.rand(8 * Hs, generator=g) < 0.5, -1.0, 1.0)
    b_ih = mag * sign
    b_hh = torch.zeros(8 * Hs)
    dy = torch.from_numpy(rng.randn(Bs, Ts, 2 * Hs).astype(np.float32))
    for b in range(Bs):
        dy[b, lens[b]:] = 0
    return lens, torch.from_numpy(x), w_ih, w_hh, b_ih, b_hh, dy


@pytest.mark.gpu
def test_packed_gate_activations_saturated_vs_float64(cuda_dev, monkeypatch):
    """The fused bf16 forward stores the gate activations packed as fp16
    (ASR_XG_ACT_H=1, the default; enc_sig / enc_tanh in lstm_xg.hip keep 1 - s
    and 1 - g^2 at fp16's relative precision).  With saturated gates, compare
    it with the f32 activation layout (ASR_XG_ACT_H=0) and with float64: the
    bias gradient of the saturated rows -- sums of d_gate = ... * s * (1 - s)
    -- is where a plain fp16 s (spacing 4.9e-4 below 1.0) would lose 1 - s."""
    global B, T, H
    lens, x, w_ih, w_hh, b_ih, b_hh, dy = _sat_case()
    Bs, Ts, Ds = x.shape
    Hs = w_hh.shape[1]
    saved = (B, T, H)
    B, T, H = Bs, Ts, Hs
    try:
        ref = _oracle(lens, x, w_ih, w_hh, b_ih, b_hh, dy)
        res = {}
        for ah in ('1', '0'):
            monkeypatch.setenv('ASR_XG_ACT_H', ah)
            res[ah] = _gpu('bf16', lens, x, w_ih, w_hh, b_ih, b_hh, dy, cuda_dev)
    finally:
        B, T, H = saved
    names = ['y', 'dx', 'dW_ih', 'dW_hh', 'db']
    refs = list(ref[:4]) + [ref[4]]
    out = {}
    for ah, got in res.items():
        got = got[:5]
        errs = {n: float((g - r).norm() / r.norm()) for n, g, r in zip(names, got, refs)}
        # every gate row's own relative error of db (the saturated rows' sums)
        row = ((got[4] - refs[4]).abs() / refs[4].abs().clamp_min(1e-30))
        errs['db_row_median'] = float(row.median())
        out[ah] = errs
    print('\nsaturated gates, rel. L2 vs float64: ACT_H=1 %s | ACT_H=0 %s' % (out['1'], out['0']))
    for n in names:
        assert out['1'][n] <= 2e-2, ('ACT_H=1', n, out['1'][n])
        assert out['1'][n] <= 1.5 * out['0'][n] + 2e-3, (n, out['1'][n], out['0'][n])
    assert out['1']['db_row_median'] <= 1.5 * out['0']['db_row_median'] + 2e-3


@pytest.mark.gpu
@pytest.mark.parametrize('Bs,Ts,Hs,Ds', [(20, 96, 384, 128), (9, 64, 512, 64), (8, 40, 64, 32)])
def test_backward_units_per_workgroup_vs_float64(Bs, Ts, Hs, Ds, cuda_dev, monkeypatch):
    """The backward recurrence with 32 hidden units per work-group (lstm_bwd_xg
    XB = 32: 16-B sweeps of four 8-unit quarters, 8 MFMA waves over 128 gate
    rows) against float64 and against 16 units per work-group: ragged batches
    that do not fill the last 8-row group, H = 384 (M blocks past the last in
    the clamped MFMA waves), H = 512 and H = 64 (two producers per group)."""
    from test_encoder_gpu import _xg_mode
    global B, T, H
    rng = np.random.RandomState(Bs + Hs)
    lens = np.sort(rng.randint(Ts // 2, Ts + 1, Bs))[::-1].astype(np.int32)
    lens[0] = Ts
    x = (rng.randn(Bs, Ts, Ds) * 0.5).astype(np.float32)
    for b in range(Bs):
        x[b, lens[b]:] = 0
    g = torch.Generator().manual_seed(Hs)
    w_ih = torch.rand(8 * Hs, Ds, generator=g) * 0.2 - 0.1
    w_hh = (torch.rand(8 * Hs, Hs, generator=g) * 2 - 1) * 0.03
    b_ih = torch.rand(8 * Hs, generator=g) * 0.2 - 0.1
    b_hh = torch.rand(8 * Hs, generator=g) * 0.2 - 0.1
    dy = torch.from_numpy(rng.randn(Bs, Ts, 2 * Hs).astype(np.float32))
    for b in range(Bs):
        dy[b, lens[b]:] = 0
    case = (lens, torch.from_numpy(x), w_ih, w_hh, b_ih, b_hh, dy)
    saved = (B, T, H)
    B, T, H = Bs, Ts, Hs
    try:
        ref = _oracle(*case)
        res = {}
        for xu in ('16', '32'):
            monkeypatch.setenv('ASR_XG_BWD_XU', xu)
            _xg_mode()
            res[xu] = _gpu('bf16', *case, cuda_dev)
            assert _xg_mode() != 0, 'the persistent tagged-granule recurrence did not run'
    finally:
        B, T, H = saved
    names = ['y', 'dx', 'dW_ih', 'dW_hh', 'db']
    refs = list(ref[:4]) + [ref[4]]
    out = {xu: {n: float((gg - r).norm() / r.norm()) for n, gg, r in zip(names, got[:5], refs)}
           for xu, got in res.items()}
    print('\nunits per work-group, rel. L2 vs float64: 16 %s | 32 %s' % (out['16'], out['32']))
    # the forward is the same kernel either way
    assert torch.equal(res['16'][0], res['32'][0])
    for n in names:
        assert out['32'][n] <= 2e-2, (n, out['32'][n])
        assert out['32'][n] <= 1.5 * out['16'][n] + 2e-3, (n, out['32'][n], out['16'][n])
