"""Pipelined input gradients between stacked BLSTM layers (native_ops
_dx_pipelined): the upper layer's dX GEMMs run on a side stream in chunks of
time steps from both sequence ends inwards while the lower layer's backward
recurrence (lstm_bwd_xg) consumes them, polling one flag per chunk before it
reads the chunk's dy rows.  Against the same layers with dX computed first on
the compute stream (ASR_DX_PIPE=0): the chunked GEMMs may split K differently,
so the comparison is at f32-rounding level propagated through the bf16
recurrence (contracting weights: no chaotic growth), plus the float64 oracle
of the two-layer stack.  Reference: models/pytorch_v3/encoders/rnn.py:343-390
(stacked nn.LSTM layers with dropout between them, rnn.py:398)."""
import numpy as np
import pytest
import torch

from oracle import asr_ref


def _stack_case(B, T, H, D0, seed=0):
    rng = np.random.RandomState(seed)
    lens = np.sort(rng.randint(T // 2, T + 1, B))[::-1].astype(np.int32)
    lens[0] = T
    x = (rng.randn(B, T, D0) * 0.5).astype(np.float32)
    for b in range(B):
        x[b, lens[b]:] = 0
    g = torch.Generator().manual_seed(seed + 7)
    layers = []
    for din in (D0, 2 * H):
        layers.append([torch.rand(8 * H, din, generator=g) * 0.2 - 0.1,
                       (torch.rand(8 * H, H, generator=g) * 2 - 1) * 0.03,
                       torch.rand(8 * H, generator=g) * 0.2 - 0.1,
                       torch.rand(8 * H, generator=g) * 0.2 - 0.1])
    dy = torch.from_numpy(rng.randn(B, T, 2 * H).astype(np.float32))
    for b in range(B):
        dy[b, lens[b]:] = 0
    return lens, torch.from_numpy(x), layers, dy


def _run(case, dev, drop, monkeypatch, pipe):
    from pytorch_end2end_speech_recognition_amd import native_ops as ops
    lens, x, layers, dy = case
    T = x.shape[1]
    monkeypatch.setenv('ASR_DX_PIPE', pipe)
    ran = []
    orig = ops._dx_pipelined

    def spy(*a, **k):
        ran.append(1)
        return orig(*a, **k)

    monkeypatch.setattr(ops, '_dx_pipelined', spy)
    ops.set_compute_dtype('bf16')
    ops.recurrence_status(dev)       # clear
    try:
        ws = [[t.clone().to(dev).requires_grad_(True) for t in l] for l in layers]
        for l in ws:
            for w in l:
                w.grad = torch.zeros_like(w)
        xd = x.to(dev).requires_grad_(True)
        lens_d = torch.from_numpy(lens).to(dev)
        y0 = ops.blstm_layer(xd, lens_d, T, *ws[0], bf16_handoff=True, out_drop=drop)
        y1 = ops.blstm_layer(y0, lens_d, T, *ws[1], drop=drop, next_rec=True)
        y1.backward(dy.to(dev))
        torch.cuda.synchronize()
        st = ops.recurrence_status(dev)
        assert int(st.max().item()) == 0, 'a recurrence gave up'
        out = [y1.detach().double().cpu(), xd.grad.double().cpu()]
        out += [w.grad.double().cpu() for l in ws for w in l]
        return out, len(ran)
    finally:
        ops.set_compute_dtype('fp32')
        monkeypatch.undo()


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['1', '2'])
@pytest.mark.parametrize('B,T,H,D0,drop', [(32, 1000, 512, 80, None), (32, 1000, 512, 80, 0.2),
                                           (20, 101, 256, 40, 0.3), (9, 37, 64, 16, None)])
def test_pipelined_dx_matches_serial(B, T, H, D0, drop, mode, cuda_dev, monkeypatch):
    """mode 1: every chunk beside the recurrence; mode 2: the outer quarter
    of the rows on the compute stream before it, the middle beside it."""
    case = _stack_case(B, T, H, D0)
    d = (drop, 12345) if drop else None
    got, n_pipe = _run(case, cuda_dev, d, monkeypatch, mode)
    ref, n_ser = _run(case, cuda_dev, d, monkeypatch, '0')
    assert n_pipe == 1 and n_ser == 0, (n_pipe, n_ser)
    names = ['y', 'dx'] + ['%s%d' % (n, l) for l in range(2)
                           for n in ('dW_ih', 'dW_hh', 'db_ih', 'db_hh')]
    assert torch.equal(got[0], ref[0])          # the forward is untouched
    errs = {n: float((g - r).norm() / r.norm()) for n, g, r in zip(names, got, ref)}
    print('\npipelined vs serial dX, rel. L2: %s' % errs)
    for n, e in errs.items():
        assert e <= 2e-3, (n, e)


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['1', '2'])
def test_pipelined_stack_vs_float64(mode, cuda_dev, monkeypatch):
    """The two-layer stack with the pipelined dX against float64 (no dropout):
    every gradient within the bf16 bound of tests/test_recurrence_full."""
    B, T, H, D0 = 16, 300, 256, 64
    lens, x, layers, dy = case = _stack_case(B, T, H, D0, seed=3)
    got, n_pipe = _run(case, cuda_dev, None, monkeypatch, mode)
    assert n_pipe == 1
    torch.set_num_threads(8)
    d = torch.float64

    def layer(xin, w, dyl):
        outs = []
        for r, sl in ((False, slice(0, 4 * H)), (True, slice(4 * H, 8 * H))):
            hs = slice(0, H) if not r else slice(H, 2 * H)
            outs.append(asr_ref.lstm_direction_bptt(xin, lens, w[0][sl].to(d), w[1][sl].to(d),
                                                    w[2][sl].to(d), w[3][sl].to(d), r,
                                                    None if dyl is None else dyl[:, :, hs]))
        return outs

    # forward both layers, then backward: layer 1 with dy, layer 0 with layer 1's dx
    y0 = torch.cat([o[0] for o in layer(x.to(d), layers[0], torch.zeros(B, T, 2 * H, dtype=d))],
                   dim=2)
    o1 = layer(y0, layers[1], dy.to(d))
    y1 = torch.cat([o1[0][0], o1[1][0]], dim=2)
    dx1 = o1[0][1] + o1[1][1]
    o0 = layer(x.to(d), layers[0], dx1)
    dx0 = o0[0][1] + o0[1][1]
    refs = [y1, dx0]
    for o in (o0, o1):
        refs += [torch.cat([o[0][2], o[1][2]]), torch.cat([o[0][3], o[1][3]]),
                 torch.cat([o[0][4], o[1][4]]), torch.cat([o[0][4], o[1][4]])]
    names = ['y', 'dx', 'dW_ih0', 'dW_hh0', 'db_ih0', 'db_hh0', 'dW_ih1', 'dW_hh1', 'db_ih1',
             'db_hh1']
    errs = {n: float((g - r).abs().max() / r.abs().max()) for n, g, r in zip(names, got, refs)}
    print('\npipelined stack vs float64, max err / max|ref|: %s' % errs)
    for n, e in errs.items():
        assert e <= 2e-2, (n, e)
