"""Co-resident work beside the persistent backward recurrence (round 5).

Rounds 3-4 saw the backward recurrence give run-to-run different gate
gradients when other kernels' work-groups shared its CUs.  The
cause (tools/ubench/pk_hazard.hip, profiles/r05_pk_hazard.txt): on gfx950 a
packed-FP32 VALU instruction whose low lane reads src1's HIGH dword
(op_sel:[x,1]) intermittently returns 0 in lanes 48-63 while other waves'
memory traffic shares the SIMD; the fault-era build's cell math compiled to
one (`v_pk_mul_f32 v[22:23], v[22:23], v[28:29] op_sel:[0,1]`).  The library
is now built so that no such instruction exists (csrc/Makefile,
tools/isa_check.py; tests/test_native_lib.py checks the built .so).

These tests run the 5x512 encoder backward of configs[1] with co-resident work
and compare every gradient BITWISE with the same backward run alone:

  * mode 3 (the default at 5x512: 32-unit backward work-groups on 128 CUs,
    weight-gradient GEMMs on the other 128) against mode 0 (weight gradients
    on the compute stream) at the full bench shape, B 32 x T 1000;
  * mode 2 (GEMM work-groups co-resident ON the recurrence's CUs, 84 KB pin --
    the configuration that reproduced the fault) against mode 0;
  * a side stream streaming 2 x 256 MB of memory traffic (the load a
    data-parallel all-reduce puts beside the recurrence now that the compute
    stream no longer waits for collectives before it) against none.
"""
import ctypes
import os

import numpy as np
import pytest
import torch

from test_grad_buckets_gpu import _batch, _kw
from test_model_ctc import _build


def _grads(sd, batch, H, L, env, side=None):
    """Forward + backward of the CTC model on `batch`; the flat gradient
    (clone).  side(dev): called on every 'recurrence' notification, right
    after a backward recurrence was enqueued (co-resident work)."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    saved = {k: os.environ.get(k) for k in env}
    os.environ.update(env)
    try:
        m = _build(_kw(H, L))
        m.load_state_dict(sd)
        m.set_cuda()
        m.zero_grad()
        dev = torch.device('cuda', 0)
        if side is not None:
            native_ops.set_grad_ready_hook(
                lambda ev, arg=None: side(dev) if ev == 'recurrence' else None)
        try:
            native_ops.recurrence_status(dev)
            loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
            loss.backward()
            torch.cuda.synchronize()
        finally:
            native_ops.set_grad_ready_hook(None)
        assert int(native_ops.recurrence_status(dev).max()) == 0
        return loss.item(), m._flat_grad.clone()
    finally:
        for k, v in saved.items():
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v


def _setup(H, L, T):
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('bf16')
    torch.manual_seed(1623)
    sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}
    for k in sd:   # contracting recurrence: any perturbation stays visible, nothing chaotic
        if 'weight_hh' in k:
            sd[k] = sd[k] * 0.3
    return sd, _batch(T=T)


def _equal(a, b, what):
    la, ga = a
    lb, gb = b
    assert la == lb, (what, la, lb)
    d = (ga != gb).nonzero()
    assert d.numel() == 0, (what, d.numel(), float((ga - gb).abs().max()))


@pytest.mark.gpu
def test_mode3_matches_mode0_bitwise_at_ctc5x512_shape(cuda_dev):
    """configs[1] encoder at its bench shape (B 32, T 1000, 5 x 512): the default
    overlap (mode 3, 32-unit backward) against every weight gradient on the
    compute stream with the same 32-unit backward (mode 0): every gradient
    element bitwise, twice."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    sd, batch = _setup(512, 5, 1000)
    try:
        assert native_ops._overlap_plan(cuda_dev, 32, 512) == ('3', 32)
        ref = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': '0', 'ASR_XG_BWD_XU': '32'})
        for _ in range(2):
            got = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': '3'})
            _equal(ref, got, 'mode 3')
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_mode2_coresident_gemms_match_mode0_bitwise(cuda_dev):
    """GEMM work-groups on the recurrence's own CUs (mode 2, 84 KB pin, 16-unit
    backward) -- the configuration that gave wrong values in rounds 3-4 (rows
    b % 4 == 3, tools/cores_locate.py) -- against mode 0, three times."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    sd, batch = _setup(512, 5, 240)
    try:
        ref = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': '0', 'ASR_XG_BWD_XU': '16'})
        for _ in range(3):
            got = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': '2', 'ASR_XG_BWD_XU': '16'})
            _equal(ref, got, 'mode 2')
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_side_stream_memory_traffic_beside_recurrence_bitwise(cuda_dev):
    """A side stream copying 2 x 256 MB back and forth, launched right after
    each backward recurrence is enqueued (what an all-reduce bucket issued at
    the 'recurrence' notification puts beside the next recurrence), at the
    bench shape: gradients bitwise those of the run without it."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    sd, batch = _setup(512, 5, 1000)
    bufs = {}

    def traffic(dev):
        s = bufs.get('side')
        if s is None:   # private buffers; made ready once, before any traffic
            s = bufs['side'] = torch.cuda.Stream(device=dev)
            with torch.cuda.stream(s):
                bufs['a'] = torch.ones(64 << 20, device=dev)
                bufs['b'] = torch.empty_like(bufs['a'])
        # no wait on the compute stream: the copies run beside the recurrence
        # just enqueued there
        with torch.cuda.stream(s):
            for _ in range(4):
                bufs['b'].copy_(bufs['a'])
                bufs['a'].copy_(bufs['b'])
        torch.cuda.current_stream(dev).wait_stream(s)

    try:
        ref = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': 'auto'})
        got = _grads(sd, batch, 512, 5, {'ASR_OVERLAP_WGRAD': 'auto'}, side=traffic)
        _equal(ref, got, 'side traffic')
    finally:
        native_ops.set_compute_dtype('fp32')


def _held_step(sd, batch, hold_us, nwg=200):
    """One train_step of the 5x512 CTC model (bf16, the default overlap mode);
    with hold_us > 0, right before the FIRST backward recurrence is enqueued a
    side stream launches nwg work-groups that hold 96 KB of LDS each (one per
    CU) for hold_us microseconds -- a long-lived kernel (an RCCL collective
    spinning on its peer) occupying CUs while the recurrence registers its
    work-groups.  Returns (loss value, weights before and after the step,
    step stats)."""
    from pytorch_end2end_speech_recognition_amd import _native as N
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training import training_loop as TL
    dev = torch.device('cuda', 0)
    m = _build(_kw(512, 5))
    m.load_state_dict(sd)
    m.set_cuda()
    m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
    side = torch.cuda.Stream(device=dev)
    fired = []
    before = m._flat_param.clone()

    def hook(ev, arg=None):
        if ev == 'pre_recurrence' and hold_us > 0 and not fired:
            fired.append(1)
            # not joined into the compute stream: it runs beside what follows
            N.call('asr_diag_hold_cus', nwg, 96 * 1024, int(hold_us),
                   ctypes.c_void_p(side.cuda_stream))
    TL.reset_step_stats()
    native_ops.recurrence_status(dev)
    native_ops.set_grad_ready_hook(hook)
    try:
        m, lv = TL.train_step(m, batch, clip_grad_norm=5.0)
    finally:
        native_ops.set_grad_ready_hook(None)
    torch.cuda.synchronize()
    side.synchronize()
    assert fired or hold_us == 0
    return float(lv), before, m._flat_param.clone(), dict(TL.STEP_STATS)


@pytest.mark.gpu
@pytest.mark.parametrize('hold_ms', [20, 4000])
def test_held_cus_beside_recurrence_bitwise_or_visible_skip(hold_ms, cuda_dev):
    """VERDICT r05 #7 / ADVICE r05: 200 CUs held by a resident kernel when the
    backward recurrence (5 x 512, B 32, T 240) registers -- 20 ms (within the
    recurrence's bounded wait: it waits, then runs) and 4 s (beyond it: its
    registered work-groups give up).  The training step either updates the
    weights BITWISE as the step without the held CUs, or is skipped in a way
    the caller sees: loss 0, weights untouched, counted in
    STEP_STATS['recurrence_give_ups'] and ['skipped'].  Never a silent
    wrong update."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    sd, batch = _setup(512, 5, 240)
    try:
        lv0, _, w0, st0 = _held_step(sd, batch, 0)
        assert st0['skipped'] == 0 and lv0 > 0
        lv1, before, w1, st1 = _held_step(sd, batch, hold_ms * 1000)
        if st1['skipped']:
            print('\nheld %d ms: the recurrence gave up; step skipped visibly %s' % (hold_ms, st1))
            assert st1['recurrence_give_ups'] == 1 and lv1 == 0.0, st1
            assert torch.equal(w1, before)
        else:
            print('\nheld %d ms: the recurrence waited; update bitwise equal' % hold_ms)
            assert lv1 == lv0
            assert torch.equal(w1, w0)
        if hold_ms <= 20:
            assert not st1['skipped'], st1
        assert int(native_ops.recurrence_status(cuda_dev).max()) == 0
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
@pytest.mark.parametrize('sync', ['1', '0'])
@pytest.mark.parametrize('H,L,T,sub,drop', [(512, 5, 240, [], 0.0),
                                            (320, 4, 400, [False, True, True, False], 0.2)])
def test_split_input_gradient_bitwise_equals_whole(H, L, T, sub, drop, sync, cuda_dev,
                                                   monkeypatch):
    """The split input gradient (round 6, native_ops._dx_split_ok): the middle
    rows t in [T/4, 3T/4) of dX = dG W_ih computed on the side stream beside
    the last quarter of the backward recurrence (gated on the progress the
    recurrence publishes at processing step 3T/4 - 1), the outer rows after it
    -- every gradient bitwise equal to the whole product (ASR_DX_SPLIT=0, both
    without split-K slabs),
    at the 5x512 shape and at a 4x320 encoder with pyramidal subsampling and
    encoder dropout (the input maps and the dX epilogue's dropout mask), and
    the split path actually ran (its progress counter advanced); also the
    two-chunk form (ASR_DX_SPLIT=2: [T/8, T/4) and [3T/4, 7T/8) at processing
    step 7T/8 - 1 as a second side-stream product).  sync=1:
    the side stream's share also waits for the whole recurrence
    (ASR_DX_SPLIT_SYNC, diagnostics: separates the row products from the
    progress hand-off)."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    monkeypatch.setenv('ASR_DX_SPLIT_SYNC', sync)
    # the split's row products take no split-K (one launch's sum per element);
    # the whole product would take it at these test sizes (T 240 / 400), so
    # both runs go without it: the comparison is then of the same arithmetic
    monkeypatch.setenv('ASR_GEMM_NOSPLIT', '1')
    # the bottom layer's banded weight gradients report progress too: off here,
    # so the counter moves only for the split input gradient
    monkeypatch.setenv('ASR_WGRAD_SPLIT', '0')
    native_ops.set_compute_dtype('bf16')
    try:
        kw = dict(_kw(H, L), subsample_list=sub, dropout_encoder=drop)
        torch.manual_seed(1623)
        sd = {k: v.clone() for k, v in _build(kw).state_dict().items()}
        batch = _batch(T=T)
        out = {}
        for flag in ('0', '1', '2'):
            before = native_ops._progress_counter(cuda_dev)[1]
            os.environ['ASR_DX_SPLIT'] = flag
            try:
                m = _build(kw)
                m.load_state_dict(sd)
                m.set_cuda()
                m.zero_grad()
                native_ops.manual_seed(7)
                native_ops.recurrence_status(cuda_dev)
                loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
                loss.backward()
                torch.cuda.synchronize()
                assert int(native_ops.recurrence_status(cuda_dev).max()) == 0
                out[flag] = (loss.item(), m._flat_grad.clone())
            finally:
                os.environ.pop('ASR_DX_SPLIT', None)
            ran = native_ops._progress_counter(cuda_dev)[1] - before
            assert (ran > 0) == (flag != '0'), (flag, ran)
        _equal(out['0'], out['1'], 'split dX')
        _equal(out['0'], out['2'], 'split dX, two chunks')
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
@pytest.mark.parametrize('B,T,T_src,H,Dsrc,t_mul,t_add,permute', [
    (32, 240, 240, 512, 1024, 1, 0, False), (8, 100, 200, 320, 640, 2, 1, True)])
def test_split_row_problems_equal_whole_product(B, T, T_src, H, Dsrc, t_mul, t_add, permute,
                                                cuda_dev):
    """The split input gradient's three row-range products (native_ops.
    _dx_rows_problem: t in [0, T/4), [T/4, 3T/4), [3T/4, T), each with its own
    A / C row maps, K unsplit) against the whole dX = dG W_ih product on the
    same bf16 operands: bitwise, with and without the batch permutation and
    the pyramidal input map.  GEMMs only (no recurrence, no progress gate)."""
    from types import SimpleNamespace
    from pytorch_end2end_speech_recognition_amd import native_ops as ops
    from pytorch_end2end_speech_recognition_amd import _native as N
    ops.set_compute_dtype('bf16')
    g = torch.Generator(device='cpu').manual_seed(5)
    dg = torch.randn(B, T, 8 * H, generator=g).to(torch.bfloat16).to(cuda_dev)
    w = (torch.randn(8 * H, Dsrc, generator=g) * 0.05).to(torch.bfloat16).to(cuda_dev)
    perm = (torch.randperm(B, generator=g).to(torch.int32).to(cuda_dev) if permute else None)
    ctx = SimpleNamespace(drop=None)
    whole = torch.zeros(B, T_src, Dsrc, device=cuda_dev)
    c_map = ops.rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
    N.call('asr_gemm_set_nosplit', 1)
    try:
        ops.run_gemm([ops.gemm_problem(ops.operand(dg, 0, ops.rowmap(8 * H)),
                                       ops.operand(w, 1, ops.rowmap(Dsrc)), whole, c_map,
                                       B * T, Dsrc, 8 * H)], cuda_dev)
        parts = torch.zeros_like(whole)
        t0 = T // 4
        for ta, tb in ((t0, T - t0), (0, t0), (T - t0, T)):
            ops.run_gemm([ops._dx_rows_problem(dg, w, parts, ctx, B, T, T_src, H, Dsrc, Dsrc, Dsrc,
                                               perm, t_mul, t_add, ta, tb)], cuda_dev)
    finally:
        N.call('asr_gemm_set_nosplit', 0)
    torch.cuda.synchronize()
    d = (whole != parts).nonzero()
    assert d.numel() == 0, (d[:5].tolist(), float((whole - parts).abs().max()))
    assert float(whole.abs().sum()) > 0


@pytest.mark.gpu
def test_bottom_layer_banded_wgrad(cuda_dev, monkeypatch):
    """The bottom BLSTM layer's weight gradients in three time bands (round 6,
    native_ops._wgrad_split_ok): the middle band beside the last quarter of
    its own backward recurrence (mode 3 at 5x512), the outer bands after it.
    Against the single product (ASR_WGRAD_SPLIT=0): every other gradient
    bitwise, the bottom layer's W_ih / W_hh within f32 re-association of the
    three band sums; the overlap actually ran (its progress counter moved)."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('bf16')
    try:
        H, L, T = 512, 5, 240
        torch.manual_seed(1623)
        sd = {k: v.clone() for k, v in _build(_kw(H, L)).state_dict().items()}
        batch = _batch(T=T)
        out = {}
        for flag in ('0', '1'):
            monkeypatch.setenv('ASR_WGRAD_SPLIT', flag)
            before = native_ops._progress_counter(cuda_dev)[1]
            m = _build(_kw(H, L))
            m.load_state_dict(sd)
            m.set_cuda()
            m.zero_grad()
            native_ops.recurrence_status(cuda_dev)
            loss = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
            loss.backward()
            torch.cuda.synchronize()
            assert int(native_ops.recurrence_status(cuda_dev).max()) == 0
            ran = native_ops._progress_counter(cuda_dev)[1] - before
            bottom = [p for n, p in m.named_parameters() if 'weight' in n and '_l0' in n]
            out[flag] = (loss.item(), m._flat_grad.clone(), ran,
                         [p.grad.clone() for p in bottom],
                         {p.grad.data_ptr() for p in bottom})
        assert out['0'][0] == out['1'][0]
        assert out['1'][2] > out['0'][2], (out['0'][2], out['1'][2])   # + the bottom layer's report
        for a, b in zip(out['0'][3], out['1'][3]):
            assert torch.allclose(a, b, rtol=1e-5, atol=1e-6 * float(a.abs().max())), (
                float((a - b).abs().max()), float(a.abs().max()))
        # everything but the bottom layer's weight gradients: bitwise
        g0, g1 = out['0'][1].clone(), out['1'][1].clone()
        flat = m._flat_grad
        for p in [p for n, p in m.named_parameters() if 'weight' in n and '_l0' in n]:
            o = (p.grad.data_ptr() - flat.data_ptr()) // 4
            g0[o:o + p.numel()] = 0
            g1[o:o + p.numel()] = 0
        assert torch.equal(g0, g1), int((g0 != g1).sum())
    finally:
        native_ops.set_compute_dtype('fp32')
