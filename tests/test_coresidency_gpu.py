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
