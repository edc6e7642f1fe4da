"""autograd wrappers over the C ABI (libasr_hip.so).

Each Function launches hand-written gfx950 kernels on torch's current stream
through ctypes; torch supplies only device memory, the stream and the autograd
tape.  No op here has a CPU path: CPU tensors raise NativeError.

Weight gradients are accumulated by the kernels directly into ``param.grad``
(views into the model's flat gradient buffer, see models/pytorch_v3/base.py);
the Functions therefore return ``None`` for weights.
"""
import ctypes
import os
import weakref

import numpy as np
import torch

from . import _native as N

F32 = N.ASR_DT_F32
BF16 = N.ASR_DT_BF16

_compute = {'dtype': F32}


def set_compute_dtype(name):
    """'fp32' (exact-f32 MFMA, parity mode) or 'bf16' (bf16 MFMA, f32 accumulate)."""
    if name not in ('fp32', 'bf16'):
        raise ValueError('compute dtype must be fp32 or bf16')
    _compute['dtype'] = BF16 if name == 'bf16' else F32


def compute_dtype():
    return _compute['dtype']


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def h2d(a, device):
    """Host array -> device tensor without blocking the host: staged through
    pinned memory (torch's caching host allocator keeps the block until the
    copy has run).  A copy from pageable memory waits for the stream to reach
    it, i.e. for the work already queued -- the host then falls behind the
    GPU and the next kernels launch into an idle queue."""
    t = torch.from_numpy(np.ascontiguousarray(a))
    if _H2D_PINNED:
        t = t.pin_memory()
    return t.to(device, non_blocking=True)


_H2D_PINNED = os.environ.get('ASR_H2D_PINNED', '1') != '0'   # (A/B: 0 = pageable copies)


# ---------------------------------------------------------------------------
# Per-step recurrence workspace arena.  Every tagged-granule launch needs its
# granule workspace zero (lstm_xg.hip); instead of one memset launch before
# each of the 2 x L layer passes of a step, the encoder forward clears one
# arena with a slot per pass (rec_arena_begin), each BLSTM forward takes a
# slot for itself and reserves one for its backward, and those launches skip
# their memset (asr_lstm_ws_prezeroed).  A slot is handed out once per
# generation; a backward whose reservation is from an older generation (the
# arena was cleared again by another forward since) takes a private workspace
# and the launch's own memset.
# ---------------------------------------------------------------------------
_arena = {'buf': None, 'gen': 0, 'off': 0, 'slot': 0}


def rec_arena_begin(dev, B, H, passes):
    """Clear the arena for `passes` recurrence launches of [B, *, H] (one fill
    on the current stream); ASR_REC_ARENA=0: off."""
    if os.environ.get('ASR_REC_ARENA', '1') == '0':
        _arena['slot'] = 0
        return
    cd = compute_dtype()
    nb = max(N.query('asr_lstm_workspace_bytes', B, H, cd, k) for k in (0, 1, 2))
    slot = (int(nb) + 255) // 256 * 256
    need = slot * int(passes)
    buf = _arena['buf']
    if buf is None or buf.device != dev or buf.numel() < need:
        buf = torch.empty(need, dtype=torch.uint8, device=dev)
    # only each slot's leading bytes must be zero (one strided fill)
    zb = min(int(N.query('asr_lstm_ws_zero_bytes', B, H)), slot)
    buf[:need].view(int(passes), slot)[:, :zb].zero_()
    _arena.update(buf=buf, gen=_arena['gen'] + 1, off=0, slot=slot)


def _arena_take(nbytes, dev):
    """(zeroed slot tensor, generation) from the current arena, or None."""
    a = _arena
    if not a['slot'] or a['buf'] is None or a['buf'].device != dev or nbytes > a['slot']:
        return None
    if a['off'] + a['slot'] > a['buf'].numel():
        return None
    t = a['buf'][a['off']:a['off'] + a['slot']]
    a['off'] += a['slot']
    return t, a['gen']


def _arena_valid(res):
    return res is not None and res[1] == _arena['gen']


class _prezeroed:
    """Tell the recurrence launch inside the block that its workspace is
    already zero (asr_lstm_ws_prezeroed), and clear the setting after it."""

    def __init__(self, on):
        self.on = bool(on)

    def __enter__(self):
        if self.on:
            N.call('asr_lstm_ws_prezeroed', 1)

    def __exit__(self, *exc):
        if self.on:
            N.call('asr_lstm_ws_prezeroed', 0)
        return False


# Gradient-ready notifications for the data-parallel bucketed all-reduce
# (utils/training/grad_buckets.py): 'recurrence' after a BLSTM layer's backward
# recurrence is enqueued, ('grads', gbufs) once its weight gradients are.
_grad_hook = [None]


def set_grad_ready_hook(fn):
    _grad_hook[0] = fn


def notify_grad_event(event, arg=None):
    fn = _grad_hook[0]
    if fn is not None:
        fn(event, arg)


def recurrence_status(device):
    """Device int32[2]: the persistent recurrences' give-up words since the
    last call (cleared), stream-ordered, no host sync."""
    st = torch.empty(2, dtype=torch.int32, device=device)
    N.call('asr_lstm_status_gather', N.ptr(st), 1, N.stream_handle(device))
    return st


class RecurrenceGaveUp(N.NativeError):
    """A persistent recurrence gave up a bounded wait: that pass's outputs are
    invalid (the pass itself can be run again)."""


def raise_if_recurrence_failed(device=None):
    """Host check (synchronises): RecurrenceGaveUp when a persistent recurrence
    gave up since the last gather (its outputs are invalid)."""
    device = device or torch.device('cuda', torch.cuda.current_device())
    st = recurrence_status(device)
    if int(st.max().item()):
        raise RecurrenceGaveUp('persistent LSTM recurrence gave up a bounded wait (status %s): '
                               'outputs of this pass are invalid' % st.tolist())


def grad_buffer(p):
    """The gradient view a kernel accumulates into (allocated on first use)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


# ---------------------------------------------------------------------------
# GEMM plumbing
# ---------------------------------------------------------------------------
def rowmap(stride_t, stride_b=0, rows_per_b=0, t_mul=1, t_add=0, t_limit=0, perm=None):
    return N.RowMap(int(stride_b), int(stride_t), int(rows_per_b), int(t_mul), int(t_add),
                    int(t_limit), perm.data_ptr() if perm is not None else None)


def operand(t, trans, rmap, offset=0):
    dt = BF16 if t.dtype == torch.bfloat16 else F32
    es = t.element_size()
    nbytes = t.untyped_storage().nbytes() - (t.storage_offset() + offset) * es
    return N.Operand(t.data_ptr() + offset * es, dt, int(trans), rmap, int(nbytes))


def gemm_problem(a, b, c, c_map, M, N_, K, alpha=1.0, beta=0.0, bias=None, bias2=None, c_offset=0,
                 batch=1, batch_strides=(0, 0, 0), drop=None):
    """drop=(p, seed): the written values get asr_dropout's mask for their
    element offsets from c (dropout's backward fused into the product)."""
    c_bf16 = c.dtype == torch.bfloat16     # bf16 C: written as bf16 (beta 0, no split-K)
    return N.Gemm(a, b, c.data_ptr() + c.element_size() * c_offset, c_map,
                  bias.data_ptr() if bias is not None else None,
                  bias2.data_ptr() if bias2 is not None else None, int(M), int(N_), int(K),
                  float(alpha), float(beta), int(batch), int(batch_strides[0]),
                  int(batch_strides[1]), int(batch_strides[2]),
                  float(drop[0]) if drop else 0.0, int(drop[1]) if drop else 0,
                  BF16 if c_bf16 else F32)


def run_gemm(problems, device, lse=None):
    """One launch of up to two products; long-K / few-tile products (weight
    gradients) get a split-K workspace from torch's caching allocator.
    lse (one product): f32 [ceil(N / 64), M, 2] tensor receiving the row
    log-sum-exp partials of the written C (asr_gemm_lse_ws)."""
    arr = (N.Gemm * len(problems))(*problems)
    parr = ctypes.cast(arr, ctypes.c_void_p)
    nb = N.query('asr_gemm_workspace_bytes', parr, len(problems))
    ws = _ws(nb, device) if nb else None
    if lse is not None:
        assert len(problems) == 1
        N.call('asr_gemm_lse_ws', parr, compute_dtype(), N.ptr(lse), N.ptr(ws), nb,
               N.stream_handle(device))
        return
    N.call('asr_gemm_ws', parr, len(problems), compute_dtype(), N.ptr(ws), nb,
           N.stream_handle(device))


def _ctc_lse_epilogue(V):
    """The CTC normaliser of a wide output layer (V > 1024) is formed in the
    head GEMM's epilogue (ASR_CTC_LSE_EPI=0: by the CTC forward's own pass
    over the logits)."""
    return V > 1024 and os.environ.get('ASR_CTC_LSE_EPI', '1') != '0'


def colsum_accumulate(g2d, out0, out1=None, alpha=1.0):
    M, Nn = g2d.shape
    nb = N.query('asr_colsum_workspace_bytes', M, Nn)
    ws = _ws(nb, g2d.device)
    N.call('asr_colsum_accumulate', N.ptr(g2d), g2d.stride(0), M, Nn, float(alpha), N.ptr(out0),
           N.ptr(out1), N.ptr(ws), nb, N.stream_handle(g2d.device))


# ---------------------------------------------------------------------------
# Linear (LinearND, linear.py:15-47): y = x W^T + b on the last dim
# ---------------------------------------------------------------------------
# bf16 mode stages f32 GEMM operands in bf16 (one conversion pass) when a
# product is at least this large, so it takes the bf16 fast / 8-wave kernels
# instead of the generic kernel converting inside its loads (the word-level CTC
# head, 8000 x 640 x 10001, ran at ~140 TF/s that way).  The padded pitches
# also put backward products whose K is the output width (the 29-class CTC
# head's dX, K = 29) on the fast kernels, so such layers are staged from
# 32 MFLOP (round 4: 250 MFLOP, the 5x512 CTC head, 32000 x 1024 x 29: -0.1
# ms/step; round 5 also the attention decoder's 29-class output layer, 4032 x
# 320 x 29, whose dX had stayed on the generic kernel); staging a layer whose
# width is already a multiple of 8 below 2 GFLOP measured slower.
_STAGE_FLOPS = 2e9
_STAGE_FLOPS_RAGGED = float(os.environ.get("ASR_LINEAR_STAGE_FLOPS", "3.2e7"))


def _staged(t, rows, cols, ld=None):
    """bf16 [rows, ld] copy of a dense f32 tensor viewed as rows x cols, the
    columns [cols, ld) zero (ld: cols rounded up to a multiple of 8 by default,
    so the copy is a legal 16-B-aligned GEMM operand)."""
    ld = (cols + 7) // 8 * 8 if ld is None else ld
    out = torch.empty(rows, ld, dtype=torch.bfloat16, device=t.device)
    N.call('asr_convert_rows_bf16_ld', N.ptr(t), rowmap(cols), int(rows), int(cols), int(ld),
           N.ptr(out), N.stream_handle(t.device))
    return out


# ---------------------------------------------------------------------------
# bf16 parameter shadow.  The fused optimizer step (optim.hip) rounds every
# updated parameter to bf16 beside its f32 write, into one shadow of the flat
# parameter buffer, so the next forward's BLSTM layers read their staged W_ih
# from it instead of converting it again (one pass over 8H x Din f32 per
# layer).  The shadow is trusted only while nothing else wrote the parameters
# since: the flat buffer's version (writes through flat views) and every
# parameter's own version (torch.optim, load_state_dict, in-place init) must be
# the ones recorded at the optimizer step.  ASR_PARAM_SHADOW=0 turns it off.
# ---------------------------------------------------------------------------
_shadows = {}   # id(flat param tensor) -> _ParamShadow (tensors compare elementwise)
SHADOW_STATS = {'hits': 0, 'linear_hits': 0}   # BLSTM / linear forwards that read the shadow


class _ParamShadow:
    __slots__ = ('flat', 'buf', 'flat_version', 'param_versions')

    def __init__(self, flat, buf):
        self.flat = weakref.ref(flat)
        self.buf = buf
        self.flat_version = None
        self.param_versions = None


def param_shadow(flat):
    """The bf16 shadow the optimizer step over `flat` should write, or None
    (fp32 mode, or switched off)."""
    if compute_dtype() != BF16 or os.environ.get('ASR_PARAM_SHADOW', '1') == '0':
        return None
    sh = _shadows.get(id(flat))
    if sh is None or sh.flat() is not flat or sh.buf.device != flat.device:
        for k in [k for k, v in _shadows.items() if v.flat() is None]:
            del _shadows[k]
        sh = _ParamShadow(flat, torch.empty(flat.numel(), dtype=torch.bfloat16,
                                            device=flat.device))
        _shadows[id(flat)] = sh
    return sh


def param_shadow_written(sh, flat, params):
    """Record the versions the shadow matches (call right after enqueueing the
    optimizer step that writes it; later writes are ordered after it and bump
    a version)."""
    sh.flat_version = flat._version
    sh.param_versions = {id(p): p._version for p in params}


def _shadow_rows(w, params):
    """bf16 view of the shadow's copy of `w` (a dense view of a flat parameter
    buffer, spanning `params`), or None when there is no current shadow."""
    if w.dtype != torch.float32 or not w.is_contiguous():
        return None
    flat = w._base
    if flat is None:
        # a module's nn.Parameter (its .data a slice of the flat buffer): the
        # flat buffer by storage
        sp = w.untyped_storage().data_ptr()
        flat = next((sh.flat() for sh in _shadows.values()
                     if sh.flat() is not None and sh.flat().untyped_storage().data_ptr() == sp),
                    None)
        if flat is None:
            return None
    sh = _shadows.get(id(flat))
    if (sh is None or sh.flat() is not flat or sh.param_versions is None or
            flat._version != sh.flat_version):
        return None
    pv = sh.param_versions
    if not params or any(pv.get(id(p)) != p._version for p in params):
        return None
    off = w.storage_offset() - flat.storage_offset()
    if off < 0 or off + w.numel() > flat.numel():
        return None
    return sh.buf[off:off + w.numel()].view(w.shape)


def _wih_bf16(w_ih, params, H, Din):
    """Staged bf16 W_ih [8H, Din] of a BLSTM layer: the optimizer's shadow
    when current, else one conversion pass."""
    w = _shadow_rows(w_ih, params)
    if w is None:
        return convert_rows_bf16(w_ih, rowmap(Din), 8 * H, Din)
    SHADOW_STATS['hits'] += 1
    return w


def _linear_stages(M, K, Nout):
    """Whether LinearND's product is staged as bf16 operands (see _STAGE_FLOPS)."""
    flops = 2.0 * M * Nout * K
    return compute_dtype() == BF16 and (
        flops >= _STAGE_FLOPS or (Nout % 8 != 0 and flops >= _STAGE_FLOPS_RAGGED))


def _linear_forward(x, weight, bias, drop, lse=None, ld=None):
    """y = dropout(x) W^T + b (f32 [..., Nout]); returns (y, xo, wo, stage):
    the GEMM operands the backward reuses (bf16 staged copies when stage).
    lse: row log-sum-exp partials of y (run_gemm).  ld: y's row pitch (>=
    Nout; y is then a strided view of [M, ld] storage)."""
    N.require_device(x, weight)
    x = x.contiguous()
    K = x.shape[-1]
    Nout = weight.shape[0]
    M = x.numel() // K
    ld = Nout if ld is None else int(ld)
    if ld == Nout:
        y = torch.empty(*x.shape[:-1], Nout, dtype=torch.float32, device=x.device)
    else:
        ybuf = torch.empty(M * ld, dtype=torch.float32, device=x.device)
        lead = tuple(x.shape[:-1])
        strides = tuple(int(np.prod(lead[i + 1:])) * ld for i in range(len(lead))) + (1,)
        y = torch.as_strided(ybuf, lead + (Nout,), strides)
    stage = _linear_stages(M, K, Nout)
    fused_drop = drop is not None and stage and K % 8 == 0
    if drop is not None and not fused_drop:        # materialise dropout(x) first
        xd = torch.empty_like(x)
        N.call('asr_dropout', N.ptr(x), N.ptr(xd), x.numel(), float(drop[0]), int(drop[1]),
               N.stream_handle(x.device))
        x = xd
    # staged copies: x [M][Kp], weight [Np][Kp] (rows Nout.. and columns K.. zero)
    Kp, Np = ((K + 7) // 8 * 8, (Nout + 7) // 8 * 8) if stage else (K, Nout)
    if stage:
        # a dense weight (no padding) from the optimizer's bf16 shadow when current
        wo = _shadow_rows(weight, (weight,)) if (Np == Nout and Kp == K) else None
        if wo is not None:
            SHADOW_STATS['linear_hits'] += 1
        elif not fused_drop and K % 8 == 0 and os.environ.get('ASR_LINEAR_MULTI', '1') != '0':
            # input, weight and zero pad rows staged in one launch (the same bits)
            xo = torch.empty(M, Kp, dtype=torch.bfloat16, device=x.device)
            wo = torch.empty(Np, Kp, dtype=torch.bfloat16, device=x.device)
            jobs = [(x, rowmap(K), M, K, xo.data_ptr()), (weight, rowmap(K), Nout, K, wo.data_ptr())]
            if Np > Nout:
                jobs.append((weight, rowmap(0, t_limit=1, rows_per_b=Np - Nout, t_add=1),
                             Np - Nout, Kp, wo.data_ptr() + Nout * Kp * 2))
            if M > 0 and _convert_multi(jobs, x.device):
                return _linear_gemm(xo, wo, y, ld, M, Nout, Kp, bias, lse, x.device) + (stage,)
        # fused_drop: K % 8 == 0, so Kp == K and the dropped copy is the operand
        xo = (convert_rows_bf16(x, rowmap(K), M, K, drop=drop) if fused_drop else
              _staged(x, M, K, Kp))
        if wo is None:
            wo = torch.empty(Np, Kp, dtype=torch.bfloat16, device=x.device)
            N.call('asr_convert_rows_bf16_ld', N.ptr(weight), rowmap(K), Nout, K, Kp, N.ptr(wo),
                   N.stream_handle(x.device))
            if Np > Nout:
                N.call('asr_convert_rows_bf16_ld', N.ptr(weight), rowmap(0, t_limit=1,
                       rows_per_b=Np - Nout, t_add=1), Np - Nout, Kp, Kp,
                       ctypes.c_void_p(wo.data_ptr() + Nout * Kp * 2), N.stream_handle(x.device))
    else:
        xo, wo = x, weight
    return _linear_gemm(xo, wo, y, ld, M, Nout, Kp, bias, lse, x.device) + (stage,)


def _linear_gemm(xo, wo, y, ld, M, Nout, Kp, bias, lse, dev):
    if M > 0:
        p = gemm_problem(operand(xo, 0, rowmap(Kp)), operand(wo, 0, rowmap(Kp)), y,
                         rowmap(ld), M, Nout, Kp, bias=bias)
        run_gemm([p], dev, lse=lse)
    return y, xo, wo


def _convert_multi(jobs, dev):
    """jobs: (src tensor, RowMap, rows, cols, dst address) -- asr_convert_rows_bf16
    of each in one launch; False when a job does not qualify (nothing launched)."""
    n = len(jobs)
    src = (ctypes.c_void_p * n)(*[j[0].data_ptr() for j in jobs])
    maps = (N.RowMap * n)(*[j[1] for j in jobs])
    rows = (ctypes.c_int * n)(*[int(j[2]) for j in jobs])
    cols = (ctypes.c_int * n)(*[int(j[3]) for j in jobs])
    dst = (ctypes.c_void_p * n)(*[j[4] for j in jobs])
    rc = N.lib().asr_convert_rows_bf16_multi(n, src, maps, rows, cols, dst,
                                              N.stream_handle(dev))
    if rc < 0:
        raise N.NativeError('asr_convert_rows_bf16_multi: launch failed')
    return rc == 1


def _linear_backward(xo, wo, bias, stage, xshape, weight, drop, dyo, need_dx, dy_bias=None,
                     wgrad=True):
    """dX and dW (+ db) of _linear_forward from dyo: the f32 dY, or with stage
    its bf16 copy [M][Np] whose columns Nout.. are zero (they meet W's zero
    rows).  dy_bias: the tensor the bias gradient is summed from (f32 [M,
    Nout] or the bf16 dyo).  wgrad=False: dX only (_linear_wgrad elsewhere)."""
    K = xshape[-1]
    Nout = weight.shape[0]
    M = int(np.prod(xshape[:-1]))
    dev = dyo.device
    Kp, Np = (xo.shape[-1], wo.shape[0]) if stage else (K, Nout)
    dx = None
    probs = []
    if need_dx:
        dx = torch.empty(xshape, dtype=torch.float32, device=dev)
        probs.append(gemm_problem(operand(dyo, 0, rowmap(Np)), operand(wo, 1, rowmap(Kp)),
                                  dx, rowmap(K), M, K, Np, drop=drop))
    if not wgrad:
        if probs:
            run_gemm(probs, dev)
        return dx
    gw = grad_buffer(weight)
    probs.append(gemm_problem(operand(dyo, 1, rowmap(Np)), operand(xo, 1, rowmap(Kp)), gw,
                              rowmap(K), Nout, K, M, beta=1.0))
    run_gemm(probs, dev)
    _linear_bias_grad(bias, dy_bias, M, Nout, dev)
    return dx


def _linear_wgrad(xo, wo, bias, stage, xshape, weight, dyo, dy_bias=None):
    """dW (+ db) of _linear_backward alone."""
    K = xshape[-1]
    Nout = weight.shape[0]
    M = int(np.prod(xshape[:-1]))
    dev = dyo.device
    Kp, Np = (xo.shape[-1], wo.shape[0]) if stage else (K, Nout)
    run_gemm([gemm_problem(operand(dyo, 1, rowmap(Np)), operand(xo, 1, rowmap(Kp)),
                           grad_buffer(weight), rowmap(K), Nout, K, M, beta=1.0)], dev)
    _linear_bias_grad(bias, dy_bias, M, Nout, dev)


def _linear_bias_grad(bias, dy_bias, M, Nout, dev):
    if bias is not None:
        if dy_bias.dtype == torch.bfloat16:
            nb = N.query('asr_colsum_workspace_bytes', M, Nout)
            ws = _ws(nb, dev)
            N.call('asr_colsum_accumulate_bf16', N.ptr(dy_bias), dy_bias.shape[-1], M, Nout, 1.0,
                   N.ptr(grad_buffer(bias)), None, N.ptr(ws), nb, N.stream_handle(dev))
        else:
            colsum_accumulate(dy_bias.view(M, Nout), grad_buffer(bias))


def _wgrad_beside(dev, plan, fn, keep, gbufs):
    """Enqueue the weight-gradient work fn() on the weight-gradient side stream
    of the recurrence shape plan = (B, H), gated on the next backward
    recurrence (as a BLSTM layer's own weight gradients); keep: tensors the
    side stream reads.  False when that shape runs weight gradients on the
    compute stream (the caller then runs fn itself)."""
    side_ent = _wgrad_side_stream(dev, *plan)
    if side_ent is None:
        return False
    side, small, gated = side_ent
    main = torch.cuda.current_stream(dev)
    side.wait_stream(main)
    if small:
        N.call('asr_gemm_set_small_tiles', 1)
    try:
        with torch.cuda.stream(side):
            if gated:
                N.call('asr_lstm_wgrad_gate', N.stream_handle(dev))
            fn()
    finally:
        if small:
            N.call('asr_gemm_set_small_tiles', 0)
    for t in keep:
        t.record_stream(side)
    if not _side_pending:
        torch.autograd.Variable._execution_engine.queue_callback(
            lambda: _join_side_wgrads(dev, notify=False))
    _side_pending.append((side, gbufs, main))
    return True


# (B, H) of the encoder recurrence whose backward follows, while the decoder-side
# linear layers of an attention model are built (wgrad_beside_encoder): their
# weight gradients then run beside that recurrence instead of before it
_beside_plan = [None]


class wgrad_beside_encoder(object):
    def __init__(self, B, H):
        self.plan = (int(B), int(H))

    def __enter__(self):
        self.prev = _beside_plan[0]
        if os.environ.get('ASR_DEC_WGRAD_SIDE', '1') != '0':
            _beside_plan[0] = self.plan
        return self

    def __exit__(self, *a):
        _beside_plan[0] = self.prev
        return False


class LinearFn(torch.autograd.Function):
    """y = dropout(x) W^T + b.  drop=(p, seed): dropout of the INPUT with
    asr_dropout's mask, folded into the bf16 staging of x (forward) and the dX
    GEMM's epilogue (backward) when the product is staged; otherwise applied
    as a separate pass first."""

    @staticmethod
    def forward(ctx, x, weight, bias, drop=None):
        y, xo, wo, stage = _linear_forward(x, weight, bias, drop)
        ctx.save_for_backward(xo, wo)
        ctx.meta = (bias, stage, tuple(x.shape), weight)
        ctx.drop = drop
        ctx.beside = _beside_plan[0]
        return y

    @staticmethod
    def backward(ctx, dy):
        xo, wo = ctx.saved_tensors
        bias, stage, xshape, weight = ctx.meta
        dy = dy.contiguous()
        Nout = weight.shape[0]
        M = dy.numel() // Nout
        if M == 0:
            return torch.zeros(xshape, dtype=torch.float32, device=dy.device), None, None, None
        Np = wo.shape[0] if stage else Nout
        dyo = _staged(dy, M, Nout, Np) if stage else dy   # zero columns meet zero W rows
        # dropout's backward = its mask, applied by the dX epilogue
        if ctx.beside is not None:
            dx = _linear_backward(xo, wo, bias, stage, xshape, weight, ctx.drop, dyo,
                                  ctx.needs_input_grad[0], dy_bias=dy, wgrad=False)
            gb = (grad_buffer(weight),) + ((grad_buffer(bias),) if bias is not None else ())
            if not _wgrad_beside(dy.device, ctx.beside,
                                 lambda: _linear_wgrad(xo, wo, bias, stage, xshape, weight, dyo,
                                                       dy_bias=dy),
                                 (xo, wo, dyo, dy), gb):
                _linear_wgrad(xo, wo, bias, stage, xshape, weight, dyo, dy_bias=dy)
            return dx, None, None, None
        dx = _linear_backward(xo, wo, bias, stage, xshape, weight, ctx.drop, dyo,
                              ctx.needs_input_grad[0], dy_bias=dy)
        return dx, None, None, None


def _ctc_forward(logits, st, sb, T, B, V, lse, labels_flat, label_lens, act_lens, max_label_len,
                 blank, zero_infinity, costs, loss, loss_scale, ws, nbytes):
    """asr_ctc_forward, or asr_ctc_forward_lse from the head GEMM's partials."""
    common = (N.ptr(labels_flat), N.ptr(label_lens), N.ptr(act_lens), int(max_label_len),
              int(blank), int(bool(zero_infinity)), N.ptr(costs), N.ptr(loss), float(loss_scale),
              N.ptr(ws), nbytes, N.stream_handle(logits.device))
    if lse is not None:
        N.call('asr_ctc_forward_lse', N.ptr(logits), st, sb, T, B, V, N.ptr(lse), lse.shape[0],
               *common)
    else:
        N.call('asr_ctc_forward', N.ptr(logits), st, sb, T, B, V, *common)


class LinearCTCFn(torch.autograd.Function):
    """The CTC output layer and its loss as ONE op (LinearND + CTC: ctc.py:30-52
    with linear.py:32-47), for heads whose product is staged in bf16.
    Forward: the staged GEMM writes the f32 logits [B, T, V] (bias fused),
    then the CTC forward (emissions + lattices) reads them.  Backward: the CTC
    gradient is written straight into the bf16 dY operand of the two GEMMs --
    rows of Np = V rounded up to 8 columns, the padding zero
    (asr_ctc_backward_bf16) -- so the f32 d logits is never written and never
    restaged (at the 10001-word head of configs[4]: 320 MB written + 480 MB
    staging traffic per call saved).  The bias gradient is summed in f32 by
    the same pass before the rounding (asr_ctc_backward_bf16_db: per-block
    column partials, then a fixed-order sum).  dX and dW equal
    ctc_loss(linear(...))'s up to the bf16 rounding of dY the staged product
    applies anyway; the bias gradient equals the f32 column sum up to
    summation order."""

    @staticmethod
    def forward(ctx, x, weight, bias, drop, labels_flat, label_lens, act_lens, max_label_len,
                loss_scale, blank, zero_infinity):
        N.require_device(labels_flat, label_lens, act_lens)
        V = weight.shape[0]
        M = x.numel() // x.shape[-1]
        lse = (torch.empty((V + 63) // 64, M, 2, dtype=torch.float32, device=x.device)
               if _ctc_lse_epilogue(V) and M > 0 else None)
        # wide heads: logits pitch V rounded up to 4 columns, so the gradient
        # pass reads 16-B aligned rows (ctc_grad_bf16's aligned form; a narrow
        # head keeps the dense layout, whose values the unfused ops reproduce
        # bit for bit)
        logits, xo, wo, stage = _linear_forward(x, weight, bias, drop, lse=lse,
                                                ld=(V + 3) // 4 * 4 if V > 1024 else V)
        assert stage, 'LinearCTCFn needs a staged (bf16) output layer'
        B, T, V = logits.shape
        nbytes = N.query('asr_ctc_workspace_bytes', T, B, V, max_label_len)
        ws = _ws(nbytes, logits.device)
        costs = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty(1, dtype=torch.float32, device=logits.device)
        _ctc_forward(logits, logits.stride(1), logits.stride(0), T, B, V, lse, labels_flat,
                     label_lens, act_lens, max_label_len, blank, zero_infinity, costs, loss,
                     loss_scale, ws, nbytes)
        ctx.save_for_backward(xo, wo, logits, labels_flat, label_lens, act_lens, ws)
        ctx.meta = (bias, tuple(x.shape), weight, int(max_label_len), int(blank),
                    float(loss_scale), nbytes)
        # produced by a BLSTM layer (through at most a few views / permutes):
        # its backward recurrence is the next one the gate can wait for
        ctx.from_blstm = _produced_by_blstm(x)
        ctx.drop = drop
        ctx.mark_non_differentiable(costs)
        return loss, costs

    @staticmethod
    def backward(ctx, g_loss, g_costs):
        xo, wo, logits, labels_flat, label_lens, act_lens, ws = ctx.saved_tensors
        bias, xshape, weight, max_label_len, blank, loss_scale, nbytes = ctx.meta
        B, T, V = logits.shape
        Np = wo.shape[0]
        dev = logits.device
        dyo = torch.empty(B * T, Np, dtype=torch.bfloat16, device=dev)
        g = g_loss.contiguous() if g_loss is not None else None
        args = (N.ptr(logits), logits.stride(1), logits.stride(0), T, B, V, N.ptr(labels_flat),
                N.ptr(label_lens),
                N.ptr(act_lens), max_label_len, blank, N.ptr(g),
                loss_scale if g is not None else 0.0, N.ptr(dyo), Np, T * Np, Np, N.ptr(ws), nbytes)
        # the bias gradient: f32 column sums formed inside the gradient pass before
        # the bf16 rounding (ASR_CTC_HEAD_DB=0: column sums of the rounded dY)
        bws = None
        if bias is not None and V <= 16384 and os.environ.get('ASR_CTC_HEAD_DB', '1') != '0':
            bnb = N.query('asr_ctc_bias_workspace_bytes', T, B, V, Np)
            bws = _ws(bnb, dev)
            N.call('asr_ctc_backward_bf16_db', *args, N.ptr(grad_buffer(bias)), N.ptr(bws), bnb,
                   N.stream_handle(dev))
        else:
            N.call('asr_ctc_backward_bf16', *args, N.stream_handle(dev))
        bias_w = None if bws is not None else bias   # bias gradient still to be summed from dY
        if ctx.from_blstm is not None and os.environ.get('ASR_HEAD_WGRAD_SIDE', '1') != '0':
            # the head's weight gradient (only the optimizer needs it) beside the
            # top BLSTM layer's backward recurrence, as that layer's own weight
            # gradients run beside the next one: dX alone on the compute stream
            dx = _linear_backward(xo, wo, bias_w, True, xshape, weight, ctx.drop, dyo,
                                  ctx.needs_input_grad[0], dy_bias=dyo, wgrad=False)
            gb = (grad_buffer(weight),) + ((grad_buffer(bias),) if bias is not None else ())
            if not _wgrad_beside(dev, ctx.from_blstm,
                                 lambda: _linear_wgrad(xo, wo, bias_w, True, xshape, weight, dyo,
                                                       dy_bias=dyo),
                                 (xo, wo, dyo), gb):
                _linear_wgrad(xo, wo, bias_w, True, xshape, weight, dyo, dy_bias=dyo)
            return (dx,) + (None,) * 10
        dx = _linear_backward(xo, wo, bias_w, True, xshape, weight, ctx.drop, dyo,
                              ctx.needs_input_grad[0], dy_bias=dyo)
        return (dx,) + (None,) * 10


class LinearCTC32Fn(torch.autograd.Function):
    """The CTC output layer and its loss as one op at reference precision (fp32
    mode; LinearND + CTC, ctc.py:30-52 with linear.py:32-47): the logits are
    written with a row pitch of V rounded up to 4 columns, and the CTC
    gradient with the same pitch, so the three products (logits, dX, dW) get
    16-B aligned rows and run on the f32 fast kernel (gemm_f32_fast) instead of
    the generic one (an unpadded 10001-column row is not 16-B aligned; the
    fast kernel zero-fills the k tail of the dX product in LDS).  Values equal
    ctc_loss(linear(...))'s up to the summation order of the products."""

    @staticmethod
    def forward(ctx, x, weight, bias, drop, labels_flat, label_lens, act_lens, max_label_len,
                loss_scale, blank, zero_infinity):
        N.require_device(x, weight, labels_flat, label_lens, act_lens)
        # the producing BLSTM layer is found from the ORIGINAL input: the
        # contiguous copy and the materialised dropout below carry no grad_fn
        ctx.from_blstm = _produced_by_blstm(x)
        x = x.contiguous()
        B, T, K = x.shape
        V = weight.shape[0]
        Vp = (V + 3) // 4 * 4
        dev = x.device
        if drop is not None:   # materialise dropout(x); the dX epilogue applies the mask
            xd = torch.empty_like(x)
            N.call('asr_dropout', N.ptr(x), N.ptr(xd), x.numel(), float(drop[0]), int(drop[1]),
                   N.stream_handle(dev))
            x = xd
        logits = torch.empty(B * T, Vp, dtype=torch.float32, device=dev)
        lse = (torch.empty((V + 63) // 64, B * T, 2, dtype=torch.float32, device=dev)
               if _ctc_lse_epilogue(V) and B * T > 0 else None)
        if B * T > 0:
            run_gemm([gemm_problem(operand(x, 0, rowmap(K)), operand(weight, 0, rowmap(K)),
                                   logits, rowmap(Vp), B * T, V, K, bias=bias)], dev, lse=lse)
        nbytes = N.query('asr_ctc_workspace_bytes', T, B, V, max_label_len)
        ws = _ws(nbytes, dev)
        costs = torch.empty(B, dtype=torch.float32, device=dev)
        loss = torch.empty(1, dtype=torch.float32, device=dev)
        _ctc_forward(logits, Vp, T * Vp, T, B, V, lse, labels_flat, label_lens, act_lens,
                     max_label_len, blank, zero_infinity, costs, loss, loss_scale, ws, nbytes)
        ctx.save_for_backward(x, logits, labels_flat, label_lens, act_lens, ws)
        ctx.meta = (bias, weight, B, T, V, Vp, int(max_label_len), int(blank), float(loss_scale),
                    nbytes)
        ctx.drop = drop
        ctx.mark_non_differentiable(costs)
        return loss, costs

    @staticmethod
    def backward(ctx, g_loss, g_costs):
        x, logits, labels_flat, label_lens, act_lens, ws = ctx.saved_tensors
        bias, weight, B, T, V, Vp, max_label_len, blank, loss_scale, nbytes = ctx.meta
        dev = logits.device
        K = x.shape[-1]
        M = B * T
        dl = torch.empty(M, Vp, dtype=torch.float32, device=dev)
        g = g_loss.contiguous() if g_loss is not None else None
        N.call('asr_ctc_backward', N.ptr(logits), Vp, T * Vp, T, B, V, N.ptr(labels_flat),
               N.ptr(label_lens), N.ptr(act_lens), max_label_len, blank, N.ptr(g),
               loss_scale if g is not None else 0.0, N.ptr(dl), Vp, T * Vp, N.ptr(ws), nbytes,
               N.stream_handle(dev))
        dx = None
        if ctx.needs_input_grad[0]:
            dx = torch.empty(B, T, K, dtype=torch.float32, device=dev)
            if M > 0:
                run_gemm([gemm_problem(operand(dl, 0, rowmap(Vp)), operand(weight, 1, rowmap(K)),
                                       dx, rowmap(K), M, K, V, drop=ctx.drop)], dev)

        def wgrad():
            if M > 0:
                run_gemm([gemm_problem(operand(dl, 1, rowmap(Vp)), operand(x, 1, rowmap(K)),
                                       grad_buffer(weight), rowmap(K), V, K, M, beta=1.0)], dev)
            if bias is not None:
                colsum_accumulate(dl[:, :V], grad_buffer(bias))
        gb = (grad_buffer(weight),) + ((grad_buffer(bias),) if bias is not None else ())
        if not (ctx.from_blstm is not None and os.environ.get('ASR_HEAD_WGRAD_SIDE', '1') != '0'
                and _wgrad_beside(dev, ctx.from_blstm, wgrad, (x, dl), gb)):
            wgrad()
        return (dx,) + (None,) * 10


def _produced_by_blstm(t, depth=4):
    """(B, H) of the BLSTMLayerFn whose output t derives from within `depth`
    autograd hops (views, permutes, fc layers), else None: its backward
    recurrence is the one a gated side stream waits for, so the overlap plan
    is built from ITS shape, not from t's width."""
    frontier = [t.grad_fn] if t.grad_fn is not None else []
    for _ in range(depth):
        nxt = []
        for fn in frontier:
            if fn is None:
                continue
            if type(fn).__name__.startswith('BLSTMLayerFn'):
                return getattr(fn, 'bh', None)
            nxt.extend(f for f, _ in getattr(fn, 'next_functions', ()))
        frontier = nxt
    return None


def linear_ctc_loss(x, weight, bias, labels_flat, label_lens, act_lens, max_label_len,
                    loss_scale=1.0, drop=None, blank=0, zero_infinity=True):
    """ctc_loss(linear(x, weight, bias, drop), ...) -> (loss [1], costs [B]);
    one fused op: LinearCTCFn when the output layer is staged in bf16,
    LinearCTC32Fn in fp32 mode (ASR_CTC_HEAD_FUSED=0 keeps the two ops)."""
    K = x.shape[-1]
    fused = os.environ.get('ASR_CTC_HEAD_FUSED', '1') != '0'
    if x.dim() == 3 and _linear_stages(x.numel() // K, K, weight.shape[0]) and fused:
        return LinearCTCFn.apply(x, weight, bias, drop, labels_flat, label_lens, act_lens,
                                 max_label_len, loss_scale, blank, zero_infinity)
    if x.dim() == 3 and compute_dtype() == F32 and fused:
        return LinearCTC32Fn.apply(x, weight, bias, drop, labels_flat, label_lens, act_lens,
                                   max_label_len, loss_scale, blank, zero_infinity)
    return ctc_loss(linear(x, weight, bias, drop), labels_flat, label_lens, act_lens,
                    max_label_len, loss_scale, blank, zero_infinity)


def linear(x, weight, bias=None, drop=None):
    """drop=(p, seed): y = dropout(x) W^T + b with dropout folded into the
    product (LinearFn)."""
    return LinearFn.apply(x, weight, bias, drop)


class LinearExFn(torch.autograd.Function):
    """y = x @ W[:, c0:c0+K]^T + b + b2, with x rows optionally gathered from a
    3-D tensor at a fixed time index (x_src[b, t_index, :]).  Covers the
    decoder-input projection of all steps (columns [0, emb) of the LSTMCell
    W_ih plus both biases) and the init_dec_state 'first' / 'final' rows."""

    @staticmethod
    def forward(ctx, x, weight, bias, bias2, c0, K, t_index):
        N.require_device(x, weight)
        x = x.contiguous()
        ldw = weight.shape[1]
        Nout = weight.shape[0]
        if t_index is None:
            M = x.numel() // K
            amap = rowmap(K)
            out_shape = tuple(x.shape[:-1]) + (Nout,)
            a_off = 0
        else:
            B, T, _ = x.shape
            M = B
            amap = rowmap(T * K)
            out_shape = (B, Nout)
            a_off = t_index * K
        y = torch.empty(out_shape, dtype=torch.float32, device=x.device)
        p = gemm_problem(operand(x, 0, amap, offset=a_off), operand(weight, 0, rowmap(ldw), offset=c0),
                         y, rowmap(Nout), M, Nout, K, bias=bias, bias2=bias2)
        run_gemm([p], x.device)
        ctx.save_for_backward(x, weight)
        ctx.meta = (bias, bias2, c0, K, t_index, M, amap, a_off)
        ctx.beside = _beside_plan[0]
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        bias, bias2, c0, K, t_index, M, amap, a_off = ctx.meta
        dy = dy.contiguous()
        ldw, Nout = weight.shape[1], weight.shape[0]
        dx = None
        probs = []
        if ctx.needs_input_grad[0]:
            dx = torch.zeros_like(x) if t_index is not None else torch.empty_like(x)
            probs.append(gemm_problem(operand(dy, 0, rowmap(Nout)),
                                      operand(weight, 1, rowmap(ldw), offset=c0), dx, amap, M, K,
                                      Nout, c_offset=a_off))

        def wgrad():
            run_gemm([gemm_problem(operand(dy, 1, rowmap(Nout)), operand(x, 1, amap, offset=a_off),
                                   grad_buffer(weight), rowmap(ldw), Nout, K, M, beta=1.0,
                                   c_offset=c0)], x.device)
            if bias is not None:
                colsum_accumulate(dy.view(M, Nout), grad_buffer(bias),
                                  grad_buffer(bias2) if bias2 is not None else None)

        if ctx.beside is not None:
            # the weight / bias gradients beside the encoder's top backward
            # recurrence (as LinearFn's), only dX on the compute stream
            if probs:
                run_gemm(probs, x.device)
            gb = tuple(grad_buffer(t) for t in (weight, bias, bias2) if t is not None)
            if not _wgrad_beside(dy.device, ctx.beside, wgrad, (x, dy), gb):
                wgrad()
            return dx, None, None, None, None, None, None
        probs.append(gemm_problem(operand(dy, 1, rowmap(Nout)), operand(x, 1, amap, offset=a_off),
                                  grad_buffer(weight), rowmap(ldw), Nout, K, M, beta=1.0,
                                  c_offset=c0))
        run_gemm(probs, x.device)
        if bias is not None:
            colsum_accumulate(dy.view(M, Nout), grad_buffer(bias),
                              grad_buffer(bias2) if bias2 is not None else None)
        return dx, None, None, None, None, None, None


def linear_ex(x, weight, bias=None, bias2=None, c0=0, K=None, t_index=None):
    K = weight.shape[1] - c0 if K is None else K
    return LinearExFn.apply(x, weight, bias, bias2, c0, K, t_index)


class MeanTimeFn(torch.autograd.Function):
    """out[b] = mean_t x[b, t, :] over all T frames of [B, T, E] (padding
    included, as enc_out.mean(dim=1) in attention_seq2seq.py:832), as one
    batched GEMM ones(1 x T) . x[b] / T; backward dx[b, t] = dout[b] / T is the
    batched K = 1 product ones(T x 1) . dout[b] / T."""

    @staticmethod
    def forward(ctx, x):
        N.require_device(x)
        x = x.contiguous()
        B, T, E = x.shape
        ones = torch.ones(T, dtype=torch.float32, device=x.device)
        out = torch.empty(B, E, dtype=torch.float32, device=x.device)
        run_gemm([gemm_problem(operand(ones, 0, rowmap(T)), operand(x, 1, rowmap(E)), out,
                               rowmap(E), 1, E, T, alpha=1.0 / T, batch=B,
                               batch_strides=(0, T * E, E))], x.device)
        ctx.shape = (B, T, E)
        return out

    @staticmethod
    def backward(ctx, dout):
        B, T, E = ctx.shape
        dout = dout.contiguous()
        ones = torch.ones(T, dtype=torch.float32, device=dout.device)
        dx = torch.empty(B, T, E, dtype=torch.float32, device=dout.device)
        run_gemm([gemm_problem(operand(ones, 0, rowmap(1)), operand(dout, 1, rowmap(E)), dx,
                               rowmap(E), T, E, 1, alpha=1.0 / T, batch=B,
                               batch_strides=(0, E, T * E))], dout.device)
        return dx


def mean_time(x):
    return MeanTimeFn.apply(x)


class Linear2Fn(torch.autograd.Function):
    """y = x1 W1^T + b1 + x2 W2^T + b2 (the attention bottleneck
    W_d(dec_out) + W_c(context), attention_seq2seq.py:788-790): two GEMMs into
    one output, no elementwise add pass."""

    @staticmethod
    def forward(ctx, x1, w1, b1, x2, w2, b2):
        N.require_device(x1, w1, x2, w2)
        x1, x2 = x1.contiguous(), x2.contiguous()
        K1, K2, Nout = x1.shape[-1], x2.shape[-1], w1.shape[0]
        M = x1.numel() // K1
        y = torch.empty(*x1.shape[:-1], Nout, dtype=torch.float32, device=x1.device)
        run_gemm([gemm_problem(operand(x1, 0, rowmap(K1)), operand(w1, 0, rowmap(K1)), y,
                               rowmap(Nout), M, Nout, K1, bias=b1, bias2=b2)], x1.device)
        run_gemm([gemm_problem(operand(x2, 0, rowmap(K2)), operand(w2, 0, rowmap(K2)), y,
                               rowmap(Nout), M, Nout, K2, beta=1.0)], x1.device)
        ctx.save_for_backward(x1, w1, x2, w2)
        ctx.biases = (b1, b2)
        return y

    @staticmethod
    def backward(ctx, dy):
        x1, w1, x2, w2 = ctx.saved_tensors
        b1, b2 = ctx.biases
        dy = dy.contiguous()
        K1, K2, Nout = x1.shape[-1], x2.shape[-1], w1.shape[0]
        M = x1.numel() // K1
        dx1, dx2 = torch.empty_like(x1), torch.empty_like(x2)
        run_gemm([gemm_problem(operand(dy, 0, rowmap(Nout)), operand(w1, 1, rowmap(K1)), dx1,
                               rowmap(K1), M, K1, Nout),
                  gemm_problem(operand(dy, 0, rowmap(Nout)), operand(w2, 1, rowmap(K2)), dx2,
                               rowmap(K2), M, K2, Nout)], x1.device)
        run_gemm([gemm_problem(operand(dy, 1, rowmap(Nout)), operand(x1, 1, rowmap(K1)),
                               grad_buffer(w1), rowmap(K1), Nout, K1, M, beta=1.0),
                  gemm_problem(operand(dy, 1, rowmap(Nout)), operand(x2, 1, rowmap(K2)),
                               grad_buffer(w2), rowmap(K2), Nout, K2, M, beta=1.0)], x1.device)
        if b1 is not None:
            colsum_accumulate(dy.view(M, Nout), grad_buffer(b1),
                              grad_buffer(b2) if b2 is not None else None)
        return dx1, None, None, dx2, None, None


def linear2(x1, w1, b1, x2, w2, b2):
    return Linear2Fn.apply(x1, w1, b1, x2, w2, b2)


# ---------------------------------------------------------------------------
# Teacher-forced location-attention decoder loop (attention_seq2seq.py:704-799)
# ---------------------------------------------------------------------------
def _attdec_forward(enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid, w_ih, w_hh, w_dec,
                    w_conv, conv_w, v, train_opts, keep_feat=False):
    """One asr_attdec_forward_ex call over S = pre_emb.shape[1] steps.  Returns
    (dims, (dec, cst, gates, x, ctx, aw), opts, buffers kept alive)."""
    N.require_device(enc, enc_a, lens, pre_emb, w_ih)
    B, T, E = enc.shape
    A = enc_a.shape[-1]
    D = w_hh.shape[1]
    S = pre_emb.shape[1]
    C, K = conv_w.shape[0], conv_w.shape[-1]
    dims = N.AttDecDims(B, T, E, A, C, K, D, S, float(sharpen), int(bool(sigmoid)))
    dev = enc.device
    cd = compute_dtype()
    f32 = dict(dtype=torch.float32, device=dev)
    dec = torch.empty(B, S, D, **f32)
    cst = torch.empty(B, S, D, **f32)
    gates = torch.empty(B, S, 4 * D, **f32)
    x = torch.empty(B, S, E + D, **f32)
    ctxv = torch.empty(B, S, E, **f32)
    aw = torch.empty(B, S, T, **f32)
    nb = N.query('asr_attdec_workspace_bytes', ctypes.byref(dims), cd, 0)
    ws = _ws(nb, dev)
    ld_ih = w_ih.shape[1]
    w_ih_ctx = ctypes.c_void_p(w_ih.data_ptr() + 4 * emb_dim)
    opts, keep = _attdec_opts(train_opts, B, S, D, emb_dim, w_ih, dev)
    # a backward will follow: the persistent pass keeps every step's conv
    # features for it (asr_attdec_set_conv_feat; ASR_ATT_CONV_FEAT=0: recomputed)
    feat = None
    if keep_feat and os.environ.get('ASR_ATT_CONV_FEAT', '1') != '0':
        fb = N.query('asr_attdec_conv_feat_bytes', ctypes.byref(dims))
        feat = torch.empty(max(int(fb) // 4, 1), dtype=torch.float32, device=dev)
        N.call('asr_attdec_set_conv_feat', N.ptr(feat))
    try:
        N.call('asr_attdec_forward_ex', ctypes.byref(dims), N.ptr_struct(opts), cd, N.ptr(enc),
               N.ptr(enc_a), N.ptr(lens), w_ih_ctx, ld_ih, N.ptr(w_hh), N.ptr(w_dec),
               N.ptr(w_conv), N.ptr(conv_w), N.ptr(v), N.ptr(pre_emb),
               N.ptr(h0.contiguous() if h0 is not None else None), N.ptr(dec), N.ptr(cst),
               N.ptr(gates), N.ptr(x), N.ptr(ctxv), N.ptr(aw), N.ptr(ws), nb,
               N.stream_handle(dev))
    finally:
        if feat is not None:
            N.call('asr_attdec_set_conv_feat', None)
    if feat is not None:
        ran = (ctypes.c_int * 2)()
        N.call("asr_attdec_persist_last", ctypes.cast(ran, ctypes.c_void_p))
        if ran[0] == 1:          # written only by the persistent forward pass
            keep['conv_feat'] = feat
    return dims, (dec, cst, gates, x, ctxv, aw), opts, keep


@torch.no_grad()
def att_decode_greedy(enc, enc_a, lens, h0, emb_dim, sharpen, sigmoid, w_ih, w_hh, w_dec, w_conv,
                      conv_w, v, gen, max_len):
    """Greedy attention decoding (attention_seq2seq.py:917-1036, bahdanau
    order) as ONE fused decoder pass: every step t >= 1 is a sampled step whose
    input token is the in-loop first argmax of logits_{t-1} = fc(tanh(W_d dec +
    b_d + W_c ctx + b_c)) -- the same machinery as scheduled sampling, with no
    dropout.  S = max_len + 1 steps run so the argmax of step max_len - 1 is
    produced too.  gen: dict(w_d, b_d, w_c, b_c, w_fc, b_fc, emb_w, emb_trans,
    b_ih, b_hh).  Returns (tokens int64 [B, max_len], aw [B, max_len, T]) on
    the device, before the all-<eos> truncation."""
    enc, enc_a = enc.contiguous(), enc_a.contiguous()
    B = enc.shape[0]
    D = w_hh.shape[1]
    S = int(max_len) + 1
    pre_emb = torch.zeros(B, S, 4 * D, dtype=torch.float32, device=enc.device)  # never read
    flags = np.ones(S, np.int32)
    flags[0] = 0
    _, outs, _, keep = _attdec_forward(enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid,
                                       w_ih, w_hh, w_dec, w_conv, conv_w, v,
                                       dict(gen, ss_steps=flags))
    return keep['tok_ss'][:, 1:], outs[5][:, :S - 1]


_last_sampled = {'tok': None}


def last_sampled_tokens():
    """The sampled tokens [B, S] (int64, device; -1 at teacher-forced steps)
    of the last fused decoder forward that had sampled steps, else None (the
    decoder pass's tok_ss output; tests read it)."""
    return _last_sampled['tok']


class AttDecoderFn(torch.autograd.Function):
    """Returns (dec_out [B,S,D], ctx [B,S,E], aw [B,S,T]).  Weights:
    w_ih [4D, emb+E] (LSTMCell; only the context columns are used here, the
    embedding columns enter through pre_emb), w_hh [4D, D], w_dec [A, D],
    w_conv [A, C], conv_w [C,1,1,K], v [1, A]."""

    @staticmethod
    def forward(ctx, enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid, w_ih, w_hh,
                w_dec, w_conv, conv_w, v, train_opts):
        enc, enc_a, pre_emb = enc.contiguous(), enc_a.contiguous(), pre_emb.contiguous()
        dims, (dec, cst, gates, x, ctxv, aw), opts, keep = _attdec_forward(
            enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid, w_ih, w_hh, w_dec, w_conv,
            conv_w, v, train_opts, keep_feat=any(ctx.needs_input_grad))
        ctx.save_for_backward(enc, enc_a, lens, w_ih, w_hh, w_dec, w_conv, conv_w, v, dec, cst,
                              gates, x, aw)
        _last_sampled['tok'] = keep.get('tok_ss')
        ctx.meta = (dims, emb_dim, h0 is not None)
        ctx.opts = (opts, keep, train_opts)
        ctx.mark_non_differentiable(aw)
        return dec, ctxv, aw

    @staticmethod
    def backward(ctx, d_dec, d_ctx, d_aw):
        (enc, enc_a, lens, w_ih, w_hh, w_dec, w_conv, conv_w, v, dec, cst, gates, x,
         aw) = ctx.saved_tensors
        dims, emb_dim, has_h0 = ctx.meta
        B, T, E, A, C, K, D, S = (dims.B, dims.T, dims.E, dims.A, dims.C, dims.K, dims.D, dims.S)
        dev = enc.device
        cd = compute_dtype()
        f32 = dict(dtype=torch.float32, device=dev)
        d_dec = d_dec.contiguous() if d_dec is not None else torch.zeros(B, S, D, **f32)
        d_ctx = d_ctx.contiguous() if d_ctx is not None else torch.zeros(B, S, E, **f32)
        dctx_tot = torch.empty(B, S, E, **f32)
        d_enc_a = torch.empty(B, T, A, **f32)
        d_h0 = torch.empty(B, D, **f32) if has_h0 else None
        dwd = torch.empty(B, S, A, **f32)
        nrow = B * N.query('asr_attdec_chunks', ctypes.byref(dims))   # per frame chunk
        dv_part = torch.empty(nrow, A, **f32)
        dwc_part = torch.empty(nrow, A * C, **f32)
        dcw_part = torch.empty(nrow, C * K, **f32)
        nb = N.query('asr_attdec_workspace_bytes', ctypes.byref(dims), cd, 1)
        ws = _ws(nb, dev)
        ld_ih = w_ih.shape[1]
        w_ih_ctx = ctypes.c_void_p(w_ih.data_ptr() + 4 * emb_dim)
        opts, keep, train_opts = ctx.opts
        sampled = 'emb_ss' in keep
        if sampled:
            d_pre = torch.empty(B, S, 4 * D, **f32)
            dg_ss = torch.empty(B, S, 4 * D, **f32)
            opts.d_pre, opts.dg_ss = d_pre.data_ptr(), dg_ss.data_ptr()
        feat = keep.get('conv_feat')
        if feat is not None:
            N.call('asr_attdec_set_conv_feat', N.ptr(feat))
        try:
            N.call('asr_attdec_backward_ex', ctypes.byref(dims), N.ptr_struct(opts), cd,
                   N.ptr(enc), N.ptr(enc_a), N.ptr(lens), w_ih_ctx, ld_ih, N.ptr(w_hh),
                   N.ptr(w_dec), N.ptr(w_conv), N.ptr(conv_w), N.ptr(v), N.ptr(dec), N.ptr(cst),
                   N.ptr(aw), N.ptr(d_dec), N.ptr(d_ctx), N.ptr(gates), N.ptr(dctx_tot),
                   N.ptr(d_enc_a), N.ptr(d_h0), N.ptr(dwd), N.ptr(dv_part), N.ptr(dwc_part),
                   N.ptr(dcw_part), N.ptr(ws), nb, N.stream_handle(dev))
        finally:
            if feat is not None:
                N.call('asr_attdec_set_conv_feat', None)
        dg = gates                          # dgates (row t = 0 is zero)
        d_pre_out = dg
        if sampled:
            # sampled steps were fed embed(argmax) (detached): their gate gradients
            # reach W_ih[:, :Y] through the embedding actually used and both
            # biases, never the teacher embedding (attention_seq2seq.py:744-748)
            emb_ss = keep['emb_ss']
            Y = emb_dim
            run_gemm([gemm_problem(operand(dg_ss, 1, rowmap(4 * D)), operand(emb_ss, 1, rowmap(Y)),
                                   grad_buffer(w_ih), rowmap(ld_ih), 4 * D, Y, B * S, beta=1.0)],
                     dev)
            colsum_accumulate(dg_ss.view(B * S, 4 * D), grad_buffer(train_opts['b_ih']),
                              grad_buffer(train_opts['b_hh']))
            d_pre_out = d_pre
        BS, G, ED = B * S, 4 * D, E + D
        # LSTMCell weights: dW_ih[:, emb:] += dG^T x[:, :E]; dW_hh += dG^T x[:, E:]
        run_gemm([gemm_problem(operand(dg, 1, rowmap(G)), operand(x, 1, rowmap(ED)),
                               grad_buffer(w_ih), rowmap(ld_ih), G, E, BS, beta=1.0,
                               c_offset=emb_dim),
                  gemm_problem(operand(dg, 1, rowmap(G)), operand(x, 1, rowmap(ED), offset=E),
                               grad_buffer(w_hh), rowmap(D), G, D, BS, beta=1.0)], dev)
        # attention weights
        run_gemm([gemm_problem(operand(dwd, 1, rowmap(A)), operand(dec, 1, rowmap(D)),
                               grad_buffer(w_dec), rowmap(D), A, D, BS, beta=1.0)], dev)
        colsum_accumulate(dv_part, grad_buffer(v))
        colsum_accumulate(dwc_part, grad_buffer(w_conv))
        colsum_accumulate(dcw_part, grad_buffer(conv_w))
        # d enc[b] = aw[b]^T dctx_tot[b]   (batched over utterances)
        d_enc = torch.empty_like(enc)
        run_gemm([gemm_problem(operand(aw, 1, rowmap(T)), operand(dctx_tot, 1, rowmap(E)), d_enc,
                               rowmap(E), T, E, S, batch=B,
                               batch_strides=(S * T, S * E, T * E))], dev)
        return (d_enc, d_enc_a, None, d_pre_out, d_h0, None, None, None, None, None, None, None,
                None, None, None)


class AttStepFn(torch.autograd.Function):
    """One location-attention step (AttentionMechanism.forward,
    attention_layer.py:123-251) on the decoder loop's kernels:
    (enc [B,T,E], enc_a [B,T,A], lens int32 [B], dec_out [B,D], aw_prev [B,T])
    -> (ctx [B,E], aw [B,T]).  Weight gradients (W_dec [A,D], W_conv [A,C],
    conv [C,1,1,K], V [1,A]) accumulate into their .grad."""

    @staticmethod
    def forward(ctx, enc, enc_a, lens, dec_out, aw_prev, w_dec, w_conv, conv_w, v, sharpen,
                sigmoid):
        N.require_device(enc, enc_a, lens, dec_out, aw_prev, w_dec)
        enc, enc_a = enc.contiguous(), enc_a.contiguous()
        dec_out, aw_prev = dec_out.contiguous(), aw_prev.contiguous()
        B, T, E = enc.shape
        A, D = w_dec.shape
        C, K = conv_w.shape[0], conv_w.shape[-1]
        dims = N.AttDecDims(B, T, E, A, C, K, D, 2, float(sharpen), int(bool(sigmoid)))
        dev = enc.device
        ctx_out = torch.empty(B, E, dtype=torch.float32, device=dev)
        aw_out = torch.empty(B, T, dtype=torch.float32, device=dev)
        nb = N.query('asr_att_step_workspace_bytes', ctypes.byref(dims))
        ws = _ws(nb, dev)
        N.call('asr_att_step_forward', ctypes.byref(dims), N.ptr(enc), N.ptr(enc_a), N.ptr(lens),
               N.ptr(w_dec), N.ptr(w_conv), N.ptr(conv_w), N.ptr(v), N.ptr(dec_out),
               N.ptr(aw_prev), N.ptr(ctx_out), N.ptr(aw_out), N.ptr(ws), nb,
               N.stream_handle(dev))
        ctx.save_for_backward(enc, enc_a, lens, dec_out, aw_prev, w_dec, w_conv, conv_w, v,
                              aw_out)
        ctx.dims = dims
        return ctx_out, aw_out

    @staticmethod
    def backward(ctx, d_ctx, d_aw):
        enc, enc_a, lens, dec_out, aw_prev, w_dec, w_conv, conv_w, v, aw_out = ctx.saved_tensors
        dims = ctx.dims
        B, T, E, A, C, K, D = dims.B, dims.T, dims.E, dims.A, dims.C, dims.K, dims.D
        dev = enc.device
        f32 = dict(dtype=torch.float32, device=dev)
        d_ctx = d_ctx.contiguous() if d_ctx is not None else torch.zeros(B, E, **f32)
        d_aw = d_aw.contiguous() if d_aw is not None else None
        d_enc_a = torch.empty(B, T, A, **f32)
        d_dec = torch.empty(B, D, **f32)
        d_aw_prev = torch.empty(B, T, **f32)
        dctx_tot = torch.empty(B, E, **f32)
        dwd = torch.empty(B, A, **f32)
        nrow = B * N.query('asr_attdec_chunks', ctypes.byref(dims))
        dv_part = torch.empty(nrow, A, **f32)
        dwc_part = torch.empty(nrow, A * C, **f32)
        dcw_part = torch.empty(nrow, C * K, **f32)
        nb = N.query('asr_att_step_workspace_bytes', ctypes.byref(dims))
        ws = _ws(nb, dev)
        N.call('asr_att_step_backward', ctypes.byref(dims), N.ptr(enc), N.ptr(enc_a), N.ptr(lens),
               N.ptr(w_dec), N.ptr(w_conv), N.ptr(conv_w), N.ptr(v), N.ptr(dec_out),
               N.ptr(aw_prev), N.ptr(aw_out), N.ptr(d_ctx), N.ptr(d_aw), N.ptr(d_enc_a),
               N.ptr(d_dec), N.ptr(d_aw_prev), N.ptr(dctx_tot), N.ptr(dwd), N.ptr(dv_part),
               N.ptr(dwc_part), N.ptr(dcw_part), N.ptr(ws), nb, N.stream_handle(dev))
        run_gemm([gemm_problem(operand(dwd, 1, rowmap(A)), operand(dec_out, 1, rowmap(D)),
                               grad_buffer(w_dec), rowmap(D), A, D, B, beta=1.0)], dev)
        colsum_accumulate(dv_part, grad_buffer(v))
        colsum_accumulate(dwc_part, grad_buffer(w_conv))
        colsum_accumulate(dcw_part, grad_buffer(conv_w))
        d_enc = torch.empty_like(enc)      # d enc[b] = aw_out[b]^T dctx_tot[b] (K = 1)
        run_gemm([gemm_problem(operand(aw_out, 1, rowmap(T)), operand(dctx_tot, 1, rowmap(E)),
                               d_enc, rowmap(E), T, E, 1, batch=B,
                               batch_strides=(T, E, T * E))], dev)
        return d_enc, d_enc_a, None, d_dec, d_aw_prev, None, None, None, None, None, None


class LSTMCellFn(torch.autograd.Function):
    """nn.LSTMCell nonlinearity on gate pre-activations: (pre [B,4D], c_prev
    [B,D]) -> (h, c).  The GEMMs are linear2 (x W_ih^T + b_ih + h W_hh^T + b_hh)."""

    @staticmethod
    def forward(ctx, pre, c_prev):
        N.require_device(pre, c_prev)
        pre, c_prev = pre.contiguous(), c_prev.contiguous()
        B, G = pre.shape
        D = G // 4
        act = torch.empty_like(pre)
        h = torch.empty(B, D, dtype=torch.float32, device=pre.device)
        c = torch.empty(B, D, dtype=torch.float32, device=pre.device)
        N.call('asr_lstm_cell_forward', N.ptr(pre), N.ptr(c_prev), B, D, N.ptr(act), N.ptr(h),
               N.ptr(c), N.stream_handle(pre.device))
        ctx.save_for_backward(act, c_prev, c)
        return h, c

    @staticmethod
    def backward(ctx, dh, dc):
        act, c_prev, c = ctx.saved_tensors
        B, D = c.shape
        dpre = torch.empty_like(act)
        dc_prev = torch.empty_like(c)
        N.call('asr_lstm_cell_backward', N.ptr(act), N.ptr(c_prev), N.ptr(c),
               N.ptr(dh.contiguous() if dh is not None else None),
               N.ptr(dc.contiguous() if dc is not None else None), B, D, N.ptr(dpre),
               N.ptr(dc_prev), N.stream_handle(c.device))
        return dpre, dc_prev


class GRUCellFn(torch.autograd.Function):
    """nn.GRUCell nonlinearity on the two GEMM outputs (gi = x W_ih^T + b_ih,
    gh = h W_hh^T + b_hh, [B, 3D]) and h -> h' (csrc/gru.hip)."""

    @staticmethod
    def forward(ctx, gi, gh, h):
        N.require_device(gi, gh, h)
        gi, gh, h = gi.contiguous(), gh.contiguous(), h.contiguous()
        B, D = h.shape
        act = torch.empty_like(gi)
        hout = torch.empty_like(h)
        N.call('asr_gru_cell_forward', N.ptr(gi), N.ptr(gh), N.ptr(h), B, D, N.ptr(act),
               N.ptr(hout), N.stream_handle(h.device))
        ctx.save_for_backward(act, gh, h)
        return hout

    @staticmethod
    def backward(ctx, dh):
        act, gh, h = ctx.saved_tensors
        B, D = h.shape
        dgi, dgh = torch.empty_like(act), torch.empty_like(act)
        dh_prev = torch.empty_like(h)
        N.call('asr_gru_cell_backward', N.ptr(act), N.ptr(gh), N.ptr(h), N.ptr(dh.contiguous()),
               B, D, N.ptr(dgi), N.ptr(dgh), N.ptr(dh_prev), N.stream_handle(h.device))
        return dgi, dgh, dh_prev


def gru_cell(x, h, w_ih, w_hh, b_ih, b_hh):
    """One nn.GRUCell step on the HIP GEMM + cell kernels."""
    return GRUCellFn.apply(linear(x, w_ih, b_ih), linear(h, w_hh, b_hh), h)


def lstm_cell(x, h, c, w_ih, w_hh, b_ih, b_hh):
    """One nn.LSTMCell step on the HIP GEMM + cell kernels."""
    pre = linear2(x, w_ih, b_ih, h, w_hh, b_hh)
    return LSTMCellFn.apply(pre, c)


def att_step(enc, enc_a, lens, dec_out, aw_prev, w_dec, w_conv, conv_w, v, sharpen=1.0,
             sigmoid=False):
    return AttStepFn.apply(enc, enc_a, lens, dec_out, aw_prev, w_dec, w_conv, conv_w, v, sharpen,
                           sigmoid)


def _attdec_opts(o, B, S, D, Y, w_ih, dev):
    """asr_attdec_opts_t from the training options dict (None = inference
    semantics: no dropout, teacher forcing).  Returns (opts | None, buffers to
    keep alive)."""
    keep = {}
    if not o:
        return None, keep
    opts = N.AttDecOpts()
    opts.dropout_hidden = float(o.get('dropout_hidden', 0.0))
    opts.seed_hidden = int(o.get('seed_hidden', 0))
    ss = o.get('ss_steps')
    if ss is not None and np.any(ss[1:]):
        flags = np.ascontiguousarray(ss, dtype=np.int32)
        keep['flags'] = flags
        f32 = dict(dtype=torch.float32, device=dev)
        keep['pre_ss'] = torch.empty(B, S, 4 * D, **f32)
        keep['emb_ss'] = torch.zeros(B, S, Y, **f32)
        keep['tok_ss'] = torch.full((B, S), -1, dtype=torch.int64, device=dev)
        opts.ss_steps_host = flags.ctypes.data
        opts.Y, opts.Dz, opts.V = Y, o['w_d'].shape[0], o['w_fc'].shape[0]
        for k in ('w_d', 'b_d', 'w_c', 'b_c', 'w_fc', 'b_fc', 'emb_w', 'b_ih', 'b_hh'):
            setattr(opts, k, o[k].data_ptr() if o.get(k) is not None else None)
        opts.drop_d, opts.seed_d = float(o.get('drop_d', 0.0)), int(o.get('seed_d', 0))
        opts.drop_c, opts.seed_c = float(o.get('drop_c', 0.0)), int(o.get('seed_c', 0))
        opts.drop_emb, opts.seed_emb = float(o.get('drop_emb', 0.0)), int(o.get('seed_emb', 0))
        opts.emb_trans = int(o.get('emb_trans', 0))
        opts.w_ih_emb, opts.ld_ih = w_ih.data_ptr(), w_ih.shape[1]
        opts.pre_ss = keep['pre_ss'].data_ptr()
        opts.emb_ss = keep['emb_ss'].data_ptr()
        opts.tok_ss = keep['tok_ss'].data_ptr()
    return opts, keep


def att_decoder(enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid, w_ih, w_hh, w_dec,
                w_conv, conv_w, v, train_opts=None):
    """train_opts (training mode): dict with dropout_hidden / seed_hidden and,
    for scheduled sampling, ss_steps (host int array [S]) plus the weights
    w_d, b_d, w_c, b_c, w_fc, b_fc, emb_w (emb_trans), b_ih, b_hh and the
    bottleneck / embedding dropout rates and seeds (drop_d, seed_d, drop_c,
    seed_c, drop_emb, seed_emb)."""
    return AttDecoderFn.apply(enc, enc_a, lens, pre_emb, h0, emb_dim, sharpen, sigmoid, w_ih,
                              w_hh, w_dec, w_conv, conv_w, v, train_opts)


# ---------------------------------------------------------------------------
# One bidirectional LSTM layer (nn.LSTM bidirectional + pack/pad, rnn.py)
# ---------------------------------------------------------------------------
class BLSTMLayerFn(torch.autograd.Function):
    """x_src [B, T_src, Din] f32; the layer input row (b, t) is
    x_src[perm[b] if perm else b, t*t_mul + t_add].  Parameters are passed as
    (w_ih [8H, Din], w_hh [8H, H], b_ih [8H], b_hh [8H]) where each is the
    forward-direction tensor immediately followed in memory by the reverse one
    (the flat layout of models/pytorch_v3/base.py).

    bf16 mode stages every GEMM operand in bf16 once (the gathered input X and
    W_ih by one conversion pass each; y and dG are written in bf16 by the
    recurrence kernels themselves), so all four layer GEMMs take the
    buffer->LDS bf16 fast path of gemm.hip.  fp32 mode reads the f32 tensors
    directly (exact-f32 MFMA, parity mode)."""

    @staticmethod
    def forward(ctx, x_src, lens, T, perm, t_mul, t_add, gbufs, concat, drop, next_rec, out_spec,
                w_ih, w_hh, b_ih, b_hh, *graph_params):
        N.require_device(x_src, lens, w_ih, w_hh, b_ih, b_hh)
        # the layer below handed its output over as staged bf16 (bf16_handoff)
        twin = _handoff_input(x_src, perm, t_mul, t_add, T, concat, drop, w_ih.shape[1])
        x_src = x_src.contiguous()
        fused_drop = drop is not None and compute_dtype() == BF16 and not concat
        if drop is not None and not fused_drop:   # materialise dropout(x_src) first
            xd = torch.empty_like(x_src)
            N.call('asr_dropout', N.ptr(x_src), N.ptr(xd), x_src.numel(), float(drop[0]),
                   int(drop[1]), N.stream_handle(x_src.device))
            x_src = xd
        B, T_src, Dsrc = x_src.shape
        # concat: the input row (b, t) spans source frames t*t_mul + t_add and the
        # next one (rnn.py:421-431), i.e. 2*Dsrc contiguous values
        Din = 2 * Dsrc if concat else Dsrc
        assert w_ih.shape[1] == Din, (tuple(w_ih.shape), Din)
        H = w_hh.shape[1]
        dev = x_src.device
        cd = compute_dtype()
        a_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
        fuse_x = False
        gx = None       # f32 gate pre-activations -> activations [B, T, 8H], or
        Dp = Din        # packed fp16 activations [B, T, 2, H, 4] (fused bf16 path)
        if twin is not None:
            x_op = twin.view(B * T, Din)
            w_op = _wih_bf16(w_ih, graph_params, H, Din)           # [8H, Din]
            y_bf = torch.empty(B, T, 2 * H, dtype=torch.bfloat16, device=dev)
        elif cd == BF16:
            if Din % 8 and not fused_drop:
                # an input width that is not a multiple of 8 (TIMIT's 123) is
                # staged with zero-padded rows of Dp columns, so the fused
                # projection and the fast GEMMs take it (the zero columns add
                # nothing): no generic-kernel GEMMs on layer 0
                Dp = (Din + 7) // 8 * 8
                x_op = torch.empty(B * T, Dp, dtype=torch.bfloat16, device=dev)
                N.call('asr_convert_rows_bf16_ld', N.ptr(x_src), a_map, B * T, Din, Dp,
                       N.ptr(x_op), N.stream_handle(dev))
                w_op = _staged(w_ih, 8 * H, Din, Dp)                  # [8H, Dp]
            else:
                x_op = convert_rows_bf16(x_src, a_map, B * T, Din,    # [B*T, Din]
                                         drop=drop if fused_drop else None)
                w_op = _wih_bf16(w_ih, graph_params, H, Din)           # [8H, Din]
            y_bf = torch.empty(B, T, 2 * H, dtype=torch.bfloat16, device=dev)
        else:
            x_op, w_op, y_bf = x_src, w_ih, None
        y = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        cst = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        nb = N.query('asr_lstm_workspace_bytes', B, H, cd, 0)
        slot = _arena_take(nb, dev)         # zeroed by rec_arena_begin
        ws = slot[0] if slot is not None else _ws(nb, dev)
        pz = slot is not None
        # the backward's slot, reserved now so the arena's one fill covers it
        ctx.bws = _arena_take(N.query('asr_lstm_workspace_bytes', B, H, cd, 2), dev) if pz else None
        whh_r = w_hh.data_ptr() + 4 * H * H * 4
        y_f32, out_drop = out_spec
        handoff = None     # (bf16 tensor the next layer stages from, its dropout)
        if cd == BF16 and _fuse_xproj_on():
            # the input projection inside the persistent recurrence (no gx GEMM);
            # ASR_ERR_UNSUPPORTED when this shape / configuration does not take it.
            # The gate activations are kept as packed fp16 (8 B per cell instead
            # of 16; ASR_XG_ACT_H=0 keeps the f32 layout)
            args = (N.ptr(x_op), Dp, N.ptr(w_op), N.ptr(b_ih), N.ptr(b_hh), N.ptr(w_hh),
                    ctypes.c_void_p(whh_r), N.ptr(lens), B, T, H)
            if _act_h_on() and not y_f32:
                # the next BLSTM layer stages its input from bf16 written here (its
                # dropout applied): no f32 y, no conversion pass
                gx = torch.empty(B, T, 2, H, 4, dtype=torch.float16, device=dev)
                fn = 'asr_lstm_forward_xh_drop'
                y_d = (torch.empty(B, T, 2 * H, dtype=torch.bfloat16, device=dev)
                       if out_drop is not None else None)
                p, seed = out_drop if out_drop is not None else (0.0, 0)
                with _prezeroed(pz):
                    rc = N.query(fn, *args, N.ptr(gx), None, N.ptr(cst), N.ptr(y_bf),
                                 N.ptr(y_d) if y_d is not None else None, ctypes.c_float(p),
                                 ctypes.c_ulonglong(seed), N.ptr(ws), nb, N.stream_handle(dev))
                if rc == 0:
                    handoff = (y_d if y_d is not None else y_bf, out_drop)
            else:
                if _act_h_on():
                    gx = torch.empty(B, T, 2, H, 4, dtype=torch.float16, device=dev)
                    fn = 'asr_lstm_forward_xh'
                else:
                    gx = torch.empty(B, T, 8 * H, dtype=torch.float32, device=dev)
                    fn = 'asr_lstm_forward_x'
                with _prezeroed(pz):
                    rc = N.query(fn, *args, N.ptr(gx), N.ptr(y), N.ptr(cst), N.ptr(y_bf),
                                 N.ptr(ws), nb, N.stream_handle(dev))
            if rc not in (0, N.ASR_ERR_UNSUPPORTED):
                raise N.NativeError('%s failed (rc=%d): %s' % (
                    fn, rc, N.lib().asr_last_error().decode(errors='replace')))
            fuse_x = rc == 0
        if not fuse_x:
            gx = torch.empty(B, T, 8 * H, dtype=torch.float32, device=dev)
            if cd == BF16:
                run_gemm([gemm_problem(operand(x_op, 0, rowmap(Dp)), operand(w_op, 0, rowmap(Dp)),
                                       gx, rowmap(8 * H), B * T, 8 * H, Dp, bias=b_ih,
                                       bias2=b_hh)], dev)
            else:
                run_gemm([gemm_problem(operand(x_src, 0, a_map), operand(w_ih, 0, rowmap(Din)), gx,
                                       rowmap(8 * H), B * T, 8 * H, Din, bias=b_ih, bias2=b_hh)],
                         dev)
            with _prezeroed(pz):
                N.call('asr_lstm_forward', N.ptr(gx), N.ptr(w_hh), ctypes.c_void_p(whh_r), F32,
                       N.ptr(lens), B, T, H, cd, N.ptr(y), N.ptr(cst), N.ptr(y_bf), N.ptr(ws),
                       nb, N.stream_handle(dev))
        ctx.save_for_backward(x_op, w_op, lens, w_hh, b_ih, b_hh, gx, cst,
                              y_bf if y_bf is not None else y)
        ctx.meta = (T, perm, t_mul, t_add, gbufs, cd, (B, T_src, Dsrc, Din, Dp), w_ih)
        ctx.bh = (B, H)     # the recurrence shape a gated side stream waits on
        ctx.drop = drop
        ctx.next_rec = bool(next_rec)
        ctx.n_graph = len(graph_params)
        ctx.handoff_in = twin is not None
        if handoff is not None:
            # y was not written: only the next BLSTM layer may consume it, through
            # the bf16 tensor (_handoff_input raises for any other use it sees)
            y._asr_handoff = handoff
        return y

    @staticmethod
    def backward(ctx, dy):
        x_op, w_op, lens, w_hh, b_ih, b_hh, act, cst, y_op = ctx.saved_tensors
        T, perm, t_mul, t_add, gbufs, cd, (B, T_src, Dsrc, Din, Dp), w_ih = ctx.meta
        H = w_hh.shape[1]
        dev = act.device
        dy = dy.contiguous()
        # dy still being written by the layer above's input-gradient GEMMs
        # (_dx_pipelined): only the packed-activation tagged-granule backward
        # reads it that way; anything else waits for them first
        pipe = getattr(dy, '_asr_dy_pipe', None)
        if pipe is not None and act.dtype != torch.float16:
            torch.cuda.current_stream(dev).wait_event(pipe[3])
            pipe = None
        if gbufs is None:
            gbufs = tuple(grad_buffer(p) for p in (w_ih, w_hh, b_ih, b_hh))
        fused_db = os.environ.get('ASR_BIAS_FUSED', '1') != '0'
        whh_r = w_hh.data_ptr() + 4 * H * H * 4
        dg_bf = (torch.empty(B, T, 8 * H, dtype=torch.bfloat16, device=dev) if cd == BF16
                 else None)
        done = False
        # data parallel: every collective issued so far completes before this
        # persistent recurrence starts (a kernel co-resident with the
        # recurrence perturbs it)
        notify_grad_event('pre_recurrence')
        # the recurrence's LDS pin: co-resident GEMM work-groups only in the
        # opt-in mode 2 (84 KB); otherwise 140 KB excludes every GEMM kernel.
        # Units per work-group: 32 where that frees the CUs for mode 3.
        mode, xu = _overlap_plan(dev, B, H)
        N.call('asr_lstm_set_bwd_pin_kb', 84 if mode == '2' else 0)
        N.call('asr_lstm_set_bwd_units', xu)
        split = None
        band_seq = None   # (t0, t1): the same row bands, computed after the recurrence
        dx_split = None
        last_main = not ctx.next_rec and os.environ.get('ASR_WGRAD_LAST_MAIN', '1') != '0'
        wsplit = last_main and _wgrad_split_ok(ctx, T, mode)
        wprog = None      # (counter, target, event) of the bottom layer's banded dW overlap
        if (act.dtype == torch.float16 and pipe is None and _dx_split_ok(ctx, B, T, dev, mode)
                and not _dx_pipeline_ok(ctx, B, T, Din, dev)):
            N.call('asr_lstm_set_bwd_units', xu)     # (arrivals follow the units setting)
            # row bands by when their gate gradients are final: [T/4, 3T/4) at
            # processing step 3T/4 - 1, with two chunks also [T/8, T/4) and
            # [3T/4, 7T/8) at 7T/8 - 1; the rest after the recurrence.  Beside the
            # recurrence in mode 3; in the other modes the same bands after it, so
            # every mode computes dX by the same products
            two = _dx_split_chunks() == 2 and T >= 128
            arrivals = N.query('asr_lstm_bwd_progress_arrivals', B, H) if mode == '3' else 0
            # dX before the recurrence: its zero fill (non-identity maps) precedes
            # the side stream's writes
            ident = perm is None and t_mul == 1 and t_add == 0 and T == T_src and Din == Dsrc
            dx_split = (torch.empty if ident else torch.zeros)(B, T_src, Dsrc,
                                                               dtype=torch.float32, device=dev)
            if arrivals > 0:
                split = (T // 4, _progress_counter(dev), int(arrivals), T // 8 if two else None)
            else:
                band_seq = (T // 4, T // 8 if two else None)
        try:
            if act.dtype == torch.float16:
                # packed fp16 activations of asr_lstm_forward_xh: the tagged-granule
                # backward reads them directly; otherwise they are unpacked to f32
                nb = N.query('asr_lstm_workspace_bytes', B, H, cd, 2)
                res, ctx.bws = ctx.bws, None      # a reserved slot serves one backward
                pz = _arena_valid(res) and nb <= res[0].numel()
                ws = res[0] if pz else _ws(nb, dev)
                if pipe is not None:
                    N.call('asr_lstm_set_dy_flags', N.ptr(pipe[0]), pipe[1], pipe[2])
                if split is None and wsplit and mode == '3':
                    arrivals = N.query('asr_lstm_bwd_progress_arrivals', B, H)
                    if arrivals > 0:
                        wprog = (_progress_counter(dev), int(arrivals))
                        N.call('asr_lstm_set_bwd_progress', N.ptr(wprog[0][0]), T - 1 - T // 4)
                        wprog_pre = torch.cuda.Event()
                        wprog_pre.record(torch.cuda.current_stream(dev))
                if split is not None:
                    if split[3] is not None:
                        N.call('asr_lstm_set_bwd_progress2', N.ptr(split[1][0]), T - 1 - split[0],
                               T - 1 - split[3])
                    else:
                        N.call('asr_lstm_set_bwd_progress', N.ptr(split[1][0]), T - 1 - split[0])
                    # everything the side stream's share of dX reads that is not
                    # written by the recurrence is enqueued by now (dx's fill included)
                    split_pre = torch.cuda.Event()
                    split_pre.record(torch.cuda.current_stream(dev))
                try:
                    with _prezeroed(pz):
                        rc = N.query('asr_lstm_backward_dgbf_h', N.ptr(dy), N.ptr(w_hh),
                                     ctypes.c_void_p(whh_r), F32, N.ptr(lens), B, T, H, cd,
                                     N.ptr(act), N.ptr(cst), N.ptr(dg_bf), N.ptr(gbufs[2]),
                                     N.ptr(gbufs[3]), N.ptr(ws), nb, N.stream_handle(dev))
                finally:
                    if split is not None or wprog is not None:
                        N.call('asr_lstm_set_bwd_progress', None, 0)
                    if pipe is not None:
                        N.call('asr_lstm_set_dy_flags', None, 16, 0)
                        # (after the launch: later compute-stream work sees all of dy)
                        torch.cuda.current_stream(dev).wait_event(pipe[3])
                        pipe = None
                if rc not in (0, N.ASR_ERR_UNSUPPORTED):
                    raise N.NativeError('asr_lstm_backward_dgbf_h failed (rc=%d): %s' % (
                        rc, N.lib().asr_last_error().decode(errors='replace')))
                done = rc == 0
                if done and wprog is not None:
                    wprog[0][1] += wprog[1]
                    wprog = (wprog[0][0], wprog[0][1], wprog_pre)
                else:
                    wprog = None
                if done and split is not None:
                    first = split[1][1] + split[2]   # the arrivals this launch adds per step
                    split[1][1] += split[2] * (2 if split[3] is not None else 1)
                    split = split + ((first, split[1][1]), split_pre)
                elif split is not None:            # no report: the same bands after it
                    band_seq = (split[0], split[3])
                    split = None
                if not done:
                    a32 = torch.empty(B, T, 8 * H, dtype=torch.float32, device=dev)
                    N.call('asr_lstm_unpack_act_h', N.ptr(act), B, T, H, N.ptr(a32),
                           N.stream_handle(dev))
                    act = a32
            nb = N.query('asr_lstm_workspace_bytes', B, H, cd, 2 if fused_db else 1)
            ws = _ws(nb, dev)
            # the saved activations become the gate gradients dG in place; the bias
            # gradients (sum of dG over b, t) are accumulated by the same call
            if done:
                pass
            elif fused_db:
                # bf16 mode: only the bf16 dG feeds the GEMMs, so the f32 dG is not stored
                fn = 'asr_lstm_backward_dgbf' if dg_bf is not None else 'asr_lstm_backward_db'
                N.call(fn, N.ptr(dy), N.ptr(w_hh), ctypes.c_void_p(whh_r), F32,
                       N.ptr(lens), B, T, H, cd, N.ptr(act), N.ptr(cst), N.ptr(dg_bf),
                       N.ptr(gbufs[2]), N.ptr(gbufs[3]), N.ptr(ws), nb, N.stream_handle(dev))
            else:   # A/B: separate column-sum pass over dG
                N.call('asr_lstm_backward', N.ptr(dy), N.ptr(w_hh), ctypes.c_void_p(whh_r), F32,
                       N.ptr(lens), B, T, H, cd, N.ptr(act), N.ptr(cst), N.ptr(dg_bf), N.ptr(ws), nb,
                       N.stream_handle(dev))
                colsum_accumulate(act.view(B * T, 8 * H), gbufs[2], gbufs[3])
        finally:
            N.call('asr_lstm_set_bwd_units', 0)   # direct API callers: the default again
        # weight gradients of the layer above, if they went to a side stream: join
        # them here (they run beside the recurrence just enqueued) so the
        # gradient-ready bucket sees them on the compute stream
        _join_side_wgrads(dev)
        notify_grad_event('recurrence')
        dg_op = dg_bf if dg_bf is not None else act
        split_done = None
        if split is not None:
            t0, (ctr, _), _, t1, targets, pre = split
            side = _wgrad_side_stream(dev, B, H)[0]
            side.wait_event(pre)         # not the recurrence itself: the gate waits on its progress
            if os.environ.get('ASR_DX_SPLIT_SYNC') == '1':   # diagnostics: after the whole recurrence
                rec_done = torch.cuda.Event()
                rec_done.record(torch.cuda.current_stream(dev))
                side.wait_event(rec_done)
            rows = lambda ta, tb: _dx_rows_problem(dg_op, w_op, dx_split, ctx, B, T, T_src, H,  # noqa: E731
                                                   Din, Dp, Dsrc, perm, t_mul, t_add, ta, tb)
            with torch.cuda.stream(side):
                N.call('asr_gemm_set_nosplit', 1)     # per output element: one launch's sum
                try:
                    N.call('asr_lstm_progress_gate', N.ptr(ctr), targets[0], N.stream_handle(dev))
                    run_gemm([rows(t0, T - t0)], dev)
                    if t1 is not None:
                        N.call('asr_lstm_progress_gate', N.ptr(ctr), targets[1],
                               N.stream_handle(dev))
                        run_gemm([rows(t1, t0), rows(T - t0, T - t1)], dev)
                finally:
                    N.call('asr_gemm_set_nosplit', 0)
                split_done = torch.cuda.Event()
                split_done.record(side)
            for tt in (dg_op, w_op, dx_split, ctr) + ((perm,) if perm is not None else ()):
                tt.record_stream(side)
        # X as the dW_ih operand: the bf16 copy is already gathered (identity map)
        if cd == BF16:
            x_map = rowmap(Dp)
        else:
            x_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                           t_limit=T_src, perm=perm)
        # the bottom layer's weight gradients have no recurrence left to run
        # beside: they take the main stream and the full-size GEMM kernels (on
        # the co-resident small tiles the 4x320 layer-0 dW_ih ran at 29 TF/s)
        side_ent = None if last_main else _wgrad_side_stream(dev, B, H)
        # pipelined input gradient (_dx_pipelined): enqueued first, and the
        # side-stream weight gradients start after it, so the CUs the next
        # recurrence leaves free serve dX -- which that recurrence waits for --
        # before the weight gradients, which only the optimizer needs
        BT = B * T
        dx = dx_done = None
        pipelined = ctx.needs_input_grad[0] and _dx_pipeline_ok(ctx, B, T, Din, dev)
        if pipelined:
            dx = torch.empty(B, T_src, Dsrc, dtype=torch.float32, device=dev)
            dx_done = _dx_pipelined(dx, dg_op, w_op, B, T, H, Din, Dp, ctx.drop, dev)
        if side_ent is None and wsplit:
            # time bands: the middle one first (beside the recurrence's last
            # quarter when it reported progress), then the outer two
            tq = T // 4
            Dx = x_op.shape[-1]
            if wprog is not None:
                ctr, target, pre = wprog
                side = _wgrad_side_stream(dev, B, H)[0]
                side.wait_event(pre)
                with torch.cuda.stream(side):
                    N.call('asr_lstm_progress_gate', N.ptr(ctr), target, N.stream_handle(dev))
                    _blstm_wgrad_rows(dg_op, x_op, Dx, y_op, T, gbufs, dev, tq, T - tq)
                    mid_done = torch.cuda.Event()
                    mid_done.record(side)
                for tt in (dg_op, x_op, y_op, ctr):
                    tt.record_stream(side)
                torch.cuda.current_stream(dev).wait_event(mid_done)
            else:
                _blstm_wgrad_rows(dg_op, x_op, Dx, y_op, T, gbufs, dev, tq, T - tq)
            _blstm_wgrad_rows(dg_op, x_op, Dx, y_op, T, gbufs, dev, 0, tq)
            _blstm_wgrad_rows(dg_op, x_op, Dx, y_op, T, gbufs, dev, T - tq, T)
            notify_grad_event('grads', gbufs)      # final on the compute stream
        elif side_ent is None:
            _blstm_wgrad(dg_op, act, x_op, x_map, y_op, T, gbufs, dev)
            notify_grad_event('grads', gbufs)      # final on the compute stream
        else:
            # weight gradients on a side stream, overlapping this layer's dX
            # GEMM and the previous layer's backward recurrence; joined back
            # into the main stream at the end of the backward pass
            side, small, gated = side_ent
            main = torch.cuda.current_stream(dev)
            side.wait_stream(main)
            if small:
                N.call('asr_gemm_set_small_tiles', 1)
            try:
                with torch.cuda.stream(side):
                    if dx_done is not None:
                        side.wait_event(dx_done)
                    elif gated and ctx.next_rec:
                        # hold the GEMMs back until the previous layer's backward
                        # recurrence (launched next on the main stream) is resident
                        N.call('asr_lstm_wgrad_gate', N.stream_handle(dev))
                    # (tools/cores_locate.py replaces _blstm_wgrad with stand-in
                    # side-stream workloads; nothing diagnostic runs here)
                    _blstm_wgrad(dg_op, act, x_op, x_map, y_op, T, gbufs, dev)
            finally:
                if small:
                    N.call('asr_gemm_set_small_tiles', 0)
            for t in (dg_op, act, x_op, y_op) + ((perm,) if perm is not None else ()):
                t.record_stream(side)
            if not _side_pending:
                torch.autograd.Variable._execution_engine.queue_callback(
                    lambda: _join_side_wgrads(dev, notify=False))
            _side_pending.append((side, gbufs, main))
        if split_done is not None:
            # the outer rows t in [0, T/4) and [3T/4, T) (two chunks: [0, T/8) and
            # [7T/8, T)) on the compute stream, then the side stream's rows joined
            t0 = split[3] if split[3] is not None else split[0]
            N.call('asr_gemm_set_nosplit', 1)
            try:
                run_gemm([_dx_rows_problem(dg_op, w_op, dx_split, ctx, B, T, T_src, H, Din, Dp,
                                           Dsrc, perm, t_mul, t_add, 0, t0),
                          _dx_rows_problem(dg_op, w_op, dx_split, ctx, B, T, T_src, H, Din, Dp,
                                           Dsrc, perm, t_mul, t_add, T - t0, T)], dev)
            finally:
                N.call('asr_gemm_set_nosplit', 0)
            torch.cuda.current_stream(dev).wait_event(split_done)
            dx = dx_split
        elif band_seq is not None:
            # the split's row bands in its order, on the compute stream
            t0, t1 = band_seq
            rows = lambda ta, tb: _dx_rows_problem(dg_op, w_op, dx_split, ctx, B, T, T_src, H,  # noqa: E731
                                                   Din, Dp, Dsrc, perm, t_mul, t_add, ta, tb)
            N.call('asr_gemm_set_nosplit', 1)
            try:
                run_gemm([rows(T // 4, T - T // 4)], dev)
                if t1 is not None:
                    run_gemm([rows(t1, t0), rows(T - t0, T - t1)], dev)
                te = t1 if t1 is not None else t0
                run_gemm([rows(0, te), rows(T - te, T)], dev)
            finally:
                N.call('asr_gemm_set_nosplit', 0)
            dx = dx_split
        elif ctx.needs_input_grad[0] and not pipelined:
            # dX [BT, Din] = dG [BT, 8H] W_ih [8H, Din], scattered back through the input map
            if perm is None and t_mul == 1 and t_add == 0 and T == T_src and Din == Dsrc:
                dx = torch.empty(B, T_src, Dsrc, dtype=torch.float32, device=dev)
            else:
                dx = torch.zeros(B, T_src, Dsrc, dtype=torch.float32, device=dev)
            c_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                           t_limit=T_src, perm=perm)
            # dropout's backward (the forward mask over x_src's flat offsets) is
            # applied by the GEMM's epilogue as it writes dX
            p = gemm_problem(operand(dg_op, 0, rowmap(8 * H)), operand(w_op, 1, rowmap(Dp)), dx,
                             c_map, BT, Din, 8 * H, drop=ctx.drop)
            run_gemm([p], dev)
        return (dx,) + (None,) * (14 + ctx.n_graph)


def _dx_rows_problem(dg_op, w_op, dx, ctx, B, T, T_src, H, Din, Dp, Dsrc, perm, t_mul, t_add,
                     ta, tb):
    """dX rows (b, t) for t in [ta, tb) of every utterance: dG [B, T, 8H] W_ih
    [8H, Din], written through the layer's input map (the dropout mask by dX's
    element offsets, as the whole-product form)."""
    n = tb - ta
    a_map = rowmap(8 * H, stride_b=T * 8 * H, rows_per_b=n, t_add=ta)
    c_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=n, t_mul=t_mul, t_add=t_add + ta * t_mul,
                   t_limit=T_src, perm=perm)
    return gemm_problem(operand(dg_op, 0, a_map), operand(w_op, 1, rowmap(Dp)), dx, c_map,
                        B * n, Din, 8 * H, drop=ctx.drop)


class BGRULayerFn(torch.autograd.Function):
    """Bidirectional GRU layer (nn.GRU, rnn.py:173-191 / :226-233) on the HIP
    recurrence of csrc/gru.hip.  Same input addressing as BLSTMLayerFn (row map
    with perm / subsampling / 'concat' rows read in place); parameters are the
    combined [fwd; rev] views (w_ih [6H, Din], w_hh [6H, H], b_ih, b_hh [6H]).
    The recurrence runs in f32 in both modes; the GEMMs take the library's
    bf16 operand staging in bf16 mode."""

    @staticmethod
    def forward(ctx, x_src, lens, T, perm, t_mul, t_add, gbufs, concat, w_ih, w_hh, b_ih, b_hh,
                *graph_params):
        N.require_device(x_src, lens, w_ih, w_hh, b_ih, b_hh)
        x_src = x_src.contiguous()
        B, T_src, Dsrc = x_src.shape
        Din = 2 * Dsrc if concat else Dsrc
        assert w_ih.shape[1] == Din, (tuple(w_ih.shape), Din)
        H = w_hh.shape[1]
        dev = x_src.device
        a_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
        gx = torch.empty(B, T, 6 * H, dtype=torch.float32, device=dev)
        run_gemm([gemm_problem(operand(x_src, 0, a_map), operand(w_ih, 0, rowmap(Din)), gx,
                               rowmap(6 * H), B * T, 6 * H, Din, bias=b_ih)], dev)
        y = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        ghn = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        N.call('asr_gru_forward', N.ptr(gx), N.ptr(w_hh), N.ptr(b_hh), N.ptr(lens), B, T, H,
               N.ptr(y), N.ptr(ghn), N.stream_handle(dev))
        ctx.save_for_backward(x_src, w_ih, w_hh, b_ih, b_hh, lens, gx, ghn, y)
        ctx.meta = (T, perm, t_mul, t_add, gbufs, Din)
        ctx.n_graph = len(graph_params)
        return y

    @staticmethod
    def backward(ctx, dy):
        x_src, w_ih, w_hh, b_ih, b_hh, lens, act, ghn, y = ctx.saved_tensors
        T, perm, t_mul, t_add, gbufs, Din = ctx.meta
        B, T_src, Dsrc = x_src.shape
        H = w_hh.shape[1]
        dev = act.device
        dy = dy.contiguous()
        if gbufs is None:
            gbufs = tuple(grad_buffer(p) for p in (w_ih, w_hh, b_ih, b_hh))
        g_ih, g_hh, g_bih, g_bhh = gbufs
        nb = N.query('asr_gru_workspace_bytes', B, H)
        ws = _ws(nb, dev)
        dgh = torch.empty(B, T, 6 * H, dtype=torch.float32, device=dev)
        # the saved activations become dgx in place
        N.call('asr_gru_backward', N.ptr(dy), N.ptr(w_hh), N.ptr(lens), B, T, H, N.ptr(act),
               N.ptr(ghn), N.ptr(y), N.ptr(dgh), N.ptr(ws), nb, N.stream_handle(dev))
        BT = B * T
        x_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
        # dW_ih [6H, Din] += dgx^T x (both directions in one problem)
        run_gemm([gemm_problem(operand(act, 1, rowmap(6 * H)), operand(x_src, 1, x_map), g_ih,
                               rowmap(Din), 6 * H, Din, BT, beta=1.0)], dev)
        # dW_hh[dir] += dgh_dir^T h_prev_dir ; h_prev = y[b, t-1, :H] (fwd), y[b, t+1, H:] (rev)
        hp_f = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=-1, t_limit=T)
        hp_r = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=1, t_limit=T)
        run_gemm([
            gemm_problem(operand(dgh, 1, rowmap(6 * H)), operand(y, 1, hp_f), g_hh, rowmap(H),
                         3 * H, H, BT, beta=1.0),
            gemm_problem(operand(dgh, 1, rowmap(6 * H), offset=3 * H),
                         operand(y, 1, hp_r, offset=H), g_hh, rowmap(H), 3 * H, H, BT, beta=1.0,
                         c_offset=3 * H * H),
        ], dev)
        colsum_accumulate(act.view(BT, 6 * H), g_bih)
        colsum_accumulate(dgh.view(BT, 6 * H), g_bhh)
        notify_grad_event('recurrence')
        notify_grad_event('grads', gbufs)
        dx = None
        if ctx.needs_input_grad[0]:
            if perm is None and t_mul == 1 and t_add == 0 and T == T_src and Din == Dsrc:
                dx = torch.empty(B, T_src, Dsrc, dtype=torch.float32, device=dev)
            else:
                dx = torch.zeros(B, T_src, Dsrc, dtype=torch.float32, device=dev)
            c_map = rowmap(Dsrc, stride_b=T_src * Dsrc, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                           t_limit=T_src, perm=perm)
            run_gemm([gemm_problem(operand(act, 0, rowmap(6 * H)), operand(w_ih, 1, rowmap(Din)),
                                   dx, c_map, BT, Din, 6 * H)], dev)
        return (dx,) + (None,) * (11 + ctx.n_graph)


def bgru_layer(x_src, lens, T, w_ih, w_hh, b_ih, b_hh, perm=None, t_mul=1, t_add=0, gbufs=None,
               graph_params=(), concat=False):
    """The bidirectional GRU counterpart of blstm_layer (same addressing)."""
    return BGRULayerFn.apply(x_src, lens, T, perm, t_mul, t_add, gbufs, bool(concat),
                             w_ih, w_hh, b_ih, b_hh, *graph_params)


def _act_h_on():
    """Fused bf16 forward: keep the gate activations as packed fp16
    (asr_lstm_forward_xh; ASR_XG_ACT_H=0 keeps f32)."""
    return os.environ.get('ASR_XG_ACT_H', '1') != '0'


def _fuse_xproj_on():
    """bf16 mode: try the layer's input projection inside the persistent
    forward recurrence (asr_lstm_forward_x) first (ASR_FUSE_XPROJ=0 keeps the
    separate GEMM)."""
    return os.environ.get('ASR_FUSE_XPROJ', '1') != '0'


def convert_rows_bf16(src, rmap, nrows, ncols, drop=None):
    """Dense bf16 [nrows, ncols] copy of the rows of `src` selected by a row map;
    drop=(p, seed): of dropout(src) with asr_dropout's mask, in the same pass."""
    out = torch.empty(nrows, ncols, dtype=torch.bfloat16, device=src.device)
    if drop is not None:
        N.call('asr_convert_rows_bf16_dropout', N.ptr(src), rmap, int(nrows), int(ncols),
               N.ptr(out), float(drop[0]), int(drop[1]), N.stream_handle(src.device))
    else:
        N.call('asr_convert_rows_bf16', N.ptr(src), rmap, int(nrows), int(ncols), N.ptr(out),
               N.stream_handle(src.device))
    return out


def fuse_dropout_ok():
    """Inter-layer dropout is folded into the next BLSTM layer's bf16 input
    staging (bf16 mode; ASR_FUSE_DROPOUT=0 keeps the separate pass)."""
    return compute_dtype() == BF16 and os.environ.get('ASR_FUSE_DROPOUT', '1') != '0'


def _blstm_wgrad(dg, dg_f32, x_op, x_map, y_op, T, gbufs, dev):
    """dW_ih, dW_hh of one BLSTM layer from its gate gradients (dg: bf16 copy
    in bf16 mode, else the f32 tensor).  db_ih / db_hh were accumulated by
    asr_lstm_backward_db."""
    B = dg.shape[0]
    H = y_op.shape[2] // 2
    BT = B * T
    g_ih, g_hh, g_bih, g_bhh = gbufs
    Din = g_ih.shape[-1]          # != x_op's width for 'concat' input rows
    # dW_ih [8H, Din] += dG^T x   (both directions in one problem)
    run_gemm([gemm_problem(operand(dg, 1, rowmap(8 * H)), operand(x_op, 1, x_map), g_ih,
                           rowmap(Din), 8 * H, Din, BT, beta=1.0)], dev)
    # dW_hh[dir] += dG_dir^T h_prev_dir ; h_prev = y[b, t-1, :H] (fwd), y[b, t+1, H:] (rev)
    hp_f = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=-1, t_limit=T)
    hp_r = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=1, t_limit=T)
    run_gemm([
        gemm_problem(operand(dg, 1, rowmap(8 * H)), operand(y_op, 1, hp_f), g_hh, rowmap(H),
                     4 * H, H, BT, beta=1.0),
        gemm_problem(operand(dg, 1, rowmap(8 * H), offset=4 * H),
                     operand(y_op, 1, hp_r, offset=H), g_hh, rowmap(H), 4 * H, H, BT, beta=1.0,
                     c_offset=4 * H * H),
    ], dev)


def _blstm_wgrad_rows(dg, x_op, Dx, y_op, T, gbufs, dev, ta, tb):
    """_blstm_wgrad over the rows (b, t), t in [ta, tb), of every utterance
    (bf16 mode: dg and x_op dense [B*T, width] rows): the weight gradients
    accumulated (beta = 1) from that band of time steps only."""
    B = dg.shape[0]
    H = y_op.shape[2] // 2
    n = tb - ta
    if n <= 0:
        return
    g_ih, g_hh, g_bih, g_bhh = gbufs
    Din = g_ih.shape[-1]
    band = lambda ld, add=0: rowmap(ld, stride_b=T * ld, rows_per_b=n, t_add=ta + add,  # noqa: E731
                                    t_limit=T)
    run_gemm([gemm_problem(operand(dg, 1, band(8 * H)), operand(x_op, 1, band(Dx)), g_ih,
                           rowmap(Din), 8 * H, Din, B * n, beta=1.0)], dev)
    run_gemm([
        gemm_problem(operand(dg, 1, band(8 * H)), operand(y_op, 1, band(2 * H, -1)), g_hh,
                     rowmap(H), 4 * H, H, B * n, beta=1.0),
        gemm_problem(operand(dg, 1, band(8 * H), offset=4 * H),
                     operand(y_op, 1, band(2 * H, 1), offset=H), g_hh, rowmap(H), 4 * H, H,
                     B * n, beta=1.0, c_offset=4 * H * H),
    ], dev)


def _wgrad_split_ok(ctx, T, mode):
    """The bottom BLSTM layer's weight gradients in three time bands (round 6,
    opt-in ASR_WGRAD_SPLIT=1; measured slower at ctc5x512, 17.48 vs 17.42
    ms/step: the band beside the recurrence costs it more than the 120 us it
    takes off the tail): the middle band [T/4, 3T/4) on the side
    stream beside the last quarter of the layer's own backward recurrence
    (gated on its progress report, mode 3), then [0, T/4) and [3T/4, T) on
    the compute stream -- in that order in every mode, so the sums are the
    same arithmetic with or without the overlap.  bf16 mode (dense staged
    operands), a layer with no recurrence left below it."""
    return (os.environ.get('ASR_WGRAD_SPLIT', '0') == '1' and not ctx.next_rec and T >= 64
            and compute_dtype() == BF16)


_side_streams = {}
_side_pending = []     # (side stream, gbufs, compute stream) of weight gradients not joined yet


def _join_side_wgrads(dev, notify=True):
    """Make the compute stream wait for the side-stream weight gradients
    enqueued so far; notify 'grads' for each (gradient-ready buckets)."""
    if not _side_pending:
        return
    for side, gbufs, main in _side_pending:
        main.wait_stream(side)
        if notify:
            notify_grad_event('grads', gbufs)
    del _side_pending[:]


def discard_side_wgrads():
    """After a backward that raised: make each compute stream wait for the
    side-stream weight gradients still pending (so a later zero of the flat
    gradient cannot race a beta = 1 accumulation) and forget them WITHOUT
    notifying 'grads' (their values belong to the skipped batch; a bucket
    hook must not see them as ready).  The end-of-backward join callback of
    a failed backward never runs, so nothing else would clear them."""
    for side, _gbufs, main in _side_pending:
        main.wait_stream(side)
    del _side_pending[:]


_warned = set()


def _warn_once(msg):
    if msg not in _warned:
        _warned.add(msg)
        import warnings
        warnings.warn(msg, RuntimeWarning, stacklevel=3)


def _num_cus(dev):
    return torch.cuda.get_device_properties(dev).multi_processor_count


def _xg_grid(B, H, ncu, xu=16):
    """Work-groups of the persistent recurrence (lstm_xg.hip xg_rows): groups of
    R = 8 utterances (16 when 8 would not fit) x direction x H / xu slices --
    the backward's xu = 32 (asr_lstm_backward_grid) only with R = 8, H <= 512."""
    if H % 32 or H // 16 > 64 or os.environ.get('ASR_LSTM_XG', '1') == '0':
        return 1 << 30        # not the tagged-granule recurrence
    for R in (8, 16):
        g = 2 * ((B + R - 1) // R) * (H // 16)
        if g <= ncu:
            if xu == 32:
                return g // 2 if R == 8 and H <= 512 else 1 << 30
            return g
    return 1 << 30


def _overlap_plan(dev, B, H):
    """(mode, units): the resolved ASR_OVERLAP_WGRAD mode for a BLSTM layer's
    backward and the hidden units per work-group of its backward recurrence.
    Modes:
      '0'  weight gradients on the compute stream;
      '1'  a CU-masked side stream (upper half of the CUs), only when the
           persistent backward recurrence fits in the other half;
      '2'  (opt-in) a plain side stream whose GEMMs use the 128 x 128 kernel
           (64 KB of LDS) while the recurrence pins 84 KB, so GEMM work-groups
           are co-resident with the recurrence's on every CU (rounds 3-4: wrong
           values, a gfx950 packed-FP32 hazard the library no longer contains,
           DESIGN.md §5; bitwise mode 0 since, tests/test_coresidency_gpu.py);
      '3'  a plain side stream with the recurrence at its default 140 KB pin,
           so no GEMM work-group can share a CU with it: the weight-gradient
           GEMMs run on the CUs the recurrence leaves free.
    auto = '3' when the recurrence leaves at least 32 CUs free -- with 16 units
    per work-group (the H = 320 configs: 160 of 256 CUs) or else with 32
    (ctc5x512: 128 of 256 CUs; ASR_XG_BWD_XU=16 keeps 16 and mode '0') --
    otherwise '0'.  Units: ASR_XG_BWD_XU=16|32 forces them; auto takes 32 only
    for mode 3 when 16 would leave fewer than 32 CUs.  All modes need bf16 and
    the persistent recurrence."""
    mode = os.environ.get('ASR_OVERLAP_WGRAD', 'auto')
    xu_env = os.environ.get('ASR_XG_BWD_XU', 'auto')
    forced = 32 if xu_env == '32' else 16
    if compute_dtype() != BF16 or os.environ.get('ASR_LSTM_PERSIST', '1') == '0' or H % 32:
        return '0', forced
    ncu = _num_cus(dev)
    roomy16 = _xg_grid(B, H, ncu) + 32 <= ncu
    roomy32 = _xg_grid(B, H, ncu, 32) + 32 <= ncu
    if mode == 'auto':
        mode = '3' if roomy16 or (xu_env != '16' and roomy32) else '0'
    if mode == '1' and _xg_grid(B, H, 2 * (ncu - ncu // 2)) > ncu // 2:
        mode = '0'
    mode = mode if mode in ('1', '2', '3') else '0'
    if xu_env in ('16', '32'):
        return mode, forced
    return mode, (32 if mode == '3' and not roomy16 and roomy32 else 16)


def _overlap_mode(dev, B, H):
    """The resolved ASR_OVERLAP_WGRAD mode (see _overlap_plan)."""
    return _overlap_plan(dev, B, H)[0]


def _wgrad_side_stream(dev, B, H):
    """Where the weight-gradient GEMMs of a BLSTM layer's backward run:
    (stream, small_tiles, gated) or None (the compute stream); see
    _overlap_mode.  gated: the GEMMs wait for the next recurrence to be
    resident (asr_lstm_wgrad_gate) so they take the CUs it leaves free rather
    than CUs it needs."""
    mode = _overlap_mode(dev, B, H)
    if mode == '0':
        return None
    key = (dev.index, mode)
    ent = _side_streams.get(key)
    if ent is None:
        ncu = _num_cus(dev)
        if mode == '1':
            h = ctypes.c_void_p()
            with torch.cuda.device(dev):
                N.call('asr_stream_create_cu_masked', ncu // 2, ncu - ncu // 2, ctypes.byref(h))
            ent = torch.cuda.ExternalStream(h.value, device=dev)
        else:
            ent = torch.cuda.Stream(device=dev)
        _side_streams[key] = ent
    return ent, mode == '2', mode != '1'


_progress = {}   # device index -> [uint64 counter (device), running total of arrivals]


def _progress_counter(dev):
    ent = _progress.get(dev.index)
    if ent is None:
        ent = _progress[dev.index] = [torch.zeros(1, dtype=torch.int64, device=dev), 0]
    return ent


def _dx_split_chunks():
    """Row chunks the split input gradient computes beside the recurrence:
    ASR_DX_SPLIT=1 one ([T/4, 3T/4)), 2 two (and [T/8, T/4) + [3T/4, 7T/8))."""
    return 2 if os.environ.get('ASR_DX_SPLIT', '1') == '2' else 1


def _dx_split_ok(ctx, B, T, dev, mode):
    """Split input gradient (round 6, ASR_DX_SPLIT=0 turns it off): the
    backward recurrence reports when the gate gradients of the middle rows t in
    [T/4, 3T/4) are final (processing step 3T/4 - 1 of both directions), and
    their share of dX = dG W_ih runs on the weight-gradient side stream beside
    the last quarter of that recurrence, on the CUs it leaves free (mode 3);
    the outer rows follow on the compute stream.  Needs the packed-activation
    tagged-granule backward (the one that reports progress).  In the other
    overlap modes the same row bands run after the recurrence, so dX is the
    same arithmetic in every mode."""
    return (os.environ.get('ASR_DX_SPLIT', '1') != '0' and T >= 64
            and compute_dtype() == BF16 and ctx.needs_input_grad[0])


DX_CHUNK = int(os.environ.get('ASR_DX_CHUNK', '64'))   # processing steps per pipelined dX chunk
_dx_state = {}


def _dx_pipeline_ok(ctx, B, T, Din, dev):
    """The input gradient of this layer feeds only the backward recurrence of
    the BLSTM layer below (its input was handed over as bf16), that recurrence
    is the packed-activation tagged-granule kernel and it leaves >= 32 CUs
    free: dX may then be computed beside it.  Opt-in (ASR_DX_PIPE=1): at 5x512
    the free half of the chip runs these GEMMs and the weight gradients too
    slowly to stay ahead of the recurrence."""
    if not getattr(ctx, 'handoff_in', False) or os.environ.get('ASR_DX_PIPE', '0') not in ('1', '2'):
        return False
    if Din % 2 or not _act_h_on() or compute_dtype() != BF16 or (T + 1) // 2 > 4096 * DX_CHUNK:
        return False
    # the GEMMs need CUs beside that recurrence (140 KB LDS pin: none on its CUs)
    _, xu = _overlap_plan(dev, B, Din // 2)
    grid = N.query('asr_lstm_backward_grid', B, Din // 2, xu)
    return grid > 0 and grid + 32 <= _num_cus(dev)


def _dx_pipelined(dx, dg_op, w_op, B, T, H, Din, Dp, drop, dev):
    """dX [B, T, Din] = dG W_ih in chunks of time steps from both ends of the
    sequence inwards -- the order in which the layer below's backward
    recurrence reads them (steps q: rows t = q and T - 1 - q) -- each chunk
    signalled by a flag (asr_lstm_dy_signal) the recurrence polls before
    reading its dy rows.  ASR_DX_PIPE=1: every chunk (ASR_DX_CHUNK steps) on a
    high-priority side stream that first waits for that recurrence to be
    resident (asr_lstm_wgrad_gate), so the GEMMs take the CUs it leaves free.
    ASR_DX_PIPE=2: two chunks of about T / 4 steps -- the outer rows on the
    main stream with the whole chip before the recurrence is launched, the
    middle rows beside it, where the recurrence reaches them ~T/4 steps later.
    dx carries (flags, c0, epoch, done-event) as _asr_dy_pipe."""
    st = _dx_state.get(dev.index)
    if st is None:
        st = {'flags': torch.zeros(4096, dtype=torch.int32, device=dev),
              'stream': torch.cuda.Stream(device=dev, priority=-1), 'epoch': 0}
        _dx_state[dev.index] = st
    st['epoch'] = st['epoch'] % 0x7ffffff0 + 1
    epoch, flags, side = st['epoch'], st['flags'], st['stream']
    main = torch.cuda.current_stream(dev)
    half = (T + 1) // 2
    head_main = os.environ.get('ASR_DX_PIPE', '0') == '2'
    c0 = DX_CHUNK
    if head_main and 'ASR_DX_CHUNK' not in os.environ:
        c0 = (half + 1) // 2

    def chunk(k):
        s0, s1 = k * c0, (k + 1) * c0
        probs = []
        for t0, t1 in ((s0, min(s1, half)), (max(T - s1, half), T - s0)):
            if t1 <= t0:
                continue
            n = t1 - t0
            a = operand(dg_op, 0, rowmap(8 * H, stride_b=T * 8 * H, rows_per_b=n, t_add=t0))
            c_map = rowmap(Din, stride_b=T * Din, rows_per_b=n, t_add=t0)
            probs.append(gemm_problem(a, operand(w_op, 1, rowmap(Dp)), dx, c_map, B * n,
                                      Din, 8 * H, drop=drop))
        run_gemm(probs, dev)
        N.call('asr_lstm_dy_signal', N.ptr(flags), k, epoch, N.stream_handle(dev))

    nch = (half + c0 - 1) // c0
    k0 = 0
    if head_main:   # the first chunk with the whole chip, before the recurrence
        chunk(0)
        k0 = 1
    side.wait_stream(main)
    small = os.environ.get('ASR_DX_SMALL', '1') != '0'   # 128 x 128 tiles: more work-groups
    with torch.cuda.stream(side):
        if k0 < nch:
            N.call('asr_lstm_wgrad_gate', N.stream_handle(dev))
        if small:
            N.call('asr_gemm_set_small_tiles', 1)
        try:
            for k in range(k0, nch):
                chunk(k)
        finally:
            if small:
                N.call('asr_gemm_set_small_tiles', 0)
        done = torch.cuda.Event()
        done.record(side)
    for t in (dx, dg_op, w_op, flags):
        t.record_stream(side)
    dx._asr_dy_pipe = (flags, c0, epoch, done)
    return done


def blstm_layer(x_src, lens, T, w_ih, w_hh, b_ih, b_hh, perm=None, t_mul=1, t_add=0, gbufs=None,
                graph_params=(), concat=False, drop=None, next_rec=False, bf16_handoff=False,
                out_drop=None):
    """gbufs: optional (g_w_ih, g_w_hh, g_b_ih, g_b_hh) gradient views to accumulate
    into; default: the tensors' own .grad.  graph_params: the nn.Parameters the
    combined [fwd; rev] views alias -- passed only so autograd records that the
    output depends on them (their gradients are written by the kernels).
    concat: input row t is [x_src[t*t_mul + t_add]; x_src[t*t_mul + t_add + 1]]
    ('concat' subsampling of the previous layer, read in place).
    drop: optional (p, seed): the layer reads dropout(x_src) (asr_dropout's mask),
    fused into the bf16 input staging; its input gradient gets the same mask.
    next_rec: another BLSTM layer's backward recurrence follows this layer's in
    the backward pass (the layer below), so ASR_OVERLAP_WGRAD=2 can run this
    layer's weight gradients beside it.
    bf16_handoff: the output's only consumer is the next BLSTM layer, reading
    it through an identity row map with drop=out_drop (its fused dropout, or
    None): in bf16 mode the fused forward then writes that layer's staged
    bf16 input (dropout applied) instead of the f32 output, whose tensor is
    returned unwritten (for autograd; reading it otherwise raises in the next
    layer, and no other consumer may read it)."""
    spec = (not (bf16_handoff and compute_dtype() == BF16 and handoff_on()),
            out_drop if bf16_handoff else None)
    return BLSTMLayerFn.apply(x_src, lens, T, perm, t_mul, t_add, gbufs, bool(concat), drop,
                              bool(next_rec), spec, w_ih, w_hh, b_ih, b_hh, *graph_params)


def handoff_on():
    """ASR_BF16_HANDOFF=0: every BLSTM layer writes its f32 output and the next
    layer stages it (A/B)."""
    return os.environ.get('ASR_BF16_HANDOFF', '1') != '0'


def _handoff_input(x_src, perm, t_mul, t_add, T, concat, drop, din):
    """The bf16 tensor a BLSTM layer's input was handed over as (see
    blstm_layer's bf16_handoff), or None for an ordinary f32 input.  Raises if
    the input was handed over but this layer cannot read it that way (its f32
    values were never written)."""
    h = getattr(x_src, '_asr_handoff', None)
    if h is None:
        return None
    t, hdrop = h
    B = x_src.shape[0]
    ok = (compute_dtype() == BF16 and perm is None and t_mul == 1 and t_add == 0 and
          not concat and x_src.shape[1] == T and x_src.shape[2] == din and din % 8 == 0 and
          drop == hdrop and t.shape == (B, T, din))
    if not ok:
        raise N.NativeError('BLSTM layer input was handed over as bf16 (its f32 values were '
                            'not written) but this layer cannot stage it that way')
    return t


# ---------------------------------------------------------------------------
# Elementwise: dropout (counter RNG), tanh, embedding
# ---------------------------------------------------------------------------
_seed = {'v': 1623}


def manual_seed(seed):
    _seed['v'] = int(seed)


_seed_log = {'on': False, 'seeds': []}   # tests: record the dropout seeds a step drew


def _next_seed():
    _seed['v'] = (_seed['v'] * 6364136223846793005 + 1442695040888963407) % (1 << 64)
    if _seed_log['on']:
        _seed_log['seeds'].append(_seed['v'])
    return _seed['v']


class DropoutFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, p, seed=None):
        N.require_device(x)
        x = x.contiguous()
        y = torch.empty_like(x)
        seed = _next_seed() if seed is None else int(seed)
        N.call('asr_dropout', N.ptr(x), N.ptr(y), x.numel(), float(p), seed,
               N.stream_handle(x.device))
        ctx.meta = (float(p), seed)
        return y

    @staticmethod
    def backward(ctx, dy):
        p, seed = ctx.meta
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        N.call('asr_dropout', N.ptr(dy), N.ptr(dx), dy.numel(), p, seed,
               N.stream_handle(dy.device))
        return dx, None, None


def dropout(x, p, seed=None):
    """nn.Dropout in training mode; element i of x is kept iff the counter RNG
    u01(seed, i) >= p (seed drawn from the module stream unless given)."""
    return DropoutFn.apply(x, p, seed) if p > 0 else x


def next_seed():
    return _next_seed()


class AddTanhFn(torch.autograd.Function):
    """y = tanh(a + b), one pass; d a = d b = dy (1 - y^2)."""

    @staticmethod
    def forward(ctx, a, b):
        N.require_device(a, b)
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.call('asr_add_tanh_forward', N.ptr(a), N.ptr(b), N.ptr(y), y.numel(),
               N.stream_handle(a.device))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        N.call('asr_tanh_backward', N.ptr(y), N.ptr(dy), N.ptr(dx), y.numel(),
               N.stream_handle(y.device))
        return dx, dx


def add_tanh(a, b):
    return AddTanhFn.apply(a, b)


class AddFn(torch.autograd.Function):
    """y = a + b (residual connections); d a = d b = dy."""

    @staticmethod
    def forward(ctx, a, b):
        N.require_device(a, b)
        a, b = a.contiguous(), b.contiguous()
        y = torch.empty_like(a)
        N.call('asr_add_forward', N.ptr(a), N.ptr(b), N.ptr(y), y.numel(),
               N.stream_handle(a.device))
        return y

    @staticmethod
    def backward(ctx, dy):
        return dy, dy


def add(a, b):
    return AddFn.apply(a, b)


class AddBatchSumFn(torch.autograd.Function):
    """y[b] = h[b] + sum_b' lower[b'] -- the reference decoder's residual
    connection ``hx_list[l] += sum(hx_list[l - 1])`` (rnn_decoder.py:100-102),
    where Python's sum runs over the BATCH dimension of the lower layer's
    output.  Both sums are [1 x B] x [B x D] products and the broadcast is a
    K = 1 product accumulated onto a copy of h (asr_gemm)."""

    @staticmethod
    def _bsum_bcast(x, out):
        """out[b] += sum_b' x[b'] for x, out [B, D] (out already holds the addend)."""
        B, D = x.shape
        dev = x.device
        ones = torch.ones(B, 1, dtype=torch.float32, device=dev)
        sm = torch.empty(1, D, dtype=torch.float32, device=dev)
        run_gemm([gemm_problem(operand(ones, 1, rowmap(1)), operand(x, 1, rowmap(D)), sm,
                               rowmap(D), 1, D, B)], dev)
        run_gemm([gemm_problem(operand(ones, 0, rowmap(1)), operand(sm, 1, rowmap(D)), out,
                               rowmap(D), B, D, 1, beta=1.0)], dev)
        return out

    @staticmethod
    def forward(ctx, h, lower):
        N.require_device(h, lower)
        return AddBatchSumFn._bsum_bcast(lower.contiguous(), h.contiguous().clone())

    @staticmethod
    def backward(ctx, dy):
        dy = dy.contiguous()
        return dy, AddBatchSumFn._bsum_bcast(dy, torch.zeros_like(dy))


def add_batch_sum(h, lower):
    return AddBatchSumFn.apply(h, lower)


class TanhFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        N.require_device(x)
        x = x.contiguous()
        y = torch.empty_like(x)
        N.call('asr_tanh_forward', N.ptr(x), N.ptr(y), x.numel(), N.stream_handle(x.device))
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        y, = ctx.saved_tensors
        dy = dy.contiguous()
        dx = torch.empty_like(dy)
        N.call('asr_tanh_backward', N.ptr(y), N.ptr(dy), N.ptr(dx), y.numel(),
               N.stream_handle(y.device))
        return dx


def tanh(x):
    return TanhFn.apply(x)


class EmbeddingFn(torch.autograd.Function):
    """trans=0: weight [V, E] (nn.Embedding); trans=1: weight [E, V] (Embedding_LS).
    idx_host (optional numpy copy of idx): the backward groups rows by token on
    the host (CSR) instead of scanning every row per (token, column)."""

    @staticmethod
    def forward(ctx, idx, weight, trans, padding_idx, idx_host=None):
        N.require_device(idx, weight)
        idx = idx.contiguous().long()
        V, E = (weight.shape[1], weight.shape[0]) if trans else weight.shape
        out = torch.empty(*idx.shape, E, dtype=torch.float32, device=idx.device)
        N.call('asr_embedding_forward', N.ptr(idx), N.ptr(weight), idx.numel(), V, E, int(trans),
               N.ptr(out), N.stream_handle(idx.device))
        ctx.save_for_backward(idx, weight)
        ctx.meta = (trans, padding_idx, V, E, idx_host)
        ctx.beside = _beside_plan[0]
        return out

    @staticmethod
    def backward(ctx, dout):
        idx, weight = ctx.saved_tensors
        trans, padding_idx, V, E, idx_host = ctx.meta
        dout = dout.contiguous()
        pad = -1 if padding_idx is None else int(padding_idx)
        dev = idx.device
        if idx_host is not None:
            flat = np.clip(np.asarray(idx_host, np.int64).reshape(-1), 0, V - 1)
            order = np.argsort(flat, kind='stable').astype(np.int32)
            starts = np.zeros(V + 1, np.int32)
            np.cumsum(np.bincount(flat, minlength=V), out=starts[1:])
            order_d = h2d(order, dev)
            starts_d = h2d(starts, dev)

            def wgrad():
                N.call('asr_embedding_backward_csr', N.ptr(order_d), N.ptr(starts_d), N.ptr(dout),
                       V, E, int(trans), pad, N.ptr(grad_buffer(weight)), N.stream_handle(dev))
            keep = (order_d, starts_d, dout)
        else:
            def wgrad():
                N.call('asr_embedding_backward', N.ptr(idx), N.ptr(dout), idx.numel(), V, E,
                       int(trans), pad, N.ptr(grad_buffer(weight)), N.stream_handle(dev))
            keep = (idx, dout)
        # the embedding gradient has no consumer but the optimizer: beside the
        # encoder's top backward recurrence when the decoder is built under
        # wgrad_beside_encoder
        if ctx.beside is None or not _wgrad_beside(dev, ctx.beside, wgrad, keep,
                                                   (grad_buffer(weight),)):
            wgrad()
        return None, None, None, None, None


def embedding(idx, weight, padding_idx=None, idx_host=None):
    return EmbeddingFn.apply(idx, weight, 0, padding_idx, idx_host)


def embedding_t(idx, weight_ev, idx_host=None):
    return EmbeddingFn.apply(idx, weight_ev, 1, None, idx_host)


class CTCLossFn(torch.autograd.Function):
    """loss = loss_scale * sum_b CTC(logits_b, labels_b); logits [B, T, V] f32
    batch-major (no time-major transpose copy).  The gradient is produced in
    backward, already multiplied by grad_output * loss_scale, in one write."""

    @staticmethod
    def forward(ctx, logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale,
                blank=0, zero_infinity=True):
        N.require_device(logits, labels_flat, label_lens, act_lens)
        logits = logits.contiguous()
        B, T, V = logits.shape
        nbytes = N.query('asr_ctc_workspace_bytes', T, B, V, max_label_len)
        ws = _ws(nbytes, logits.device)
        costs = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty(1, dtype=torch.float32, device=logits.device)
        N.call('asr_ctc_forward', N.ptr(logits), V, T * V, T, B, V, N.ptr(labels_flat),
               N.ptr(label_lens), N.ptr(act_lens), int(max_label_len), int(blank),
               int(bool(zero_infinity)), N.ptr(costs), N.ptr(loss), float(loss_scale), N.ptr(ws),
               nbytes, N.stream_handle(logits.device))
        ctx.save_for_backward(logits, labels_flat, label_lens, act_lens, ws)
        ctx.meta = (int(max_label_len), int(blank), float(loss_scale), nbytes)
        ctx.mark_non_differentiable(costs)
        return loss, costs

    @staticmethod
    def backward(ctx, g_loss, g_costs):
        logits, labels_flat, label_lens, act_lens, ws = ctx.saved_tensors
        max_label_len, blank, loss_scale, nbytes = ctx.meta
        B, T, V = logits.shape
        grads = torch.empty_like(logits)
        g = g_loss.contiguous() if g_loss is not None else None
        N.call('asr_ctc_backward', N.ptr(logits), V, T * V, T, B, V, N.ptr(labels_flat),
               N.ptr(label_lens), N.ptr(act_lens), max_label_len, blank, N.ptr(g),
               loss_scale if g is not None else 0.0, N.ptr(grads), V, T * V, N.ptr(ws), nbytes,
               N.stream_handle(logits.device))
        return grads, None, None, None, None, None, None, None


class XentFn(torch.autograd.Function):
    """Fused CE (ignore -1) + uniform label smoothing over rows of logits."""

    @staticmethod
    def forward(ctx, logits, targets, lens, T, ce_scale, ls_scale):
        N.require_device(logits)
        logits = logits.contiguous()
        V = logits.shape[-1]
        R = logits.numel() // V
        nb = N.query('asr_xent_workspace_bytes', R)
        ws = _ws(nb, logits.device)
        loss = torch.empty(1, dtype=torch.float32, device=logits.device)
        tg = targets.contiguous().long() if targets is not None else None
        ln = lens.contiguous().int() if lens is not None else None
        N.call('asr_xent_forward', N.ptr(logits), R, V, int(T), N.ptr(tg), N.ptr(ln),
               float(ce_scale), float(ls_scale), N.ptr(loss), N.ptr(ws), nb,
               N.stream_handle(logits.device))
        ctx.save_for_backward(logits, ws)
        ctx.meta = (tg, ln, int(T), float(ce_scale), float(ls_scale), nb)
        return loss

    @staticmethod
    def backward(ctx, g):
        logits, ws = ctx.saved_tensors
        tg, ln, T, ce_scale, ls_scale, nb = ctx.meta
        V = logits.shape[-1]
        R = logits.numel() // V
        d = torch.empty_like(logits)
        g = g.contiguous()
        N.call('asr_xent_backward', N.ptr(logits), R, V, T, N.ptr(tg), N.ptr(ln), ce_scale,
               ls_scale, N.ptr(g), 1.0, N.ptr(d), N.ptr(ws), nb, N.stream_handle(logits.device))
        return d, None, None, None, None, None


def xent(logits, targets=None, lens=None, T=0, ce_scale=1.0, ls_scale=0.0):
    """Returns loss [1] = ce_scale * CE_sum + ls_scale * LS_sum (see asr_xent_forward)."""
    return XentFn.apply(logits, targets, lens, T, ce_scale, ls_scale)


def softmax(x):
    N.require_device(x)
    x = x.contiguous()
    y = torch.empty_like(x)
    V = x.shape[-1]
    N.call('asr_softmax', N.ptr(x), x.numel() // V, V, N.ptr(y), N.stream_handle(x.device))
    return y


def ctc_best_path(logits, lens, blank=0):
    """CTC greedy best path on device: returns (hyps int32 [B, T], hyp_lens int32 [B])."""
    N.require_device(logits, lens)
    logits = logits.contiguous()
    B, T, V = logits.shape
    hyps = torch.empty(B, T, dtype=torch.int32, device=logits.device)
    hl = torch.empty(B, dtype=torch.int32, device=logits.device)
    N.call('asr_ctc_best_path', N.ptr(logits), V, T * V, T, B, V, N.ptr(lens.int().contiguous()),
           int(blank), N.ptr(hyps), N.ptr(hl), N.stream_handle(logits.device))
    return hyps, hl


def row_argmax(x):
    N.require_device(x)
    x = x.contiguous()
    V = x.shape[-1]
    out = torch.empty(x.shape[:-1], dtype=torch.int64, device=x.device)
    N.call('asr_row_argmax', N.ptr(x), x.numel() // V, V, N.ptr(out), N.stream_handle(x.device))
    return out


def ctc_loss(logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale=1.0, blank=0,
             zero_infinity=True):
    """Returns (loss [1], costs [B])."""
    return CTCLossFn.apply(logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale,
                           blank, zero_infinity)


# ---------------------------------------------------------------------------
# VGG front-end (CNNEncoder, models/pytorch_v3/encoders/cnn.py:124-165)
# ---------------------------------------------------------------------------
def _tap_operand(t, trans, stride, group, pitch, sign):
    op = operand(t, trans, rowmap(stride))
    op.tap_group, op.tap_pitch, op.tap_sign = int(group), int(pitch), int(sign)
    return op


def _pool_dims(T, F, pt, pf, ceil):
    To, Fo = ctypes.c_int(), ctypes.c_int()
    N.call('asr_vgg_pool_dims', T, F, pt, pf, ceil, ctypes.byref(To), ctypes.byref(Fo))
    return To.value, Fo.value


def _halo_only(C, dtype):
    """A padded VGG operand whose producer writes every interior pixel needs
    only its halo zeroed (16-B rows; ASR_VGG_HALO_ONLY=0 zero-fills it whole)."""
    size = 2 if dtype == torch.bfloat16 else 4
    return C % 4 == 0 and (C * size) % 16 == 0 and os.environ.get('ASR_VGG_HALO_ONLY', '1') != '0'


def _zero_halo(buf, B, T, F, C):
    N.call('asr_vgg_zero_halo', N.ptr(buf), BF16 if buf.dtype == torch.bfloat16 else F32, int(B),
           int(T), int(F), int(C), N.stream_handle(buf.device))


_TWO_GIB = 1 << 31


def _conv_tr_ok(cin, cout, fp, P, out_bytes):
    """bf16 mode: the tap-resident convolution kernel (csrc/conv.hip) takes this
    channel pair and operand sizes -- every operand below 2 GiB, the kernel's
    buffer-resource limit (ASR_VGG_TR=0 keeps the tap-addressed GEMM, for A/B)."""
    return (compute_dtype() == BF16 and os.environ.get('ASR_VGG_TR', '1') != '0' and
            P * cin * 2 < _TWO_GIB and P * cout * out_bytes < _TWO_GIB and
            N.query('asr_conv3x3_tr_supported', int(cin), int(cout), int(fp)) == 1)


def _c1_wgrad_ok(B, T, F, co):
    """The first layer's weight gradient from the raw features
    (asr_conv3x3_c1_wgrad_xs) takes this shape: 64 output channels, the bf16 dz
    operand below 2 GiB and the LDS tile of one frequency row (F) within 64 KB;
    decided in the forward, which then skips the padded operand."""
    P = B * (T + 2) * (F + 2)
    lds = 256 * co * 2 + (256 + 2 * (F + 3)) * 4
    return co == 64 and P * co * 2 < _TWO_GIB and lds <= 64 * 1024


def conv3x3_tr(inp, P, cin, fp, sign, w, cout, bias, out):
    """out[p][n] = bias[n] + sum_tap sum_c inp[p + sign*shift(tap)][c] w[n][tap cin + c]
    on the tap-resident kernel (asr_conv3x3_tr); inp / w bf16, out f32 or bf16."""
    N.require_device(inp, w, out)
    od = BF16 if out.dtype == torch.bfloat16 else F32
    N.call('asr_conv3x3_tr', N.ptr(inp), int(P), int(cin), int(fp), int(sign), N.ptr(w),
           int(cout), N.ptr(bias), N.ptr(out), od, N.stream_handle(inp.device))


def conv3x3_tr_wgrad(x, dz, P, cin, fp, cout, packed):
    """packed[n][tap cin + c] = sum_p dz[p][n] x[p + shift(tap)][c] on the
    tap-resident weight-gradient kernel; False when the shape does not take it."""
    if compute_dtype() != BF16 or os.environ.get('ASR_VGG_TR', '1') == '0':
        return False
    if P * cin * 2 >= _TWO_GIB or P * cout * 2 >= _TWO_GIB:   # the kernel's buffer limit
        return False
    nb = N.query('asr_conv3x3_tr_wgrad_workspace_bytes', int(P), int(cin), int(cout), int(fp))
    if not nb:
        return False
    N.require_device(x, dz, packed)
    ws = _ws(nb, x.device)
    N.call('asr_conv3x3_tr_wgrad', N.ptr(x), N.ptr(dz), int(P), int(cin), int(fp), int(cout),
           N.ptr(packed), N.ptr(ws), nb, N.stream_handle(x.device))
    return True


class VGGFn(torch.autograd.Function):
    """The whole conv stack as one op.  Layer l input: zero-haloed channels-last
    [B][T_l+2][F_l+2][C_in] (compute dtype for GEMM layers, f32 for direct
    ones); conv output z_l f32 over the same padded pixels; the 3x3 conv of a
    layer with C_in, C_out multiples of 16 = ONE GEMM with tap-addressed
    operands (csrc/gemm.hip), other layers (C_in = 1) = asr_conv_direct_*;
    ReLU, pool, batch norm and dropout = asr_vgg_block_*.  Output
    [B, T', F'*C] f32."""

    @staticmethod
    def forward(ctx, xs, specs, training, p_drop, *params):
        N.require_device(xs)
        xs = xs.contiguous()
        dev = xs.device
        cd = compute_dtype()
        B, T, F = xs.shape
        f32 = dict(dtype=torch.float32, device=dev)
        opdt = torch.bfloat16 if cd == BF16 else torch.float32
        # GEMM layers need C_in and C_out multiples of 16; the single input
        # channel of layer 0 is padded to 16 (zero channels, zero weights)
        use_gemm = [sp['w'].shape[0] % 16 == 0 and (sp['w'].shape[1] % 16 == 0 or l == 0)
                    for l, sp in enumerate(specs)]
        cC = 1
        cCp = 16 if use_gemm[0] else 1
        # bf16, 64-channel first layer: its forward stencil and its weight gradient
        # (asr_conv3x3_c1_wgrad_xs) both read the raw features, so the padded
        # 16-channel operand is never built
        co0 = specs[0]['w'].shape[0]
        c1w = (cd == BF16 and use_gemm[0] and _c1_wgrad_ok(B, T, F, co0) and
               os.environ.get('ASR_VGG_C1_DIRECT', '1') != '0' and
               os.environ.get('ASR_VGG_C1_XS', '1') != '0' and
               os.environ.get('ASR_VGG_C1_WGRAD', '1') != '0')
        if c1w:
            x_op = xs
        else:
            x_op = torch.empty(B * (T + 2) * (F + 2), cCp, dtype=opdt if use_gemm[0] else
                               torch.float32, device=dev)
            N.call('asr_vgg_pad_input_ch', N.ptr(xs), B, T, F, cCp, cd if use_gemm[0] else F32,
                   N.ptr(x_op), N.stream_handle(dev))
        ctx.c1w = c1w
        cT, cF = T, F
        saved, layers = [], []
        L = len(specs)
        for l, sp in enumerate(specs):
            w = sp['w']
            Co = w.shape[0]
            npad = B * (cT + 2) * (cF + 2)
            # bf16 mode: the GEMM / stencil layers write the conv output as bf16
            # (read twice more: ReLU + pool, and the ReLU mask in the backward)
            c1_xs = (use_gemm[l] and cC == 1 and Co % 4 == 0 and 256 % (Co // 4) == 0 and
                     os.environ.get('ASR_VGG_C1_DIRECT', '1') != '0' and
                     os.environ.get('ASR_VGG_C1_XS', '1') != '0')
            z_bf = (cd == BF16 and Co % 4 == 0 and (c1_xs or not (cC == 1)) and use_gemm[l] and
                    os.environ.get('ASR_VGG_Z_BF16', '1') != '0')
            pt, pf, ceil = sp['pt'], sp['pf'], sp['ceil']
            # unpooled stencil layer followed by batch norm: the stencil writes P and
            # the BN moment partials itself (asr_vgg_c1_forward_relu_p), no z
            c1p = (c1_xs and z_bf and not pt and sp['gamma'] is not None and Co % 8 == 0 and
                   (not training or sp['run_mean'] is not None) and
                   os.environ.get('ASR_VGG_P_BF16', '1') != '0' and
                   os.environ.get('ASR_VGG_ROWS', '1') != '0' and
                   os.environ.get('ASR_VGG_C1_RELU_P', '1') != '0')
            z = (None if c1p else
                 torch.empty(npad, Co, dtype=torch.bfloat16 if z_bf else torch.float32, device=dev))
            if c1p:
                P = torch.empty(B * cT * cF, Co, dtype=torch.bfloat16, device=dev)
                nblk = N.query('asr_vgg_c1_relu_p_blocks', B, cT)
                mqp = torch.empty(2, nblk, Co, **f32) if training else None
                N.call('asr_vgg_c1_forward_relu_p', N.ptr(xs), int(cd == BF16), B, cT, cF, Co,
                       N.ptr(w), N.ptr(sp['b']), N.ptr(P),
                       N.ptr(sp['run_mean']) if training else None,
                       N.ptr(mqp[0]) if training else None, N.ptr(mqp[1]) if training else None,
                       N.stream_handle(dev))
            elif not use_gemm[l]:
                N.call('asr_conv_direct_forward', N.ptr(x_op), B, cT, cF, cC, Co, N.ptr(w),
                       N.ptr(sp['b']), N.ptr(z), N.stream_handle(dev))
            elif cC == 1 and Co % 4 == 0 and os.environ.get('ASR_VGG_C1_DIRECT', '1') != '0':
                # one input channel: a direct stencil from channel 0 of the padded
                # operand (the GEMM would run K = 144 for 9 useful taps); the
                # backward still takes the weight-gradient GEMM over this operand
                if c1_xs:
                    # from the raw features (contiguous rows; rounded to bf16 as the
                    # staged operand is in bf16 mode)
                    N.call('asr_conv3x3_c1_forward_xs', N.ptr(xs), int(cd == BF16), B, cT, cF, Co,
                           N.ptr(w), N.ptr(sp['b']), N.ptr(z), BF16 if z_bf else F32,
                           N.stream_handle(dev))
                else:
                    N.call('asr_conv3x3_c1_forward', N.ptr(x_op), cd, cCp, B, cT, cF, Co,
                           N.ptr(w), N.ptr(sp['b']), N.ptr(z), N.stream_handle(dev))
            else:
                wg = (torch.zeros if cCp != cC else torch.empty)(Co, 9 * cCp, dtype=opdt,
                                                                 device=dev)
                N.call('asr_conv_weight_pack_pad', N.ptr(w), Co, cC, cCp, 0, cd, N.ptr(wg),
                       N.stream_handle(dev))
                if _conv_tr_ok(cCp, Co, cF + 2, npad, z.element_size()):
                    # the input rows stay in an LDS ring across the nine taps
                    conv3x3_tr(x_op, npad, cCp, cF + 2, 1, wg, Co, sp['b'], z)
                else:
                    p = gemm_problem(_tap_operand(x_op, 0, cCp, cCp, cF + 2, 1),
                                     operand(wg, 0, rowmap(9 * cCp)), z, rowmap(Co), npad, Co,
                                     9 * cCp, bias=sp['b'])
                    run_gemm([p], dev)
            To, Fo = _pool_dims(cT, cF, pt, pf, ceil) if pt else (cT, cF)
            # P = max(0, max z) of a bf16 z is itself a bf16 value: stored bf16 it
            # is exact and halves P's write and four reads
            p_bf = z_bf and os.environ.get('ASR_VGG_P_BF16', '1') != '0'
            if not c1p:
                P = torch.empty(B * To * Fo, Co, dtype=torch.bfloat16 if p_bf else torch.float32,
                                device=dev)
            slot = torch.empty(B * To * Fo * Co, dtype=torch.uint8, device=dev) if pt else None
            bn = sp['gamma'] is not None
            mean = torch.empty(Co, **f32) if bn else None
            rstd = torch.empty(Co, **f32) if bn else None
            drop = float(p_drop) if training else 0.0
            seed = _next_seed() if drop > 0 else 0
            last = l == L - 1
            if last:
                out = torch.empty(B, To, Fo * Co, **f32)
                out_dt, flat = F32, 1
            else:
                nxt_dt = opdt if use_gemm[l + 1] else torch.float32
                if _halo_only(Co, nxt_dt):
                    # the block kernel writes every interior pixel: zero only the halo
                    out = torch.empty(B * (To + 2) * (Fo + 2), Co, dtype=nxt_dt, device=dev)
                    _zero_halo(out, B, To, Fo, Co)
                else:
                    out = torch.zeros(B * (To + 2) * (Fo + 2), Co, dtype=nxt_dt, device=dev)
                out_dt, flat = (cd if use_gemm[l + 1] else F32), 0
            nb = N.query('asr_vgg_block_workspace_bytes', B, To, Fo, Co)
            ws = _ws(nb, dev)
            if c1p:
                N.call('asr_vgg_block_forward_given_p', N.ptr(P), B, cT, cF, Co,
                       N.ptr(sp['gamma']), N.ptr(sp['beta']), N.ptr(sp['run_mean']),
                       N.ptr(sp['run_var']), int(bool(training)), float(sp['momentum']),
                       float(sp['eps']), N.ptr(mean), N.ptr(rstd), drop, seed, N.ptr(out),
                       out_dt, flat, N.ptr(mqp[0]) if training else None,
                       N.ptr(mqp[1]) if training else None, nblk if training else 0, N.ptr(ws),
                       nb, N.stream_handle(dev))
                z = P     # the backward masks from P (asr_vgg_block_backward_zdp: z == P)
            else:
                N.call('asr_vgg_block_forward_zp', N.ptr(z), BF16 if z_bf else F32, B, cT, cF,
                       Co, pt, pf, ceil, N.ptr(P), BF16 if p_bf else F32, N.ptr(slot),
                       N.ptr(sp['gamma']), N.ptr(sp['beta']), N.ptr(sp['run_mean']),
                       N.ptr(sp['run_var']), int(bool(training)), float(sp['momentum']),
                       float(sp['eps']), N.ptr(mean), N.ptr(rstd), drop, seed, N.ptr(out),
                       out_dt, flat, N.ptr(ws), nb, N.stream_handle(dev))
            saved += [x_op, z, P, slot, mean, rstd]
            layers.append((cT, cF, cC, cCp, Co, pt, pf, ceil, drop, seed, use_gemm[l]))
            x_op, cT, cF, cC, cCp = out, To, Fo, Co, Co
        ctx.save_for_backward(*[t if t is not None else torch.empty(0, device=dev)
                                for t in saved])
        ctx.layers = layers
        ctx.specs = specs
        ctx.B = B
        return x_op

    @staticmethod
    def backward(ctx, dout):
        saved = ctx.saved_tensors
        specs, layers, B = ctx.specs, ctx.layers, ctx.B
        dev = dout.device
        cd = compute_dtype()
        f32 = dict(dtype=torch.float32, device=dev)
        opdt = torch.bfloat16 if cd == BF16 else torch.float32
        dnext, flat = dout.contiguous(), 1
        for l in range(len(layers) - 1, -1, -1):
            x_op, z, P, slot, mean, rstd = saved[6 * l:6 * l + 6]
            slot = slot if slot.numel() else None
            mean = mean if mean.numel() else None
            rstd = rstd if rstd.numel() else None
            cT, cF, cC, cCp, Co, pt, pf, ceil, drop, seed, gemm = layers[l]
            sp = specs[l]
            npad = B * (cT + 2) * (cF + 2)
            # dz is the GEMM operand (compute dtype) of GEMM layers; their conv
            # bias gradient is summed from the f32 values inside the kernel
            dz_f32 = not gemm
            if not dz_f32 and _halo_only(Co, opdt) and os.environ.get('ASR_VGG_POST_FULL',
                                                                   '1') != '0':
                # the full-resolution pass writes every interior pixel of dz
                dz = torch.empty(npad, Co, dtype=opdt, device=dev)
                _zero_halo(dz, B, cT, cF, Co)
            else:
                dz = torch.zeros(npad, Co, **f32) if dz_f32 else torch.zeros(npad, Co, dtype=opdt,
                                                                              device=dev)
            fused_bias = gemm and sp['b'] is not None
            To, Fo = _pool_dims(cT, cF, pt, pf, ceil) if pt else (cT, cF)
            nb = N.query('asr_vgg_block_workspace_bytes', B, To, Fo, Co)
            ws = _ws(nb, dev)
            bn = sp['gamma'] is not None
            N.call('asr_vgg_block_backward_zdp', N.ptr(dnext),
                   BF16 if dnext.dtype == torch.bfloat16 else F32, flat, N.ptr(z),
                   BF16 if z.dtype == torch.bfloat16 else F32, B, cT, cF, Co, pt,
                   pf, ceil, N.ptr(P), BF16 if P.dtype == torch.bfloat16 else F32, N.ptr(slot),
                   N.ptr(sp['gamma']), N.ptr(mean), N.ptr(rstd),
                   N.ptr(grad_buffer(sp['gamma']) if bn else None),
                   N.ptr(grad_buffer(sp['beta']) if bn else None), drop, seed, N.ptr(dz),
                   F32 if dz_f32 else cd,
                   N.ptr(grad_buffer(sp['b']) if fused_bias else None), N.ptr(ws), nb,
                   N.stream_handle(dev))
            w = sp['w']
            if not gemm:
                nb = N.query('asr_conv_direct_wgrad_workspace_bytes', B, cT, cF, cC, Co)
                ws = _ws(nb, dev)
                N.call('asr_conv_direct_wgrad', N.ptr(x_op), N.ptr(dz), B, cT, cF, cC, Co,
                       N.ptr(grad_buffer(w)),
                       N.ptr(grad_buffer(sp['b']) if sp['b'] is not None else None), N.ptr(ws),
                       nb, N.stream_handle(dev))
                if l == 0:
                    break
                dx = torch.empty(npad, cC, **f32)
                N.call('asr_conv_direct_dgrad', N.ptr(dz), B, cT, cF, cC, Co, N.ptr(w), N.ptr(dx),
                       N.stream_handle(dev))
                dnext, flat = dx, 0
                continue
            if Co <= 64 and cd == BF16 and os.environ.get('ASR_VGG_DW_T', '0') == '1':
                # transposed image [9 Ci][Co] = X^T dz: C_out becomes the narrow N
                # of the 256 x 64 kernel (dz^T X puts C_out on half-empty 128-row
                # tiles).  Opt-in: measured 0.27 ms / step SLOWER at vgg_hier (the
                # K-major 256 x 64 tile needs 96 KB of LDS, one work-group per CU)
                packed_t = torch.empty(9 * cCp, Co, **f32)
                N.call('asr_gemm_set_n64_kmode', 1)
                try:
                    run_gemm([gemm_problem(_tap_operand(x_op, 1, cCp, cCp, cF + 2, 1),
                                           operand(dz, 1, rowmap(Co)), packed_t, rowmap(Co),
                                           9 * cCp, Co, npad)], dev)
                finally:
                    N.call('asr_gemm_set_n64_kmode', 0)
                N.call('asr_conv_weight_unpack_acc_pad_t', N.ptr(packed_t), Co, cC, cCp,
                       N.ptr(grad_buffer(w)), N.stream_handle(dev))
            else:
                # dW image [Co][9 Ci] = dz^T X (taps on the output index), K = padded pixels.
                # On a side stream (ASR_VGG_WGRAD_SIDE, default on): only the
                # optimizer reads it, so it runs beside this layer's input-gradient
                # convolution and the layer below's element-wise passes
                side = _vgg_wgrad_stream(dev)
                if side is not None:
                    main = torch.cuda.current_stream(dev)
                    side.wait_stream(main)
                with torch.cuda.stream(side) if side is not None else _nullctx():
                    packed = torch.empty(Co, 9 * cCp, **f32)
                    if l == 0 and ctx.c1w:   # x_op is the raw features xs
                        nb = N.query('asr_conv3x3_c1_wgrad_workspace_bytes', Co)
                        ws = _ws(nb, dev)
                        N.call('asr_conv3x3_c1_wgrad_xs', N.ptr(x_op), 1, B, cT, cF, Co, N.ptr(dz),
                               cCp, N.ptr(packed), N.ptr(ws), nb, N.stream_handle(dev))
                    elif not conv3x3_tr_wgrad(x_op, dz, npad, cCp, cF + 2, Co, packed):
                        run_gemm([gemm_problem(operand(dz, 1, rowmap(Co)),
                                               _tap_operand(x_op, 1, cCp, cCp, cF + 2, 1), packed,
                                               rowmap(9 * cCp), Co, 9 * cCp, npad)], dev)
                    N.call('asr_conv_weight_unpack_acc_pad', N.ptr(packed), Co, cC, cCp,
                           N.ptr(grad_buffer(w)), N.stream_handle(dev))
                if side is not None:
                    for t in (x_op, dz):
                        t.record_stream(side)
                    if not _side_pending:
                        torch.autograd.Variable._execution_engine.queue_callback(
                            lambda: _join_side_wgrads(dev, notify=False))
                    _side_pending.append((side, (grad_buffer(w),), main))
            if l == 0:
                break
            # d input (padded rows of layer l's input) = dz (taps, mirrored) x W^T image
            wt = torch.empty(cC, 9 * Co, dtype=opdt, device=dev)
            N.call('asr_conv_weight_pack', N.ptr(w), Co, cC, 1, cd, N.ptr(wt),
                   N.stream_handle(dev))
            # bf16 mode: the input gradient goes to the layer below as bf16 when that
            # layer's pool / ReLU / BN backward reads it on its bf16 full-resolution
            # pass (half the bytes of the largest tensors of the VGG backward)
            lo = layers[l - 1]
            dx_bf = (cd == BF16 and lo[10] and cC % 4 == 0 and
                     saved[6 * (l - 1) + 1].dtype == torch.bfloat16 and
                     os.environ.get('ASR_VGG_POST_FULL', '1') != '0' and
                     os.environ.get('ASR_VGG_DX_BF16', '1') != '0')
            dx = torch.empty(npad, cC, dtype=torch.bfloat16 if dx_bf else torch.float32,
                             device=dev)
            if _conv_tr_ok(Co, cC, cF + 2, npad, dx.element_size()):
                conv3x3_tr(dz, npad, Co, cF + 2, -1, wt, cC, None, dx)
            else:
                run_gemm([gemm_problem(_tap_operand(dz, 0, Co, Co, cF + 2, -1),
                                       operand(wt, 0, rowmap(9 * Co)), dx, rowmap(cC), npad, cC,
                                       9 * Co)], dev)
            dnext, flat = dx, 0
        return (None, None, None, None) + (None,) * len(ctx.needs_input_grad[4:])


_vgg_side = {}


def _vgg_wgrad_stream(dev):
    """The stream the VGG convolutions' weight gradients run on, or None (the
    compute stream; ASR_VGG_WGRAD_SIDE=0)."""
    if os.environ.get('ASR_VGG_WGRAD_SIDE', '1') == '0':
        return None
    st = _vgg_side.get(dev.index)
    if st is None:
        st = _vgg_side[dev.index] = torch.cuda.Stream(device=dev)
    return st


class _nullctx(object):
    def __enter__(self):
        return self

    def __exit__(self, *a):
        return False


def vgg_front(xs, specs, training, p_drop):
    params = [t for sp in specs for t in (sp['w'], sp['b'], sp['gamma'], sp['beta'])
              if t is not None]
    return VGGFn.apply(xs, specs, training, p_drop, *params)
