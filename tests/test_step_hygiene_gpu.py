"""Step hygiene around failures (training_loop.py:69-76 skip contract):

* a backward that raises while weight-gradient GEMMs are still pending on the
  side stream (ASR_OVERLAP_WGRAD=3) must not leak them into the next step --
  the next clean step equals a clean step from the same weights, bitwise;
* an eval forward / decode whose persistent recurrence gave up raises instead
  of returning invalid values, and consumes the status words so the next
  train_step is not skipped for it.
"""
import numpy as np
import pytest
import torch

from test_model_ctc import _build


def _kw():
    # a shape that takes the persistent recurrence and the side stream
    return dict(input_size=40, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=256, encoder_num_proj=0, encoder_num_layers=3, fc_list=[],
                dropout_input=0, dropout_encoder=0, num_classes=29, parameter_init=0.1,
                subsample_list=[], subsample_type='drop')


def _batch(seed=11, B=16, T=160):
    rng = np.random.RandomState(seed)
    x_lens = np.sort(rng.randint(100, T + 1, B)).astype(np.int32)[::-1].copy()
    x_lens[0] = T
    y_lens = rng.randint(10, 30, B).astype(np.int32)
    xs = rng.randn(B, T, 40).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 30), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    return dict(xs=xs, ys=ys, x_lens=x_lens, y_lens=y_lens)


@pytest.mark.gpu
def test_failed_backward_with_pending_side_wgrads_then_clean_step(cuda_dev, monkeypatch):
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    monkeypatch.setenv('ASR_OVERLAP_WGRAD', '3')
    batch = _batch()
    native_ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(1623)
        sd = {k: v.clone() for k, v in _build(_kw()).state_dict().items()}

        def fresh():
            m = _build(_kw())
            m.load_state_dict(sd)
            m.set_cuda()
            m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
            return m

        # clean reference: one step from the initial weights
        ref = fresh()
        native_ops.recurrence_status(cuda_dev)
        ref, lv_ref = train_step(ref, batch, clip_grad_norm=5.0)
        torch.cuda.synchronize()
        assert lv_ref > 0

        # a backward that raises while the top layer's side-stream weight
        # gradients are pending (raised from inside their join, before the
        # pending list is cleared)
        m = fresh()
        seen = []

        def hook(event, arg=None):
            seen.append(event)
            if event == 'grads' and seen.count('grads') == 1:
                assert native_ops._side_pending, 'side stream not in use'
                raise RuntimeError('injected failure inside the backward')

        native_ops.set_grad_ready_hook(hook)
        try:
            m, lv = train_step(m, batch, clip_grad_norm=5.0)
        finally:
            native_ops.set_grad_ready_hook(None)
        torch.cuda.synchronize()
        assert lv == 0.0 and m.optimizer._step == 0
        assert not native_ops._side_pending
        assert float(m._flat_grad.abs().max()) == 0.0

        # the next clean step equals the reference's step bitwise (a leaked
        # pending accumulation would add a whole layer's weight gradient)
        m, lv = train_step(m, batch, clip_grad_norm=5.0)
        torch.cuda.synchronize()
        assert lv == lv_ref
        for (k, p1), p0 in zip(m.named_parameters(), ref.parameters()):
            assert torch.equal(p1.grad, p0.grad), k
        assert torch.equal(m._flat_param, ref._flat_param)
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_eval_and_decode_retry_then_raise_on_recurrence_give_up(cuda_dev):
    """The dev-loss eval (the reference's training scripts call
    model(..., is_eval=True) every print_step) and decode: one give-up during
    the pass re-runs it (same value as a healthy pass, a warning); a give-up on
    the re-run too raises RecurrenceGaveUp (a NativeError)."""
    from pytorch_end2end_speech_recognition_amd import _native as N
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    batch = _batch(seed=3, B=8, T=120)
    native_ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(1623)
        m = _build(_kw())
        m.set_cuda()
        m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
        native_ops.recurrence_status(cuda_dev)
        # healthy eval: no error
        v = m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'], is_eval=True)
        assert np.isfinite(v)
        h0 = m.decode(batch['xs'], batch['x_lens'], beam_width=1)[0]
        # one give-up during the eval pass (the status word a bounded spin
        # sets): retried, the same loss
        N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
        assert m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'], is_eval=True) == v
        N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
        h1 = m.decode(batch['xs'], batch['x_lens'], beam_width=1)[0]
        assert all(np.array_equal(a, b) for a, b in zip(h0, h1))
        # a give-up in every pass: raises after the one retry
        enc = m._encode

        def failing(*a, **k):
            N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
            return enc(*a, **k)
        m._encode = failing
        try:
            with pytest.raises(native_ops.RecurrenceGaveUp):
                m(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'], is_eval=True)
            with pytest.raises(N.NativeError):
                m.decode(batch['xs'], batch['x_lens'], beam_width=1)
        finally:
            del m._encode
        # the words were consumed: the next train_step trains
        m, lv = train_step(m, batch, clip_grad_norm=5.0)
        assert lv > 0 and m.optimizer._step == 1
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_checkpoint_resolves_deferred_skipped_step(cuda_dev, tmp_path):
    """save_checkpoint / FlatOptimizer.state_dict after a train_step(sync=False)
    whose batch was skipped record the undone Adam step count."""
    from pytorch_end2end_speech_recognition_amd import _native as N
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    batch = _batch(seed=4, B=8, T=120)
    native_ops.set_compute_dtype('bf16')
    try:
        torch.manual_seed(1623)
        m = _build(_kw())
        m.set_cuda()
        m.set_optimizer('adam', 1e-3, weight_decay=1e-6)
        native_ops.recurrence_status(cuda_dev)
        m, _ = train_step(m, batch, clip_grad_norm=5.0, sync=False)
        # a give-up inside the second step (injected after its start-of-step clear)
        orig = m.forward

        def fwd(*a, **k):
            N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
            return orig(*a, **k)

        m.forward = fwd
        m, _ = train_step(m, batch, clip_grad_norm=5.0, sync=False)
        m.forward = orig
        path = m.save_checkpoint(str(tmp_path), 1, 2, 1e-3, 0.0)
        ck = torch.load(path, map_location='cpu', weights_only=True)
        steps = {float(s['step']) for s in ck['optimizer']['state'].values()}
        assert steps == {1.0}, steps
    finally:
        native_ops.set_compute_dtype('fp32')
