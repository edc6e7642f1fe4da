"""Drop-in CTC model (models.pytorch_v3.ctc.ctc.CTC) vs the reference.

CPU: construction under the reference's seed reproduces the reference's
initial state_dict bit for bit (same module tree, same RNG consumption), the
flat buffer keeps every LSTM fwd/rev pair adjacent, load_model builds the same
name.  GPU: loss / all gradients / greedy best path vs the golden vectors, and
one train_step (fused clip + Adam) vs torch.optim.Adam on the CPU oracle.
"""
import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_params
from oracle import asr_ref


def _build(kw):
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.ctc.ctc import CTC
    torch.manual_seed(1623)
    return CTC(**kw)


CTC_MODELS = ['model_ctc_sub', 'model_ctc_fast', 'model_ctc_gru_fast', 'model_ctc_gru_sub',
              'model_ctc_proj', 'model_ctc_concat',
              'model_ctc_proj_concat', 'model_ctc_res', 'model_ctc_dres']


@pytest.mark.parametrize('name', CTC_MODELS)
def test_init_matches_reference_state_dict(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    model = _build(kw)
    sd = model.state_dict()
    ref = {k[3:]: d[k] for k in d.files if k.startswith('sd/')}
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


def test_flat_layout_pairs_adjacent():
    d = golden('model_ctc_sub')
    model = _build(json.loads(str(d['kwargs'])))
    enc = model.encoder
    for l in range(enc.num_layers):
        for f, r in enc._layer_params(l):
            assert r.data_ptr() == f.data_ptr() + 4 * f.numel()
            assert f.grad.data_ptr() + 4 * f.numel() == r.grad.data_ptr()
    assert model._flat_param.data_ptr() % 64 == 0


def test_load_model_name():
    from pytorch_end2end_speech_recognition_amd.models.load_model import load
    import yaml
    params = yaml.safe_load(open(__file__.replace('test_model_ctc.py',
                                                  'golden/char_blstm_ctc_100h.yml')))['param']
    params['num_classes'] = 28
    model = load('ctc', params, 'pytorch')
    # YAML 1.1 reads `1e-3` as a string, exactly as the reference's yaml.load does
    assert model.name == 'blstm320H4L_drop4_adam_lr1e-3_dropen0.2_input80'
    assert model.total_parameters == sum(p.numel() for p in model.parameters())


def _to_gpu_model(kw, sd, dev):
    model = _build(kw)
    model.load_state_dict({k: v for k, v in sd.items()})
    model.set_cuda()
    return model


@pytest.mark.gpu
@pytest.mark.parametrize('name', CTC_MODELS)
def test_ctc_model_matches_golden(name, cuda_dev):
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('fp32')
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    sd, g = golden_params(d)
    model = _to_gpu_model(kw, sd, cuda_dev)
    model.zero_grad()
    loss = model(d['xs'], d['ys'], d['x_lens'], d['y_lens'])
    assert tuple(loss.shape) == (1,)
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.item(), float(d['loss'][0]), rtol=1e-4)
    for k, p in model.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g[k], rtol=1e-3, atol=2e-5, err_msg=k)
    hyps, aw, perm = model.decode(d['xs'], d['x_lens'], beam_width=1)
    assert aw is None
    np.testing.assert_array_equal(perm, d['perm'])
    np.testing.assert_array_equal([len(h) for h in hyps], d['hyp_lens'])
    flat = np.concatenate(list(hyps)) if len(hyps) else np.zeros(0)
    np.testing.assert_array_equal(flat, d['hyp_flat'])
    ev = model(d['xs'], d['ys'], d['x_lens'], d['y_lens'], is_eval=True)
    assert isinstance(ev, float)
    np.testing.assert_allclose(ev, float(d['loss'][0]), rtol=1e-4)


@pytest.mark.gpu
def test_train_step_matches_torch_adam(cuda_dev):
    """One reference train_step (clip 5 + Adam wd 1e-6) on GPU vs the oracle +
    torch.optim.Adam + clip_grad_norm_ on CPU."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    native_ops.set_compute_dtype('fp32')
    d = golden('model_ctc_sub')
    kw = json.loads(str(d['kwargs']))
    sd, _ = golden_params(d)
    model = _to_gpu_model(kw, sd, cuda_dev)
    model.set_optimizer('adam', 1e-3, weight_decay=1e-6)
    batch = dict(xs=d['xs'], ys=d['ys'], x_lens=d['x_lens'], y_lens=d['y_lens'])
    for _ in range(2):
        model, lv = train_step(model, batch, clip_grad_norm=0.5)
    torch.cuda.synchronize()

    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    opt = torch.optim.Adam(list(p.values()), lr=1e-3, weight_decay=1e-6)
    cfg = dict(num_layers=kw['encoder_num_layers'], subsample_list=kw['subsample_list'],
               fc_list=kw['fc_list'])
    for _ in range(2):
        opt.zero_grad()
        loss, _, _, _ = asr_ref.ctc_model_loss(p, cfg, d['xs'], d['ys'], d['x_lens'],
                                               d['y_lens'])
        loss.backward()
        torch.nn.utils.clip_grad_norm_(list(p.values()), 0.5)
        opt.step()
    np.testing.assert_allclose(lv, float(loss), rtol=1e-4)
    for k, v in model.state_dict().items():
        np.testing.assert_allclose(v.cpu().numpy(), p[k].detach().numpy(), rtol=1e-4, atol=1e-6,
                                   err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize('variant', [dict(encoder_num_proj=48, subsample_type='concat'),
                                     dict(encoder_residual=True, subsample_type='concat'),
                                     dict(encoder_dense_residual=True, encoder_num_proj=64,
                                          subsample_list=[])])
def test_encoder_variants_bf16_vs_oracle(variant, cuda_dev):
    """bf16 mode (staged bf16 operands, incl. the in-place 'concat' rows of
    twice the source width) for projection / concat / residual encoders at
    H = 64 vs the fp32 CPU oracle."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=16, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=64, encoder_num_proj=0, encoder_num_layers=4, fc_list=[],
              dropout_input=0, dropout_encoder=0, num_classes=9, parameter_init=0.1,
              subsample_list=[True, False, False, False], subsample_type='drop')
    kw.update(variant)
    model = _build(kw)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    rng = np.random.RandomState(5)
    B, T = 4, 41
    x_lens = np.array([41, 33, 27, 40], np.int32)
    y_lens = np.array([6, 4, 5, 3], np.int32)
    xs = rng.randn(B, T, 16).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 6), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 9, y_lens[b])
    from test_oracle_golden import ctc_cfg
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref, _, _, _ = asr_ref.ctc_model_loss(p, ctc_cfg(kw), xs, ys, x_lens, y_lens)
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
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < 2e-2
    for k, prm in model.named_parameters():
        ga = p[k].grad.numpy()
        gw = prm.grad.cpu().numpy()
        scale = np.abs(ga).max() + 1e-6
        assert np.abs(gw - ga).max() / scale < 5e-2, (k, np.abs(gw - ga).max(), scale)


@pytest.mark.gpu
def test_recurrence_give_up_skips_the_batch(cuda_dev):
    """A persistent recurrence whose bounded spin gave up (simulated with the
    status hook, exactly the word a give-up sets) must not update the weights:
    the fused optimizer kernel sees the device guard, train_step returns 0 and
    skips (training_loop.py:69-76), Adam's step count is unchanged, and the
    next clean step trains normally."""
    from pytorch_end2end_speech_recognition_amd import _native as N
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    native_ops.set_compute_dtype('bf16')
    try:
        d = golden('model_ctc_sub')
        kw = json.loads(str(d['kwargs']))
        sd, _ = golden_params(d)
        model = _to_gpu_model(kw, sd, cuda_dev)
        model.set_optimizer('adam', 1e-3, weight_decay=1e-6)
        batch = dict(xs=d['xs'], ys=d['ys'], x_lens=d['x_lens'], y_lens=d['y_lens'])
        native_ops.recurrence_status(cuda_dev)             # clear
        before = model._flat_param.clone()
        # a give-up during the step's own pass (train_step drops status words
        # left from before it starts)
        orig = model.forward

        def fwd(*a, **k):
            N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
            return orig(*a, **k)

        model.forward = fwd
        model, lv = train_step(model, batch, clip_grad_norm=5.0)
        model.forward = orig
        torch.cuda.synchronize()
        assert lv == 0.0
        assert torch.equal(before, model._flat_param)
        assert model.optimizer._step == 0
        assert int(native_ops.recurrence_status(cuda_dev).max().item()) == 0   # cleared
        model, lv = train_step(model, batch, clip_grad_norm=5.0)
        torch.cuda.synchronize()
        assert lv > 0 and model.optimizer._step == 1
        assert not torch.equal(before, model._flat_param)
        N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
        with pytest.raises(N.NativeError):
            native_ops.raise_if_recurrence_failed(cuda_dev)
    finally:
        native_ops.set_compute_dtype('fp32')


@pytest.mark.gpu
def test_deferred_loss_readback_matches_synchronous_steps(cuda_dev):
    """train_step(sync=False) (the loss read back one step late, so steps queue
    back to back) applies the same updates as the synchronous loop: bitwise
    equal weights and losses over four steps, one of them skipped by a
    recurrence give-up -- its step count is undone before the next update and
    its gradients are not zeroed under the next step."""
    from pytorch_end2end_speech_recognition_amd import _native as N
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import train_step
    native_ops.set_compute_dtype('bf16')
    try:
        d = golden('model_ctc_sub')
        kw = json.loads(str(d['kwargs']))
        sd, _ = golden_params(d)
        batch = dict(xs=d['xs'], ys=d['ys'], x_lens=d['x_lens'], y_lens=d['y_lens'])
        runs = []
        for sync in (True, False):
            model = _to_gpu_model(kw, sd, cuda_dev)
            model.set_optimizer('adam', 1e-3, weight_decay=1e-6)
            native_ops.recurrence_status(cuda_dev)             # clear
            vals = []
            orig = model.forward

            def fwd(*a, **k):
                N.call('asr_lstm_status_inject', 1, N.stream_handle(cuda_dev))
                return orig(*a, **k)

            for k in range(4):
                model.forward = fwd if k == 1 else orig     # a give-up inside step 1
                model, lv = train_step(model, batch, clip_grad_norm=5.0, sync=sync)
                vals.append(lv)
            model.forward = orig
            vals = [float(v) for v in vals]
            torch.cuda.synchronize()
            runs.append((vals, model._flat_param.clone(), model.optimizer._step))
        (v0, p0, s0), (v1, p1, s1) = runs
        assert v0 == v1 and v0[1] == 0.0 and v0[0] > 0, (v0, v1)
        assert s0 == s1 == 3
        assert torch.equal(p0, p1)
    finally:
        native_ops.set_compute_dtype('fp32')


def test_wgrad_overlap_auto_mode(monkeypatch):
    """auto: the weight-gradient GEMMs go to a side stream (mode 3, the
    recurrence at its 140 KB LDS pin so no GEMM work-group can share its CUs)
    when the persistent backward recurrence leaves >= 32 of the 256 CUs free
    (the H = 320 configs; ctc5x512 with 32 units per backward work-group),
    else they stay on the compute stream; co-resident
    GEMMs (mode 2) are never chosen automatically."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    monkeypatch.delenv('ASR_OVERLAP_WGRAD', raising=False)
    monkeypatch.setattr(native_ops, '_num_cus', lambda dev: 256)
    prev = native_ops.compute_dtype()
    native_ops.set_compute_dtype('bf16')
    try:
        cpu = torch.device('cpu')
        # 5x512: 256 work-groups at 16 units each, 128 at 32 -> mode 3 with 32
        assert native_ops._overlap_plan(cpu, 32, 512) == ('3', 32)
        assert native_ops._overlap_plan(cpu, 32, 320) == ('3', 16)
        assert native_ops._overlap_plan(cpu, 64, 512) == ('0', 16)   # 256 even at 32
        monkeypatch.setenv('ASR_XG_BWD_XU', '16')
        assert native_ops._overlap_mode(cpu, 32, 512) == '0'
        monkeypatch.delenv('ASR_XG_BWD_XU')
        assert native_ops._overlap_mode(cpu, 32, 320) == '3'     # 160
        assert native_ops._overlap_mode(cpu, 16, 256) == '3'     # 64
        assert native_ops._overlap_mode(cpu, 32, 500) == '0'     # no persistent recurrence
        monkeypatch.setenv('ASR_OVERLAP_WGRAD', '1')
        assert native_ops._overlap_mode(cpu, 32, 320) == '0'     # 160 > 128: no half fits
        assert native_ops._overlap_mode(cpu, 16, 256) == '1'
        native_ops.set_compute_dtype('fp32')
        monkeypatch.setenv('ASR_OVERLAP_WGRAD', '3')
        assert native_ops._overlap_mode(cpu, 16, 256) == '0'     # fp32 parity mode
    finally:
        native_ops.set_compute_dtype('bf16' if prev == native_ops.BF16 else 'fp32')


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['1', '3'])
def test_wgrad_side_stream_matches_main_stream(mode, cuda_dev, monkeypatch):
    """Weight gradients computed on the side stream (ASR_OVERLAP_WGRAD=1: CU-masked
    half of the chip; 3: the CUs the next layer's persistent backward
    recurrence leaves free) equal the main-stream ones -- bitwise: the same GEMM
    kernels on the same operands -- at a shape that takes the persistent
    recurrence (B = 16, H = 256, three layers, T = 160), and the recurrence did
    not give up."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=40, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=256, encoder_num_proj=0, encoder_num_layers=3, fc_list=[],
              dropout_input=0, dropout_encoder=0, num_classes=29, parameter_init=0.1,
              subsample_list=[], subsample_type='drop')
    model = _build(kw)
    rng = np.random.RandomState(11)
    B, T = 16, 160
    x_lens = np.sort(rng.randint(100, T + 1, B)).astype(np.int32)[::-1].copy()
    x_lens[0] = T
    y_lens = rng.randint(10, 30, B).astype(np.int32)
    xs = rng.randn(B, T, 40).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 30), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    native_ops.set_compute_dtype('bf16')
    grads, events = {}, {}
    try:
        model.set_cuda()
        for m in ('0', mode):
            monkeypatch.setenv('ASR_OVERLAP_WGRAD', m)
            native_ops.recurrence_status(cuda_dev)             # clear
            model.zero_grad()
            ev, pre = [], []
            native_ops.set_grad_ready_hook(
                lambda e, arg=None: ev.append(e) if e != 'pre_recurrence' else pre.append(e))
            try:
                loss = model(xs, ys, x_lens, y_lens)
                loss.backward()
            finally:
                native_ops.set_grad_ready_hook(None)
            torch.cuda.synchronize()
            assert int(native_ops.recurrence_status(cuda_dev).max().item()) == 0
            grads[m] = {k: p.grad.detach().cpu().numpy().copy()
                        for k, p in model.named_parameters()}
            events[m] = ev
            assert len(pre) == 3     # one before every backward recurrence
    finally:
        native_ops.set_compute_dtype('fp32')
    # gradient-ready notifications (DP buckets): every layer above the lowest is
    # reported before the next recurrence in both modes
    assert events['0'] == ['recurrence', 'grads'] * 3
    # side modes: the CTC head's weight gradient runs beside the top layer's
    # recurrence and is joined (and reported) as that recurrence is enqueued
    ev = events[mode][1:] if events[mode][:1] == ['grads'] else events[mode]
    assert ev[:5] == ['recurrence', 'grads', 'recurrence', 'grads', 'recurrence'], events[mode]
    for k, g0 in grads['0'].items():
        np.testing.assert_array_equal(grads[mode][k], g0, err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype', ['fp32', 'bf16'])
def test_gru_encoder_vs_oracle(dtype, cuda_dev):
    """BGRU CTC model (rnn.py:173-191 / :226-233, per-layer path with 'drop'
    subsampling) at H = 96, three layers, ragged lengths, vs the fp32 CPU
    oracle (asr_ref.gru_direction): loss and every gradient (fp32 mode: 1e-4 /
    2e-3 of max |g|; bf16 mode: the GEMMs on bf16 operands, 2e-2 / 5e-2)."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=24, encoder_type='gru', encoder_bidirectional=True,
              encoder_num_units=96, encoder_num_proj=0, encoder_num_layers=3, fc_list=[],
              dropout_input=0, dropout_encoder=0, num_classes=11, parameter_init=0.1,
              subsample_list=[False, True, False], subsample_type='drop')
    model = _build(kw)
    sd = {k: v.clone() for k, v in model.state_dict().items()}
    rng = np.random.RandomState(8)
    B, T = 5, 57
    x_lens = np.array([57, 40, 52, 31, 45], np.int32)
    y_lens = np.array([7, 5, 6, 3, 4], np.int32)
    xs = rng.randn(B, T, 24).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 7), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 11, y_lens[b])
    from test_oracle_golden import ctc_cfg
    p = {k: v.clone().requires_grad_(True) for k, v in sd.items()}
    ref, _, _, _ = asr_ref.ctc_model_loss(p, ctc_cfg(kw), xs, ys, x_lens, y_lens)
    ref.backward()
    native_ops.set_compute_dtype(dtype)
    try:
        model.set_cuda()
        model.zero_grad()
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        torch.cuda.synchronize()
    finally:
        native_ops.set_compute_dtype('fp32')
    tl, tg = (1e-4, 2e-3) if dtype == 'fp32' else (2e-2, 5e-2)
    assert abs(loss.item() - ref.item()) / abs(ref.item()) < tl, (loss.item(), ref.item())
    for k, prm in model.named_parameters():
        ga = p[k].grad.numpy()
        gw = prm.grad.cpu().numpy()
        scale = np.abs(ga).max() + 1e-6
        assert np.abs(gw - ga).max() / scale < tg, (k, np.abs(gw - ga).max(), scale)


@pytest.mark.gpu
def test_output_dropout_folded_into_head_bitwise(cuda_dev, monkeypatch):
    """bf16 training with encoder dropout: the last BLSTM layer's output
    dropout handed to the CTC head (LinearND input_drop: the mask applied in
    the head's bf16 staging and its dX GEMM epilogue) and the inter-layer
    dropouts folded into the next layer's staging give the same loss and
    gradients, bit for bit, as separate asr_dropout passes (ASR_FUSE_DROPOUT=0)
    under the same seed stream."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=40, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=64, encoder_num_proj=0, encoder_num_layers=2, fc_list=[],
              dropout_input=0, dropout_encoder=0.3, num_classes=29, parameter_init=0.1,
              subsample_list=[], subsample_type='drop')
    rng = np.random.RandomState(3)
    B, T = 8, 60
    x_lens = np.sort(rng.randint(40, T + 1, B)).astype(np.int32)[::-1].copy()
    x_lens[0] = T
    y_lens = rng.randint(5, 15, B).astype(np.int32)
    xs = rng.randn(B, T, 40).astype(np.float32)
    ys = np.full((B, 15), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    outs = []
    native_ops.set_compute_dtype('bf16')
    # stage the head's operands at this size too (the path the dropout folds into)
    monkeypatch.setattr(native_ops, '_STAGE_FLOPS_RAGGED', 1.0)
    try:
        for fuse in ('1', '0'):
            monkeypatch.setenv('ASR_FUSE_DROPOUT', fuse)
            native_ops.manual_seed(1234)
            model = _build(kw)
            model.set_cuda()
            model.zero_grad()
            loss = model(xs, ys, x_lens, y_lens)
            loss.backward()
            torch.cuda.synchronize()
            outs.append((loss.item(), model._flat_grad.clone()))
    finally:
        native_ops.set_compute_dtype('fp32')
    (l1, g1), (l0, g0) = outs
    assert l1 == l0, (l1, l0)
    assert torch.equal(g1, g0)
    assert g1.abs().sum().item() > 0


@pytest.mark.gpu
@pytest.mark.parametrize('training', [True, False])
def test_bf16_handoff_between_layers_bitwise(training, cuda_dev, monkeypatch):
    """bf16 mode: a BLSTM layer whose output feeds only the next one writes that
    layer's staged bf16 input itself (dropout applied with the same mask,
    asr_lstm_forward_xh_drop) and no f32 output -- the same loss and gradients,
    bit for bit, as writing the f32 output and staging it in a separate pass
    (ASR_BF16_HANDOFF=0), in training (encoder dropout 0.2) and in eval."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=40, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=256, encoder_num_proj=0, encoder_num_layers=3, fc_list=[],
              dropout_input=0, dropout_encoder=0.2, num_classes=29, parameter_init=0.1,
              subsample_list=[], subsample_type='drop')
    rng = np.random.RandomState(12)
    B, T = 16, 120
    x_lens = np.sort(rng.randint(80, T + 1, B)).astype(np.int32)[::-1].copy()
    x_lens[0] = T
    y_lens = rng.randint(10, 30, B).astype(np.int32)
    xs = rng.randn(B, T, 40).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 30), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    used = []
    orig = native_ops._handoff_input

    def spy(*a):
        t = orig(*a)
        used.append(t is not None)
        return t

    monkeypatch.setattr(native_ops, '_handoff_input', spy)
    outs = {}
    native_ops.set_compute_dtype('bf16')
    try:
        for on in ('1', '0'):
            monkeypatch.setenv('ASR_BF16_HANDOFF', on)
            native_ops.manual_seed(99)
            del used[:]
            model = _build(kw)
            model.set_cuda()
            model.train(training)
            model.zero_grad()
            loss = model(xs, ys, x_lens, y_lens)
            loss.backward()
            torch.cuda.synchronize()
            outs[on] = (loss.item(), model._flat_grad.clone(), list(used))
    finally:
        native_ops.set_compute_dtype('fp32')
    assert outs['1'][2] == [False, True, True], outs['1'][2]    # layers 1 and 2 took it
    assert outs['0'][2] == [False, False, False]
    assert outs['1'][0] == outs['0'][0], (outs['1'][0], outs['0'][0])
    assert torch.equal(outs['1'][1], outs['0'][1])
    assert outs['1'][1].abs().sum().item() > 0


def test_handoff_input_refuses_other_reads(monkeypatch):
    """A handed-over layer output (its f32 values never written) is readable
    only as the next layer's identity-mapped input with the same dropout:
    anything else raises instead of reading the unwritten tensor."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    prev = native_ops.compute_dtype()
    native_ops.set_compute_dtype('bf16')
    try:
        y = torch.empty(2, 5, 16)
        tw = torch.zeros(2, 5, 16, dtype=torch.bfloat16)
        y._asr_handoff = (tw, (0.2, 7))
        assert native_ops._handoff_input(y, None, 1, 0, 5, False, (0.2, 7), 16) is tw
        assert native_ops._handoff_input(torch.empty(2, 5, 16), None, 1, 0, 5, False, None,
                                         16) is None
        for args in [(torch.zeros(2, dtype=torch.int32), 1, 0, 5, False, (0.2, 7), 16),
                     (None, 2, 1, 2, False, (0.2, 7), 16),
                     (None, 1, 0, 5, True, (0.2, 7), 32),
                     (None, 1, 0, 5, False, None, 16),
                     (None, 1, 0, 5, False, (0.2, 8), 16)]:
            with pytest.raises(native_ops.N.NativeError):
                native_ops._handoff_input(y, *args)
    finally:
        native_ops.set_compute_dtype('bf16' if prev == native_ops.BF16 else 'fp32')


def test_eval_retry_policy_cpu():
    """models/pytorch_v3/base.eval_retry: a RecurrenceGaveUp re-runs the pass
    once; a second one propagates; other errors propagate at once."""
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.base import eval_retry
    from pytorch_end2end_speech_recognition_amd.native_ops import RecurrenceGaveUp

    class M(object):
        def __init__(self, fails, exc=RecurrenceGaveUp):
            self.fails, self.calls, self.exc = fails, 0, exc

        @eval_retry
        def forward(self, x, is_eval=True):
            self.calls += 1
            if self.calls <= self.fails:
                raise self.exc('gave up')
            return x + 1

    m = M(1)
    assert m.forward(1) == 2 and m.calls == 2
    m = M(2)
    with pytest.raises(RecurrenceGaveUp):
        m.forward(1)
    assert m.calls == 2
    m = M(1, exc=ValueError)
    with pytest.raises(ValueError):
        m.forward(1)
    assert m.calls == 1


@pytest.mark.gpu
def test_ctc_head_weight_gradient_beside_recurrence_bitwise(cuda_dev, monkeypatch):
    """bf16 mode: the fused CTC head's weight / bias gradient enqueued on the
    weight-gradient side stream, gated on the top BLSTM layer's backward
    recurrence (LinearCTCFn.backward) -- the same loss and flat gradient, bit
    for bit, as computing it on the compute stream (ASR_HEAD_WGRAD_SIDE=0)."""
    from pytorch_end2end_speech_recognition_amd import native_ops
    kw = dict(input_size=40, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=256, encoder_num_proj=0, encoder_num_layers=2, fc_list=[],
              dropout_input=0, dropout_encoder=0.2, num_classes=29, parameter_init=0.1,
              subsample_list=[], subsample_type='drop')
    rng = np.random.RandomState(13)
    B, T = 32, 100
    x_lens = np.sort(rng.randint(70, T + 1, B)).astype(np.int32)[::-1].copy()
    x_lens[0] = T
    y_lens = rng.randint(10, 25, B).astype(np.int32)
    xs = rng.randn(B, T, 40).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    ys = np.full((B, 25), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, 28, y_lens[b])
    calls = []
    orig = native_ops._linear_wgrad

    def spy(*a, **k):
        calls.append(torch.cuda.current_stream().cuda_stream)
        return orig(*a, **k)

    monkeypatch.setattr(native_ops, '_linear_wgrad', spy)
    # the fused head (LinearCTCFn) at this small shape: stage the 29-class product
    monkeypatch.setattr(native_ops, '_STAGE_FLOPS_RAGGED', 1e6)
    seen = []
    orig_p, orig_s = native_ops._produced_by_blstm, native_ops._wgrad_side_stream

    def spy_p(t, *a):
        r = orig_p(t, *a)
        seen.append(('from_blstm', r, type(t.grad_fn).__name__))
        return r

    def spy_s(*a):
        r = orig_s(*a)
        seen.append(('side', a[1:], r is not None))
        return r

    monkeypatch.setattr(native_ops, '_produced_by_blstm', spy_p)
    monkeypatch.setattr(native_ops, '_wgrad_side_stream', spy_s)
    outs = {}
    native_ops.set_compute_dtype('bf16')
    try:
        for on in ('1', '0'):
            monkeypatch.setenv('ASR_HEAD_WGRAD_SIDE', on)
            native_ops.manual_seed(7)
            del calls[:]
            model = _build(kw)
            model.set_cuda()
            model.train()
            model.zero_grad()
            loss = model(xs, ys, x_lens, y_lens)
            loss.backward()
            torch.cuda.synchronize()
            outs[on] = (loss.item(), model._flat_grad.clone(), len(calls))
    finally:
        native_ops.set_compute_dtype('fp32')
    assert outs['1'][2] == 1 and outs['0'][2] == 0, (outs['1'][2], outs['0'][2], seen)
    assert outs['1'][0] == outs['0'][0]
    assert torch.equal(outs['1'][1], outs['0'][1])
    assert outs['1'][1].abs().sum().item() > 0
