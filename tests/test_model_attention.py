"""Drop-in AttentionSeq2seq (location attention, bahdanau, +/- auxiliary CTC)
vs the reference's golden vectors.  CPU: bit-identical initial state_dict under
the reference's seed.  GPU: loss and every parameter gradient."""
import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_params

NAMES = ['model_att', 'model_att_hybrid', 'model_att_ls']


def _build(kw):
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.attention.attention_seq2seq \
        import AttentionSeq2seq
    torch.manual_seed(1623)
    return AttentionSeq2seq(**kw)


@pytest.mark.parametrize('name', NAMES)
def test_init_matches_reference_state_dict(name):
    d = golden(name)
    model = _build(json.loads(str(d['kwargs'])))
    sd = model.state_dict()
    ref = {k[3:]: d[k] for k in d.files if k.startswith('sd/')}
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


def test_load_model_attention_config():
    import yaml
    from pytorch_end2end_speech_recognition_amd.models.load_model import load
    params = yaml.safe_load(open(__file__.replace('test_model_attention.py',
                                                  'golden/char_blstm_att_100h.yml')))['param']
    params['num_classes'] = 28
    model = load('attention', params, 'pytorch')
    assert model.name.startswith('blstm320H4L_drop4_lstm320H1L_adam_lr1e-3_location')
    assert model.total_parameters > 0


@pytest.mark.gpu
@pytest.mark.parametrize('name', NAMES)
def test_attention_model_matches_golden(name, cuda_dev):
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
    assert tuple(loss.shape) == (1,)
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.item(), float(d['loss'][0]), rtol=1e-4)
    for k, p in model.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g[k], rtol=2e-3, atol=2e-5, err_msg=k)
