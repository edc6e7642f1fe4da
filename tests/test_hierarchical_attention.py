"""Hierarchical attention (models/pytorch_v3/attention/
hierarchical_attention_seq2seq.py): word decoder on the top encoder layer +
character decoder (and character CTC) on layer encoder_num_layers_sub, vs
golden vectors recorded from the reference.  CPU: bit-identical initial
state_dict, oracle vs golden, the load_model branch.  GPU: the three losses and
every gradient through the fused HIP decoders, train_hierarchical_step, and
greedy decoding of both tasks."""
import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_params
from oracle import asr_ref

NAMES = ['model_hatt', 'model_hatt_ctc']


def _build(kw):
    from pytorch_end2end_speech_recognition_amd.models.pytorch_v3.attention.\
        hierarchical_attention_seq2seq import HierarchicalAttentionSeq2seq
    torch.manual_seed(1623)
    return HierarchicalAttentionSeq2seq(**kw)


def _g(v):
    return v.grad.numpy() if v.grad is not None else np.zeros(v.shape, np.float32)


@pytest.mark.parametrize('name', NAMES)
def test_hatt_init_matches_reference_state_dict(name):
    d = golden(name)
    model = _build(json.loads(str(d['kwargs'])))
    sd = model.state_dict()
    ref = {k[3:]: d[k] for k in d.files if k.startswith('sd/')}
    assert sorted(sd) == sorted(ref)
    for k, v in ref.items():
        np.testing.assert_array_equal(sd[k].numpy(), v, err_msg=k)


@pytest.mark.parametrize('name', NAMES)
def test_hatt_oracle_matches_golden(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    p, g = golden_params(d)
    for v in p.values():
        v.requires_grad_(True)
    loss, lm, ls = asr_ref.hierarchical_attention_loss(p, kw, d['xs'], d['ys'], d['x_lens'],
                                                       d['y_lens'], d['ys_sub'],
                                                       d['y_lens_sub'])
    np.testing.assert_allclose(float(loss), float(d['loss'][0]), rtol=1e-5)
    np.testing.assert_allclose(float(lm), float(d['loss_main'][0]), rtol=1e-5)
    np.testing.assert_allclose(float(ls), float(d['loss_sub'][0]), rtol=1e-5)
    loss.backward()
    for k, v in p.items():
        gv = _g(v)
        # nn.Embedding(padding_idx=-1): the <sos>/<eos> row gets no gradient
        if k in ('embed_0.embed.weight', 'embed_1.embed.weight'):
            gv = gv.copy()
            gv[-1] = 0
        np.testing.assert_allclose(gv, g[k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_load_model_hierarchical_attention_name():
    from pytorch_end2end_speech_recognition_amd.models.load_model import load
    import yaml
    params = yaml.safe_load(open(__file__.replace('test_hierarchical_attention.py',
                                                  'golden/char_blstm_att_100h.yml')))['param']
    params.update(model_type='hierarchical_attention', encoder_num_layers_sub=3,
                  decoder_num_units_sub=320, decoder_num_layers_sub=1, embedding_dim_sub=32,
                  main_loss_weight=0.8, sub_loss_weight=0.2, ctc_loss_weight_sub=0,
                  num_classes=100, num_classes_sub=28, bottleneck_dim_sub=256,
                  backward_sub=False, num_heads_sub=1)
    model = load('hierarchical_attention', params, 'pytorch')
    assert model.model_type == 'hierarchical_attention'
    assert '4L3L' in model.name and '_main0.8_sub0.2_input' in model.name
    assert model.fc_1_fwd.fc.weight.shape[0] == 29


@pytest.mark.gpu
@pytest.mark.parametrize('name', NAMES)
def test_hatt_model_matches_golden(name, cuda_dev):
    from pytorch_end2end_speech_recognition_amd import native_ops
    native_ops.set_compute_dtype('fp32')
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    sd, g = golden_params(d)
    model = _build(kw)
    model.load_state_dict(sd)
    model.set_cuda()
    model.zero_grad()
    loss, lm, ls = model(d['xs'], d['ys'], d['x_lens'], d['y_lens'], d['ys_sub'],
                         d['y_lens_sub'])
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_allclose(loss.item(), float(d['loss'][0]), rtol=1e-4)
    np.testing.assert_allclose(lm.item(), float(d['loss_main'][0]), rtol=1e-4)
    np.testing.assert_allclose(ls.item(), float(d['loss_sub'][0]), rtol=1e-4)
    for k, p in model.named_parameters():
        np.testing.assert_allclose(p.grad.cpu().numpy(), g[k], rtol=2e-3, atol=2e-5, err_msg=k)


@pytest.mark.gpu
def test_train_hierarchical_attention_step_and_decode(cuda_dev):
    from pytorch_end2end_speech_recognition_amd import native_ops
    from pytorch_end2end_speech_recognition_amd.utils.training.training_loop import \
        train_hierarchical_step
    native_ops.set_compute_dtype('fp32')
    d = golden('model_hatt_ctc')
    kw = json.loads(str(d['kwargs']))
    sd, _ = golden_params(d)
    model = _build(kw)
    model.load_state_dict(sd)
    model.set_cuda()
    model.set_optimizer('adam', 1e-3, weight_decay=1e-6, lr_schedule=False)
    before = model._flat_param.clone()
    batch = {k: d[k] for k in ('xs', 'ys', 'x_lens', 'y_lens', 'ys_sub', 'y_lens_sub')}
    model, l, lm, ls = train_hierarchical_step(model, batch, 5.0)
    np.testing.assert_allclose(l, float(d['loss'][0]), rtol=1e-4)
    assert not torch.equal(before, model._flat_param)
    for task, V in ((0, kw['num_classes'] + 1), (1, kw['num_classes_sub'] + 1)):
        hyps, aw, perm = model.decode(d['xs'], d['x_lens'], beam_width=1, max_decode_len=6,
                                      task_index=task)
        assert hyps.shape[0] == len(d['xs']) and 1 <= hyps.shape[1] <= 6
        assert hyps.min() >= 0 and hyps.max() < V
        np.testing.assert_allclose(aw.sum(-1), 1.0, rtol=1e-4)
