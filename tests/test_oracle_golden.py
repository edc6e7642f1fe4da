"""Pin the CPU oracle against golden vectors produced by the reference itself
(tests/golden/make_golden.py).  CPU only."""
import json

import numpy as np
import pytest
import torch

from conftest import golden, golden_params
from oracle import asr_ref, ctc_ref


def _g(v):
    return np.zeros(v.shape, np.float32) if v.grad is None else v.grad.numpy()


@pytest.mark.parametrize('name', ['ctc_v6', 'ctc_v29', 'ctc_v1000'])
def test_ctc_oracle_matches_golden(name):
    d = golden(name)
    costs, grads = ctc_ref.ctc_batch(d['acts'], d['labels'], d['label_lens'], d['act_lens'])
    np.testing.assert_allclose(costs, d['costs'], rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(grads, d['grads'], rtol=1e-4, atol=1e-5)


@pytest.mark.parametrize('name', ['enc_fast', 'enc_sub'])
def test_encoder_oracle_matches_golden(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    p, g = golden_params(d)
    for v in p.values():
        v.requires_grad_(True)
    xs = torch.from_numpy(d['xs']).requires_grad_(True)
    out, lens, perm = asr_ref.blstm_encoder(p, '', kw, xs, d['x_lens'])
    np.testing.assert_array_equal(perm, d['perm'])
    np.testing.assert_array_equal(lens, d['out_lens'])
    np.testing.assert_allclose(out.detach().numpy(), d['out'], rtol=1e-5, atol=1e-6)
    (out * torch.from_numpy(d['R'])).sum().backward()
    np.testing.assert_allclose(xs.grad.numpy(), d['dxs'], rtol=1e-4, atol=1e-6)
    for k, v in p.items():
        np.testing.assert_allclose(_g(v), g[k], rtol=1e-4, atol=1e-6, err_msg=k)


def test_attention_step_oracle_matches_golden():
    d = golden('att_step')
    kw = json.loads(str(d['kwargs']))
    p, g = golden_params(d)
    for v in p.values():
        v.requires_grad_(True)
    enc_out = torch.from_numpy(d['enc_out']).requires_grad_(True)
    enc_out_a = torch.from_numpy(d['enc_out_a'][..., 0]).requires_grad_(True)
    dec_out = torch.from_numpy(d['dec_out'][:, 0]).requires_grad_(True)
    aw_in = torch.from_numpy(d['aw_in'][..., 0]).requires_grad_(True)
    ctx, aw = asr_ref.location_attention(p, '', enc_out, enc_out_a, d['x_lens'], dec_out,
                                         aw_in, kw['sharpening_factor'])
    np.testing.assert_allclose(ctx.detach().numpy(), d['ctx'][:, 0], rtol=1e-5, atol=1e-6)
    np.testing.assert_allclose(aw.detach().numpy(), d['aw_out'][..., 0], rtol=1e-5, atol=1e-7)
    ((ctx * torch.from_numpy(d['Rc'][:, 0])).sum()
     + (aw * torch.from_numpy(d['Ra'][..., 0])).sum()).backward()
    np.testing.assert_allclose(enc_out.grad.numpy(), d['d_enc_out'], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(enc_out_a.grad.numpy(), d['d_enc_out_a'][..., 0],
                               rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(dec_out.grad.numpy(), d['d_dec_out'][:, 0], rtol=1e-4, atol=1e-6)
    np.testing.assert_allclose(aw_in.grad.numpy(), d['d_aw_in'][..., 0], rtol=1e-4, atol=1e-6)
    for k, v in p.items():
        np.testing.assert_allclose(_g(v), g[k], rtol=1e-4, atol=1e-6, err_msg=k)


CTC_MODELS = ['model_ctc_sub', 'model_ctc_fast', 'model_ctc_gru_fast', 'model_ctc_gru_sub',
              'model_ctc_proj', 'model_ctc_concat',
              'model_ctc_proj_concat', 'model_ctc_res', 'model_ctc_dres']


def ctc_cfg(kw):
    """Oracle encoder config from the CTC constructor kwargs."""
    return dict(num_layers=kw['encoder_num_layers'], subsample_list=kw['subsample_list'],
                fc_list=kw['fc_list'], num_proj=kw.get('encoder_num_proj', 0),
                subsample_type=kw.get('subsample_type', 'drop'),
                residual=kw.get('encoder_residual', False),
                dense_residual=kw.get('encoder_dense_residual', False),
                rnn_type=kw.get('encoder_type', 'lstm'))


@pytest.mark.parametrize('name', CTC_MODELS)
def test_ctc_model_oracle_matches_golden(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    cfg = ctc_cfg(kw)
    p, g = golden_params(d)
    for v in p.values():
        v.requires_grad_(True)
    loss, logits, out_lens, perm = asr_ref.ctc_model_loss(p, cfg, d['xs'], d['ys'],
                                                          d['x_lens'], d['y_lens'])
    np.testing.assert_allclose(float(loss), float(d['loss'][0]), rtol=1e-5)
    np.testing.assert_allclose(logits.detach().numpy(), d['logits'], rtol=1e-5, atol=1e-6)
    np.testing.assert_array_equal(perm, d['perm'])
    np.testing.assert_array_equal(out_lens, d['out_lens'])
    loss.backward()
    for k, v in p.items():
        np.testing.assert_allclose(_g(v), g[k], rtol=1e-4, atol=1e-6, err_msg=k)
    hyps = ctc_ref.greedy_best_path(d['logits'], d['out_lens'])
    np.testing.assert_array_equal([len(h) for h in hyps], d['hyp_lens'])
    flat = np.concatenate(hyps) - 1 if len(hyps) else np.zeros(0)
    np.testing.assert_array_equal(flat, d['hyp_flat'])


@pytest.mark.parametrize('name', ['model_att', 'model_att_hybrid', 'model_att_ls', 'model_att_mean'])
def test_attention_model_oracle_matches_golden(name):
    d = golden(name)
    kw = json.loads(str(d['kwargs']))
    p, g = golden_params(d)
    for v in p.values():
        v.requires_grad_(True)
    loss = asr_ref.attention_model_loss(p, kw, d['xs'], d['ys'], d['x_lens'], d['y_lens'])
    np.testing.assert_allclose(float(loss), float(d['loss'][0]), rtol=1e-5)
    loss.backward()
    pad = asr_ref.embedding_padding_row(kw)
    for k, v in p.items():
        gv = v.grad.numpy().copy()
        if k == 'embed_0.embed.weight':
            gv[pad] = 0
        np.testing.assert_allclose(gv, g[k], rtol=1e-4, atol=1e-6, err_msg=k)
