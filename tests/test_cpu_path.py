"""oracle/cpu_path.py (the packed nn.LSTM CPU path bench.py times as the
reference CPU baseline) against the fixture recorded from the reference
itself (tests/golden/model_ctc_fast.npz: fast-path BLSTM CTC, loss and every
gradient) and against the oracle's restatement."""
import json

import numpy as np
import torch

from oracle import asr_ref
from oracle.cpu_path import CTCCPUPath, eval_loss


def _golden():
    d = np.load('tests/golden/model_ctc_fast.npz')
    kw = json.loads(str(d['kwargs']))
    sd = {k[3:]: torch.from_numpy(d[k].copy()) for k in d.files if k.startswith('sd/')}
    return d, kw, sd


def test_cpu_path_matches_reference_fixture():
    d, kw, sd = _golden()
    m = CTCCPUPath(kw['input_size'], kw['encoder_num_units'], kw['encoder_num_layers'],
                   kw['num_classes'])
    m.load_reference_state(sd)
    batch = dict(xs=d['xs'], ys=d['ys'], x_lens=d['x_lens'], y_lens=d['y_lens'])
    assert abs(eval_loss(m, batch) - float(d['loss'][0])) <= 1e-5 * abs(float(d['loss'][0]))
    m.train()
    m.zero_grad()
    m.loss(d['xs'], d['ys'], d['x_lens'], d['y_lens']).backward()
    for name, prm in m.named_parameters():
        ref = 'encoder.lstm.' + name[5:] if name.startswith('lstm.') else 'fc_out.fc.' + name[3:]
        np.testing.assert_allclose(prm.grad.numpy(), d['grad/' + ref], rtol=1e-4, atol=1e-6,
                                   err_msg=name)


def test_cpu_path_matches_oracle_restatement():
    rng = np.random.RandomState(3)
    B, T, Fd, H, V = 3, 40, 12, 8, 9
    m = CTCCPUPath(Fd, H, 2, V)
    sd = {'encoder.lstm.' + k[5:]: v.detach().clone() for k, v in m.state_dict().items()
          if k.startswith('lstm.')}
    sd.update({'fc_out.fc.' + k[3:]: v.detach().clone() for k, v in m.state_dict().items()
               if k.startswith('fc.')})
    x_lens = np.array([33, 40, 21], np.int32)
    y_lens = np.array([5, 7, 3], np.int32)
    xs = rng.randn(B, T, Fd).astype(np.float32)
    ys = np.full((B, 7), -1, np.int32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
        ys[b, :y_lens[b]] = rng.randint(0, V, y_lens[b])
    got = eval_loss(m, dict(xs=xs, ys=ys, x_lens=x_lens, y_lens=y_lens))
    ref, _, _, _ = asr_ref.ctc_model_loss(sd, dict(num_layers=2, subsample_list=[], fc_list=[]),
                                          xs, ys, x_lens, y_lens)
    np.testing.assert_allclose(got, float(ref), rtol=1e-5)
