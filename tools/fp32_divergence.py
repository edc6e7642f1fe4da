"""Where does the fp32 GPU encoder leave the float64 trajectory at the
reference initialisation (at T = 1000 the headline fp32
loss error is 3x the reference's own float32 error)?

ctc5x512's encoder (5 x 512 BLSTM, reference init, dropout off) on the bench's
first 6 synthetic utterances, layer by layer:
  f64  -- the oracle restatement (oracle/asr_ref.lstm_direction) in float64;
  cpu  -- the reference's own CPU float32 modules (torch nn.LSTM, one
          bidirectional layer at a time, packed sequences), each layer fed
          its own float32 output of the layer below;
  gpu  -- native_ops.blstm_layer in fp32 mode (the exact-f32 per-step kernels),
          each layer fed its own output of the layer below.
For every layer and direction: max |y - y64| over (utterance, unit) at
processing steps 0, 1, 10, 50, 100, 200, 500, 999 (forward direction: t = step;
reverse: t = len - 1 - step), and the error-growth exponent between steps 50
and 200 (log10 per 100 steps).  Same growth with a later onset = chaos
amplifying rounding; a step-0 or early jump = a systematic difference.

usage (GPU box): python tools/fp32_divergence.py > gpurun_out/fp32_divergence.txt
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle import asr_ref  # noqa: E402
from pytorch_end2end_speech_recognition_amd import native_ops as ops  # noqa: E402
from pytorch_end2end_speech_recognition_amd.models.load_model import load  # noqa: E402

STEPS = [0, 1, 10, 50, 100, 200, 500, 999]


def per_step_err(y, ref, lens, H, rev):
    """max over (b, unit) of |y - ref| at each processing step of a direction."""
    B, T, _ = y.shape
    d = (y - ref).abs()
    sl = slice(H, 2 * H) if rev else slice(0, H)
    out = np.zeros(T)
    for s in range(T):
        m = 0.0
        for b in range(B):
            if s >= lens[b]:
                continue
            t = lens[b] - 1 - s if rev else s
            m = max(m, float(d[b, t, sl].max()))
        out[s] = m
    return out


def main():
    torch.set_num_threads(min(16, len(os.sched_getaffinity(0))))
    cfg = bench.CONFIGS['ctc5x512']
    p = cfg['params']
    torch.manual_seed(1623)
    model = load(cfg['model_type'], dict(p), 'pytorch')
    sd = {k: v.detach().clone() for k, v in model.state_dict().items()}
    batch = bench.synthetic_batch(32, 1000, bench.input_dim(p), p['num_classes'], seed=0)
    n = 6
    xs = torch.from_numpy(batch['xs'][:n])
    lens = batch['x_lens'][:n].astype(np.int64)        # sorted descending
    L, H = p['encoder_num_layers'], p['encoder_num_units']
    dev = torch.device('cuda:0')

    def w(l, rev, dtype):
        sfx = '_reverse' if rev else ''
        pre = 'encoder.rnn.'
        keys = ['weight_ih_l%d%s', 'weight_hh_l%d%s', 'bias_ih_l%d%s', 'bias_hh_l%d%s']
        got = []
        for k in keys:
            name = [s for s in sd if s.endswith(k % (l, sfx)) and 'encoder' in s]
            got.append(sd[name[0]].to(dtype))
        return got

    x64 = xs.double()
    x32c = xs.float()
    x32g = xs.float().to(dev)
    lens_d = torch.from_numpy(lens.astype(np.int32)).to(dev)
    T = xs.shape[1]
    ops.set_compute_dtype('fp32')
    print('ctc5x512 encoder, reference init, %d utterances x %d frames, dropout off' % (n, T))
    with torch.no_grad():
        for l in range(L):
            y64 = torch.cat([asr_ref.lstm_direction(x64, lens, *w(l, r, torch.float64), r)
                             for r in (False, True)], dim=2)
            # the reference's own float32 CPU kernels: one bidirectional nn.LSTM layer
            lstm = torch.nn.LSTM(x32c.shape[2], H, 1, batch_first=True, bidirectional=True)
            for r in (False, True):
                sfx = '_reverse' if r else ''
                wi, wh, bi, bh = w(l, r, torch.float32)
                getattr(lstm, 'weight_ih_l0' + sfx).copy_(wi)
                getattr(lstm, 'weight_hh_l0' + sfx).copy_(wh)
                getattr(lstm, 'bias_ih_l0' + sfx).copy_(bi)
                getattr(lstm, 'bias_hh_l0' + sfx).copy_(bh)
            packed = torch.nn.utils.rnn.pack_padded_sequence(x32c, torch.from_numpy(lens),
                                                             batch_first=True)
            yc, _ = lstm(packed)
            yc, _ = torch.nn.utils.rnn.pad_packed_sequence(yc, batch_first=True, total_length=T)
            # the GPU op (fp32 mode), combined [fwd; rev] parameters
            wf, wr = w(l, False, torch.float32), w(l, True, torch.float32)
            comb = [torch.cat([a, b]).contiguous().to(dev) for a, b in zip(wf, wr)]
            yg = ops.blstm_layer(x32g, lens_d, T, *comb)
            torch.cuda.synchronize()
            for name, y in (('cpu', yc.double()), ('gpu', yg.double().cpu())):
                for r in (False, True):
                    e = per_step_err(y, y64, lens, H, r)
                    a, b = np.log10(max(e[50], 1e-30)), np.log10(max(e[200], 1e-30))
                    print('layer %d %s %-3s ' % (l, 'rev' if r else 'fwd', name) +
                          ' '.join('s%d %.1e' % (s, e[s]) for s in STEPS if s < T) +
                          '  growth %.2f dec/100 steps' % ((b - a) / 1.5))
            x64, x32c, x32g = y64, yc.detach(), yg.detach()
            sys.stdout.flush()


if __name__ == '__main__':
    main()
