"""The reference's CPU training path for the BLSTM-CTC models, restated with the
same torch CPU modules it uses (oracle; test / bench-baseline infrastructure
only, never imported by the product package).

What the reference runs on CPU for a CTC model (models/pytorch_v3/ctc/ctc.py
:272-342 with encoders/rnn.py fast path :166-172, :319-390):
  * sort the batch by length (rnn.py:319-326), ``pack_padded_sequence`` ->
    ONE multi-layer bidirectional ``nn.LSTM`` (batch_first, inter-layer
    dropout) -> ``pad_packed_sequence`` (rnn.py:343-390), dropout on the output;
  * ``fc_out`` (LinearND = ``nn.Linear`` on the last dim, linear.py:32-47);
  * warp-ctc on ``[T, B, V]`` acts with softmax inside, blank 0, summed over
    utterances, divided by B (ctc.py:319-323) -- restated with
    ``F.ctc_loss(log_softmax(.), reduction='sum')`` (the
    designated stand-in for the unvendored warp-ctc);
  * ``clip_grad_norm(5.0)`` and ``optim.Adam(weight_decay)``
    (utils/training/training_loop.py:27-83, base.py:141-213).

Parameters load from a state_dict keyed by the reference's names
(``encoder.lstm.weight_ih_l{l}{_reverse}``, ``fc_out.fc.weight``), so the GPU
model's initial state_dict drives it directly.  This is what bench.py times as
``cpu_baseline`` (kind "port") and uses as the loss oracle of its ``parity``
field.
"""
import time

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F
from torch.nn.utils.rnn import pack_padded_sequence, pad_packed_sequence


class CTCCPUPath(nn.Module):
    def __init__(self, input_size, num_units, num_layers, num_classes, dropout_input=0.0,
                 dropout_encoder=0.0):
        super().__init__()
        self.lstm = nn.LSTM(input_size, num_units, num_layers=num_layers, bias=True,
                            batch_first=True, dropout=dropout_encoder, bidirectional=True)
        self.fc = nn.Linear(2 * num_units, num_classes + 1)     # + blank (ctc.py:98)
        self.p_in = float(dropout_input)
        self.p_enc = float(dropout_encoder)

    def load_reference_state(self, sd):
        own = {}
        for k, v in sd.items():
            if k.startswith('encoder.lstm.'):
                own['lstm.' + k[len('encoder.lstm.'):]] = v
            elif k.startswith('fc_out.fc.'):
                own['fc.' + k[len('fc_out.fc.'):]] = v
        self.load_state_dict(own)

    def loss(self, xs, ys, x_lens, y_lens):
        """ctc.py:272-342: returns the [1]-shaped loss sum_b cost_b / B."""
        B = len(xs)
        x = torch.from_numpy(np.asarray(xs, np.float32)).to(self.fc.weight.dtype)
        x = F.dropout(x, self.p_in, self.training)
        x_lens = np.asarray(x_lens)
        perm = np.argsort(-x_lens, kind='stable')                 # rnn.py:319-326
        x = x[torch.as_tensor(perm)]
        lens = x_lens[perm]
        packed = pack_padded_sequence(x, torch.as_tensor(lens, dtype=torch.long),
                                      batch_first=True)
        out, _ = self.lstm(packed)
        h, _ = pad_packed_sequence(out, batch_first=True)
        h = F.dropout(h, self.p_enc, self.training)               # rnn.py:393 (last layer)
        logits = self.fc(h)                                        # [B, T, V]
        ys_s = (np.asarray(ys) + 1)[perm]                          # blank = 0 (ctc.py:300)
        yl_s = np.asarray(y_lens)[perm]
        labels = torch.from_numpy(np.concatenate(
            [ys_s[b, :yl_s[b]] for b in range(B)]).astype(np.int64))
        lp = torch.log_softmax(logits.transpose(0, 1), dim=-1)     # [T, B, V] (ctc.py:319)
        cost = F.ctc_loss(lp, labels, torch.as_tensor(lens, dtype=torch.long),
                          torch.as_tensor(yl_s, dtype=torch.long), blank=0,
                          reduction='sum', zero_infinity=True)
        return (cost / B).reshape(1)


def ctc_cpu_path(params, state_dict):
    mult = 1 + int(bool(params.get('use_delta'))) + int(bool(params.get('use_double_delta')))
    m = CTCCPUPath(params['input_freq'] * mult,      # load_model.py input_size rule
                   params['encoder_num_units'], params['encoder_num_layers'],
                   params['num_classes'], params.get('dropout_input', 0),
                   params.get('dropout_encoder', 0))
    m.load_reference_state(state_dict)
    return m


def eval_loss(model, batch, dtype=None):
    """Dropout-free loss (the parity reference for the GPU's is_eval loss);
    dtype=torch.float64 evaluates the same path in double precision."""
    if dtype is not None:
        import copy
        model = copy.deepcopy(model).to(dtype)
    model.eval()
    with torch.no_grad():
        return float(model.loss(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens']))


def time_train_step(model, batch, lr, weight_decay, clip):
    """One full reference training step (training_loop.py:27-83) on CPU;
    returns (seconds, loss)."""
    model.train()
    opt = torch.optim.Adam(model.parameters(), lr=lr, weight_decay=weight_decay)
    t0 = time.perf_counter()
    opt.zero_grad()
    loss = model.loss(batch['xs'], batch['ys'], batch['x_lens'], batch['y_lens'])
    loss.backward()
    torch.nn.utils.clip_grad_norm_(model.parameters(), clip)
    opt.step()
    lv = float(loss.item())
    return time.perf_counter() - t0, lv
