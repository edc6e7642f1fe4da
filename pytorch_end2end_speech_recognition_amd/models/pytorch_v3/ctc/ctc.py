"""CTC model (reference models/pytorch_v3/ctc/ctc.py) on the MI355X hot path.

Drop-in: same constructor kwargs and defaults (ctc.py:115-145), same
``forward(xs, ys, x_lens, y_lens, is_eval=False)`` contract (numpy in; a
shape-[1] loss tensor in training, a Python float when ``is_eval``), same
``decode`` / ``posteriors`` return conventions, same state_dict keys.

Differences by design (MI355X-first):
  * the CTC loss is the HIP lattice kernel (native_ops.ctc_loss) on the
    batch-major logits -- no [T,B,V] transpose copy, lengths and labels stay on
    device, no host round trip of costs (ctc.py:319-326 did three);
  * the gradient is produced in backward already scaled by grad_output / B
    (the chain rule; SURVEY §8c decision for the unpinned warp-ctc binding);
  * infeasible alignments give cost 0 / gradient 0 (zero_infinity).
"""
import numpy as np
import torch

from .... import native_ops as ops
from ..base import ModelBase, check_recurrences, eval_retry
from ..linear import LinearND
from ..encoders.load_encoder import load
from ..criterion import cross_entropy_label_smoothing
from .decoders.greedy_decoder import GreedyDecoder


class _Head(object):
    """An output layer not applied yet: its input, the LinearND and the input
    dropout handed over by the encoder (CTC._encode(defer_head=True))."""
    __slots__ = ('x', 'fc', 'drop')

    def __init__(self, x, fc, drop):
        self.x, self.fc, self.drop = x, fc, drop


def _concatenate_labels_np(ys, y_lens):
    """ctc.py:532-549 on the host, vectorised: [B, L] padded -> int32 [sum L]."""
    ys = np.asarray(ys)
    y_lens = np.asarray(y_lens).astype(np.int64)
    mask = np.arange(ys.shape[1])[None, :] < y_lens[:, None]
    return np.ascontiguousarray(ys[mask]).astype(np.int32)


class CTC(ModelBase):
    """The Connectionist Temporal Classification model (ctc.py:72-113)."""

    def __init__(self, input_size, encoder_type, encoder_bidirectional, encoder_num_units,
                 encoder_num_proj, encoder_num_layers, fc_list, dropout_input, dropout_encoder,
                 num_classes, parameter_init_distribution='uniform', parameter_init=0.1,
                 recurrent_weight_orthogonal=False, init_forget_gate_bias_with_one=True,
                 subsample_list=[], subsample_type='drop', logits_temperature=1, num_stack=1,
                 splice=1, input_channel=1, conv_channels=[], conv_kernel_sizes=[],
                 conv_strides=[], poolings=[], activation='relu', batch_norm=False,
                 label_smoothing_prob=0, weight_noise_std=0, encoder_residual=False,
                 encoder_dense_residual=False):
        super(ModelBase, self).__init__()
        self.model_type = 'ctc'
        self.input_size = input_size
        self.num_stack = num_stack
        self.encoder_type = encoder_type
        self.encoder_num_units = encoder_num_units * (2 if encoder_bidirectional else 1)
        self.fc_list = fc_list
        self.fc_list_sub = []
        self.subsample_list = subsample_list
        self.num_classes = num_classes + 1
        self.logits_temperature = logits_temperature
        self.weight_noise_injection = False
        self.weight_noise_std = float(weight_noise_std)
        self.ls_prob = label_smoothing_prob

        if encoder_type in ['lstm', 'gru', 'rnn']:
            self.encoder = load(encoder_type=encoder_type)(
                input_size=input_size, rnn_type=encoder_type,
                bidirectional=encoder_bidirectional, num_units=encoder_num_units,
                num_proj=encoder_num_proj, num_layers=encoder_num_layers,
                dropout_input=dropout_input, dropout_hidden=dropout_encoder,
                subsample_list=subsample_list, subsample_type=subsample_type, batch_first=True,
                merge_bidirectional=False, pack_sequence=True, num_stack=num_stack,
                splice=splice, input_channel=input_channel, conv_channels=conv_channels,
                conv_kernel_sizes=conv_kernel_sizes, conv_strides=conv_strides,
                poolings=poolings, activation=activation, batch_norm=batch_norm,
                residual=encoder_residual, dense_residual=encoder_dense_residual, nin=0)
        else:
            raise NotImplementedError('encoder_type=%s' % encoder_type)

        # the first layer after the encoder folds the encoder's output dropout
        # into its product (bf16 mode; rnn.py:392-393 semantics, same mask)
        self.encoder.defer_output_dropout = True
        if len(fc_list) > 0:
            for i in range(len(fc_list)):
                din = self.encoder_num_units if i == 0 else fc_list[i - 1]
                setattr(self, 'fc_' + str(i), LinearND(din, fc_list[i], dropout=dropout_encoder))
            self.fc_out = LinearND(fc_list[-1], self.num_classes)
        else:
            self.fc_out = LinearND(self.encoder_num_units, self.num_classes)

        # ctc.py:248-264
        self.init_weights(parameter_init, distribution=parameter_init_distribution,
                          ignore_keys=['bias'])
        self.init_weights(0, distribution='constant', keys=['bias'])
        if recurrent_weight_orthogonal:
            self.init_weights(parameter_init, distribution='orthogonal',
                              keys=[encoder_type, 'weight'], ignore_keys=['bias'])
        if init_forget_gate_bias_with_one:
            self.init_forget_gate_bias_with_one()

        self._decode_greedy_np = GreedyDecoder(blank_index=0)
        self.flatten_parameters_()
        self.encoder.__dict__['_owner'] = self

    # ------------------------------------------------------------------
    @eval_retry
    def forward(self, xs, ys, x_lens, y_lens, is_eval=False):
        """ctc.py:272-342."""
        if is_eval:
            self.eval()
        else:
            self.train()
            if self.weight_noise_injection:
                self.inject_weight_noise(mean=0, std=self.weight_noise_std)
        B = len(xs)
        xs_d = self.np2var(xs, dtype='float')
        logits, out_lens_d, perm_d = self._encode(xs_d, x_lens, defer_head=True)
        if self.logits_temperature != 1:
            logits = logits * (1.0 / self.logits_temperature)

        loss = self._ctc_term(logits, out_lens_d, ys, y_lens, self.encoder.last_perm_np, B)
        if is_eval:
            check_recurrences(self)
            return float(loss.item())
        return loss

    def _head_fusable(self, fc):
        """The output layer and the CTC loss can run as one op (LinearCTCFn):
        nothing but the CTC term reads the logits."""
        return (self.logits_temperature == 1 and self.ls_prob == 0 and
                not (self.training and fc.dropout_p > 0))

    def _encode(self, xs, x_lens, is_multi_task=False, defer_head=False):
        """ctc.py:344-396.  defer_head: the output layer(s) whose only consumer
        is the CTC loss are returned as _Head(x, fc, drop) for _ctc_term's
        fused LinearND + CTC op instead of being applied here."""
        if is_multi_task:
            xs, x_lens, xs_sub, x_lens_sub, perm_idx = self.encoder(
                xs, x_lens, volatile=not self.training)
        else:
            xs, x_lens, perm_idx = self.encoder(xs, x_lens, volatile=not self.training)
        # the encoder's output dropout, when handed over, is folded into the
        # first layer that reads xs (LinearND input_drop: same mask)
        pd = self.encoder.pending_output_drop
        self.encoder.pending_output_drop = None
        for i in range(len(self.fc_list)):
            xs = getattr(self, 'fc_' + str(i))(xs, input_drop=pd)
            pd = None
        if defer_head and self._head_fusable(self.fc_out):
            logits = _Head(xs, self.fc_out, pd)
        else:
            logits = self.fc_out(xs, input_drop=pd)
        if is_multi_task:
            for i in range(len(self.fc_list_sub)):
                xs_sub = getattr(self, 'fc_sub_' + str(i))(xs_sub)
            if defer_head and self._head_fusable(self.fc_out_sub):
                logits_sub = _Head(xs_sub, self.fc_out_sub, None)
            else:
                logits_sub = self.fc_out_sub(xs_sub)
            return logits, x_lens, logits_sub, x_lens_sub, perm_idx
        return logits, x_lens, perm_idx

    def _ctc_term(self, logits, lens_d, ys, y_lens, perm, B):
        """sum_b cost_b / B on the HIP CTC kernel (+ label smoothing, ctc.py:319-337)."""
        ys_s = (np.asarray(ys) + 1)[perm]                      # blank = 0 (ctc.py:300)
        yl_s = np.asarray(y_lens).astype(np.int32)[perm]
        labels = self.np2var(_concatenate_labels_np(ys_s, yl_s))
        yl_d = self.np2var(yl_s)
        max_l = int(yl_s.max()) if len(yl_s) else 0
        if isinstance(logits, _Head):     # LinearND + CTC as one op (no f32 d logits)
            h = logits
            loss, _ = ops.linear_ctc_loss(h.x, h.fc.fc.weight, h.fc.fc.bias, labels, yl_d, lens_d,
                                          max_l, loss_scale=1.0 / B, drop=h.drop)
            return loss
        loss, _ = ops.ctc_loss(logits, labels, yl_d, lens_d, max_l, loss_scale=1.0 / B)
        if self.ls_prob > 0:
            loss_ls = cross_entropy_label_smoothing(
                logits, y_lens=lens_d, label_smoothing_prob=self.ls_prob,
                distribution='uniform', size_average=False) * (1.0 / B)
            loss = loss * (1 - self.ls_prob) + loss_ls
        return loss

    def inject_weight_noise(self, mean, std):
        """base.py:85-99 (Gaussian weight noise; not on the default hot path)."""
        with torch.no_grad():
            self._flat_param.add_(torch.randn_like(self._flat_param) * std + mean)

    @eval_retry
    @torch.no_grad()
    def decode(self, xs, x_lens, beam_width, max_decode_len=None, min_decode_len=0,
               length_penalty=0, coverage_penalty=0, task_index=0):
        """ctc.py:398-452.  beam_width == 1: device best path (HIP kernel);
        returns (best_hyps [B] object array of int arrays, None, perm_idx)."""
        self.eval()
        if beam_width != 1:
            raise NotImplementedError('CTC prefix beam search is host-side inference, out of '
                                      'the training hot path (SURVEY §2 #12)')
        xs_d = self.np2var(xs, dtype='float')
        logits, out_lens_d, perm_d = self._encode(xs_d, x_lens)
        check_recurrences(self)
        best_hyps = self._decode_greedy_np(logits, out_lens_d)
        best_hyps = np.array([h - 1 for h in best_hyps] + [None], dtype=object)[:-1]
        return best_hyps, None, self.encoder.last_perm_np.copy()

    @eval_retry
    @torch.no_grad()
    def posteriors(self, xs, x_lens, temperature=1, blank_scale=None, task_idx=0):
        """ctc.py:455-502."""
        self.eval()
        if blank_scale is not None:
            raise NotImplementedError
        xs_d = self.np2var(xs, dtype='float')
        logits, out_lens_d, perm_d = self._encode(xs_d, x_lens)
        check_recurrences(self)
        probs = ops.softmax(logits * (1.0 / temperature))
        return self.var2np(probs), self.encoder.last_lens_np.copy(), \
            self.encoder.last_perm_np.copy()

    def decode_from_probs(self, probs, x_lens, beam_width=1, max_decode_len=None):
        """ctc.py:504-529 (host numpy, as the reference)."""
        if beam_width != 1:
            raise NotImplementedError
        log_probs = np.log(probs + 1e-10)
        best = self._decode_greedy_np(log_probs, x_lens)
        return np.array([h - 1 for h in best] + [None], dtype=object)[:-1]
