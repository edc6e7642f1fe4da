"""RNNEncoder: the reference's (B)LSTM / (B)GRU encoder
(models/pytorch_v3/encoders/rnn.py) on the MI355X HIP layer ops.

Same constructor kwargs, same parameter names (``lstm.weight_ih_l{l}[_reverse]``
for the fast path, ``lstm_l{l}.weight_ih_l0[_reverse]`` for the per-layer path,
``gru...`` likewise: rnn.py:162-246) and the same torch RNG consumption at
construction, so a model built under the same seed holds bit-identical initial
weights.  ``nn.LSTM`` / ``nn.GRU`` modules are used only as parameter holders;
their forward never runs (GRU layers: native_ops.bgru_layer, csrc/gru.hip).

Forward semantics (rnn.py:284-487): input dropout, the optional VGG front-end
(encoders/cnn.py, rnn.py:143-160, 314-316), length sort (perm_idx is
returned; outputs stay in sorted order), packed-sequence behaviour through
per-utterance length masks, dropout after every layer, and between layers
(rnn.py:409-465): the projection ``tanh(proj_l(x))``, pyramidal ``drop``
subsampling ``xs[:, 1::2]`` or ``concat`` subsampling (successive frame pairs
side by side) -- both read in place by the next layer's input GEMM through its
row map -- and residual / dense-residual sums from the last subsampling layer
on; plus the reference's x_lens quirk: after any subsampling every
utterance's length is the padded length (rnn.py:435-439).
"""
import numpy as np
import torch
import torch.nn as nn

from .... import native_ops as ops
from ..linear import LinearND
from .cnn import CNNEncoder


class RNNEncoder(nn.Module):

    def __init__(self, input_size, rnn_type, bidirectional, num_units, num_proj, num_layers,
                 dropout_input, dropout_hidden, subsample_list=[], subsample_type='drop',
                 use_cuda=False, batch_first=False, merge_bidirectional=False,
                 pack_sequence=True, num_stack=1, splice=1, input_channel=1, conv_channels=[],
                 conv_kernel_sizes=[], conv_strides=[], poolings=[], activation='relu',
                 batch_norm=False, residual=False, dense_residual=False, num_layers_sub=0,
                 nin=0):
        super(RNNEncoder, self).__init__()
        if len(subsample_list) > 0 and len(subsample_list) != num_layers:
            raise ValueError('subsample_list must be the same size as num_layers.')
        if subsample_type not in ['drop', 'concat']:
            raise TypeError('subsample_type must be "drop" or "concat".')
        if num_layers_sub < 0 or (num_layers_sub > 1 and num_layers < num_layers_sub):
            raise ValueError('Set num_layers_sub between 1 to num_layers.')
        if rnn_type not in ('lstm', 'gru', 'rnn'):
            raise ValueError('rnn_type must be "lstm" or "gru" or "rnn".')
        unsupported = []
        if rnn_type == 'rnn':
            unsupported.append('rnn_type=rnn')
        if not bidirectional:
            unsupported.append('unidirectional')
        if nin or merge_bidirectional or not batch_first or not pack_sequence:
            unsupported.append('nin/merge/time-major/no-pack')
        if unsupported:
            raise NotImplementedError('MI355X RNNEncoder: not yet supported: ' +
                                      ', '.join(unsupported))

        self.rnn_type = rnn_type
        self.bidirectional = bidirectional
        self.num_directions = 2
        self.num_units = num_units
        self.num_proj = num_proj if num_proj is not None else 0
        self.num_layers = num_layers
        self.batch_first = batch_first
        self.pack_sequence = pack_sequence
        self.num_layers_sub = num_layers_sub
        self.subsample_list = list(subsample_list) if len(subsample_list) else [False] * num_layers
        self.subsample_type = subsample_type
        self.dropout_input_p = float(dropout_input)
        self.dropout_hidden_p = float(dropout_hidden)
        # set by a model whose head consumes the output directly: the last
        # layer's dropout is then handed over in pending_output_drop instead of
        # applied (the head folds it into its product; training mode only)
        self.defer_output_dropout = False
        self.pending_output_drop = None
        self.dropout_input = nn.Dropout(p=dropout_input)
        self.batch_norm = batch_norm
        assert not (residual and dense_residual)
        self.residual = residual
        self.dense_residual = dense_residual
        subsample_last_layer = 0                      # rnn.py:126-133
        for l_reverse, is_subsample in enumerate(self.subsample_list[::-1]):
            if is_subsample:
                subsample_last_layer = num_layers - l_reverse
                break
        self.residual_start_layer = subsample_last_layer + 1
        if len(conv_channels) > 0 and len(conv_channels) == len(conv_kernel_sizes) and \
                len(conv_kernel_sizes) == len(conv_strides):   # rnn.py:143-160
            assert num_stack == 1 and splice == 1
            self.conv = CNNEncoder(input_size, input_channel=input_channel,
                                   conv_channels=conv_channels,
                                   conv_kernel_sizes=conv_kernel_sizes,
                                   conv_strides=conv_strides, poolings=poolings, dropout_input=0,
                                   dropout_hidden=dropout_hidden, activation=activation,
                                   batch_norm=batch_norm)
            input_size = self.conv.output_size
        else:
            self.conv = None
            input_size = input_size * splice * num_stack
        self.input_size = input_size

        # rnn.py:162 (batch_norm forces the per-layer modules, as in the reference)
        self.fast_impl = (sum(self.subsample_list) == 0 and self.num_proj == 0 and not residual and
                          not dense_residual and num_layers_sub == 0 and not batch_norm)
        cell = nn.LSTM if rnn_type == 'lstm' else nn.GRU
        if self.fast_impl:   # rnn.py:162-198: one multi-layer nn.LSTM / nn.GRU
            setattr(self, rnn_type,
                    cell(input_size, hidden_size=num_units, num_layers=num_layers, bias=True,
                         batch_first=batch_first, dropout=dropout_hidden, bidirectional=True))
            self.dropout_last = nn.Dropout(p=dropout_hidden)
        else:                # rnn.py:200-251: one nn.LSTM / nn.GRU per layer (+ projection)
            for l in range(num_layers):
                if l == 0:
                    din = input_size
                else:
                    din = self.num_proj if self.num_proj > 0 else num_units * 2
                    if subsample_type == 'concat' and self.subsample_list[l - 1]:
                        din *= 2
                setattr(self, '%s_l%d' % (rnn_type, l),
                        cell(din, hidden_size=num_units, num_layers=1, bias=True,
                             batch_first=batch_first, dropout=0, bidirectional=True))
                setattr(self, 'dropout_l%d' % l, nn.Dropout(p=dropout_hidden))
                if l != num_layers - 1 and self.num_proj > 0:
                    setattr(self, 'proj_l%d' % l,
                            LinearND(num_units * 2, self.num_proj, dropout=dropout_hidden))

    # parameters of layer l: (w_ih_f, w_ih_r), (w_hh_f, w_hh_r), (b_ih_f, b_ih_r), (b_hh_f, b_hh_r)
    def _layer_params(self, l):
        if self.fast_impl:
            mod, k = getattr(self, self.rnn_type), l
        else:
            mod, k = getattr(self, '%s_l%d' % (self.rnn_type, l)), 0
        return [(getattr(mod, '%s_l%d' % (n, k)), getattr(mod, '%s_l%d_reverse' % (n, k)))
                for n in ('weight_ih', 'weight_hh', 'bias_ih', 'bias_hh')]

    def flat_order(self):
        """Forward and reverse tensors of each LSTM weight adjacent in the flat
        buffer, so one GEMM / one recurrence launch covers both directions."""
        groups = []
        for l in range(self.num_layers):
            for pair in self._layer_params(l):
                groups.append(list(pair))
        return groups

    def _layer_tensors(self, l):
        """Combined [fwd; rev] views (params and their grads) of layer l."""
        model = self._owner
        ts, gs = [], []
        for f, r in self._layer_params(l):
            n = f.numel() + r.numel()
            shape = (f.shape[0] * 2,) + tuple(f.shape[1:])
            ts.append(model.flat_view(f, n).view(shape))
            gs.append(model.flat_view(f, n, grad=True).view(shape))
        return ts, gs

    def forward(self, xs, x_lens, volatile=False):
        """xs: device tensor [B, T, input_size]; x_lens: numpy / list / tensor [B].
        Returns (xs [B, T', 2H], x_lens int32 device tensor [B], perm_idx int64
        device tensor [B]) like rnn.py:284-487; host copies of the output
        lengths and perm are kept in ``self.last_lens_np`` / ``self.last_perm_np``."""
        if torch.is_tensor(x_lens):
            x_lens = x_lens.detach().cpu().numpy()
        x_lens = np.asarray(x_lens).astype(np.int64)
        dev = xs.device
        if self.training and self.dropout_input_p > 0:
            xs = ops.dropout(xs, self.dropout_input_p)
        if self.conv is not None:                                   # rnn.py:314-316
            self.conv.train(self.training)
            xs, x_lens = self.conv(xs, x_lens)
            x_lens = x_lens.astype(np.int64)

        perm = np.argsort(-x_lens, kind='stable')                   # rnn.py:319-326
        lens = x_lens[perm]
        perm_d = ops.h2d(perm.astype(np.int32), dev)
        T = int(lens.max())                                          # pad_packed length
        h, pm, t_mul, t_add, concat = xs.contiguous(), perm_d, 1, 0, False
        h_sub = lens_sub = None
        res_outputs = []
        pending = None   # (p, seed): this layer's dropout, fused into the next layer's staging
        self.pending_output_drop = None
        lens_d, lens_key = None, None
        if self.rnn_type != 'gru':
            # one fill for the recurrence workspaces of every layer's forward and
            # backward pass (instead of a memset launch before each)
            ops.rec_arena_begin(dev, int(h.shape[0]), self.num_units, 2 * self.num_layers)
        for l in range(self.num_layers):
            (w_ih, w_hh, b_ih, b_hh), gbufs = self._layer_tensors(l)
            # one H2D copy per distinct length vector (they change only where a
            # layer subsamples), not one per layer on the compute stream
            if lens_key is None or not np.array_equal(lens_key, lens):
                lens_key = lens.copy()
                lens_d = ops.h2d(lens.astype(np.int32), dev)
            graph = tuple(p for pair in self._layer_params(l) for p in pair)
            if self.rnn_type == 'gru':
                if pending is not None:
                    h = ops.dropout(h, pending[0], seed=pending[1])
                h = ops.bgru_layer(h, lens_d, T, w_ih, w_hh, b_ih, b_hh, perm=pm, t_mul=t_mul,
                                   t_add=t_add, gbufs=tuple(gbufs), graph_params=graph,
                                   concat=concat)
            # this layer's output feeds only the next BLSTM layer, through an
            # identity row map: bf16 mode hands it over as that layer's staged
            # bf16 input (dropout applied) instead of an f32 tensor
            handoff = (self.rnn_type != 'gru' and ops.fuse_dropout_ok() and
                       l < self.num_layers - 1 and
                       not (self.num_layers_sub >= 1 and l == self.num_layers_sub - 1) and
                       not (self.residual or self.dense_residual or self.num_proj > 0) and
                       not self.subsample_list[l])
            drop_out = self.training and self.dropout_hidden_p > 0
            # same seed stream either way (one seed per layer, drawn in order)
            seed = ops.next_seed() if drop_out and handoff else None
            if self.rnn_type != 'gru':
                h = ops.blstm_layer(h, lens_d, T, w_ih, w_hh, b_ih, b_hh, perm=pm, t_mul=t_mul,
                                    t_add=t_add, gbufs=tuple(gbufs), graph_params=graph,
                                    concat=concat, drop=pending, next_rec=l > 0,
                                    bf16_handoff=handoff,
                                    out_drop=(self.dropout_hidden_p, seed) if seed is not None
                                    else None)
            pending = None
            if drop_out:
                # fused when the next consumer is the next layer's input staging
                # and nothing else reads the dropped h
                if seed is None:
                    seed = ops.next_seed()
                if (ops.fuse_dropout_ok() and l < self.num_layers - 1 and
                        not (self.num_layers_sub >= 1 and l == self.num_layers_sub - 1) and
                        not (self.residual or self.dense_residual or self.num_proj > 0) and
                        not (self.subsample_list[l] and self.subsample_type != 'drop')):
                    pending = (self.dropout_hidden_p, seed)
                elif (l == self.num_layers - 1 and self.defer_output_dropout and
                      self.num_layers_sub < 1 and ops.fuse_dropout_ok()):
                    # the owning model folds the output dropout into its head's
                    # product (LinearND input_drop); same seed, same mask
                    self.pending_output_drop = (self.dropout_hidden_p, seed)
                else:
                    h = ops.dropout(h, self.dropout_hidden_p, seed=seed)
            if self.num_layers_sub >= 1 and l == self.num_layers_sub - 1:   # rnn.py:400-407
                h_sub, lens_sub = h, lens.astype(np.int32)
            pm, t_mul, t_add, concat = None, 1, 0, False
            if l == self.num_layers - 1 or not (self.residual or self.dense_residual or
                                                self.num_proj > 0 or self.subsample_list[l]):
                continue
            if self.num_proj > 0:                                    # rnn.py:409-411
                h = ops.tanh(getattr(self, 'proj_l%d' % l)(h))
            if self.subsample_list[l]:                               # rnn.py:413-439
                # fused into the next layer's input GEMM: 'drop' reads frame 2t+1,
                # 'concat' reads frames 2t and 2t+1 as one row of twice the width
                T = T // 2
                if self.subsample_type == 'drop':
                    t_mul, t_add = 2, 1
                else:
                    t_mul, t_add, concat = 2, 0, True
                lens = np.full_like(lens, T)
            elif (self.residual or self.dense_residual) and l >= self.residual_start_layer - 1:
                for lower in res_outputs:                            # rnn.py:454-462
                    h = ops.add(h, lower)
                res_outputs = [h] if self.residual else res_outputs + [h]
        assert t_mul == 1
        self.last_lens_np = lens.astype(np.int32)
        self.last_perm_np = perm.astype(np.int64)
        out_lens = ops.h2d(self.last_lens_np, dev)
        perm_idx = ops.h2d(self.last_perm_np, dev)
        if self.num_layers_sub >= 1:                              # rnn.py:479-487
            self.last_lens_sub_np = lens_sub
            lens_sub_d = ops.h2d(lens_sub, dev)
            return h, out_lens, h_sub, lens_sub_d, perm_idx
        return h, out_lens, perm_idx
