"""CNNEncoder: the reference's VGG front-end (models/pytorch_v3/encoders/cnn.py)
on the MI355X HIP kernels (csrc/cnn.hip + tap-addressed MFMA GEMMs).

Same constructor arguments and the same ``layers`` nn.Sequential (Conv2d, ReLU,
MaxPool2d, BatchNorm2d, Dropout modules in the reference's order, cnn.py:74-122),
so state_dict keys, the construction-time RNG consumption and
``output_size`` are identical; the modules are parameter / running-stat
holders and their forwards never run.  Forward semantics (cnn.py:124-165):
input dropout, [B, T, F] viewed as [B, 1, F, T], per layer conv 3x3 ->
activation -> max-pool (first floor mode, later ceil mode) -> batch norm ->
dropout, output [B, T', F' * C], and x_lens from ConvOutSize (cnn_utils.py:
34-37) which applies the FLOOR rule to every pool, so a ceil-mode pool over an
odd length reports one frame fewer than the tensor holds (reference quirk).
"""
import math

import numpy as np
import torch.nn as nn

from .... import native_ops as ops


class CNNEncoder(nn.Module):

    def __init__(self, input_size, input_channel, conv_channels, conv_kernel_sizes, conv_strides,
                 poolings, dropout_input, dropout_hidden, activation='relu', batch_norm=False):
        super(CNNEncoder, self).__init__()
        self.input_channel = input_channel
        assert input_size % input_channel == 0
        self.input_freq = input_size // input_channel
        assert len(conv_channels) > 0
        assert len(conv_channels) == len(conv_kernel_sizes) == len(conv_strides) == len(poolings)
        unsupported = []
        if input_channel != 1:
            unsupported.append('input_channel=%d' % input_channel)
        if activation != 'relu':
            unsupported.append('activation=%s' % activation)
        for k, st, pl in zip(conv_kernel_sizes, conv_strides, poolings):
            if list(k) != [3, 3] or list(st) != [1, 1]:
                unsupported.append('conv kernel %s stride %s (3x3 / 1x1 only)' % (k, st))
            if len(pl) and (len(pl) != 2 or min(pl) < 1):
                unsupported.append('pooling %s' % (pl,))
        if unsupported:
            raise NotImplementedError('MI355X CNNEncoder: not yet supported: ' +
                                      ', '.join(unsupported))
        self.dropout_input_p = float(dropout_input)
        self.dropout_hidden_p = float(dropout_hidden)
        self.dropout_input = nn.Dropout(p=dropout_input)
        self.batch_norm = batch_norm

        layers, self._plan = [], []
        in_c, in_freq = self.input_channel, self.input_freq
        first_max_pool = True
        for l in range(len(conv_channels)):
            conv = nn.Conv2d(in_channels=in_c, out_channels=conv_channels[l],
                             kernel_size=tuple(conv_kernel_sizes[l]),
                             stride=tuple(conv_strides[l]), padding=tuple(conv_strides[l]),
                             bias=not batch_norm)
            layers.append(conv)
            in_freq = math.floor((in_freq + 2 * conv.padding[0] - conv.kernel_size[0]) /
                                 conv.stride[0] + 1)
            layers.append(nn.ReLU())
            pool = None
            if len(poolings[l]) > 0:
                pool = nn.MaxPool2d(kernel_size=tuple(poolings[l]), stride=tuple(poolings[l]),
                                    padding=(0, 0), ceil_mode=False if first_max_pool else True)
                first_max_pool = False
                layers.append(pool)
                in_freq = math.floor((in_freq + 2 * pool.padding[0] - pool.kernel_size[0]) /
                                     pool.stride[0] + 1)
            bn = None
            if batch_norm:
                bn = nn.BatchNorm2d(conv_channels[l])
                layers.append(bn)
            layers.append(nn.Dropout(p=dropout_hidden))
            self._plan.append((conv, pool, bn))
            in_c = conv_channels[l]
        self.layers = nn.Sequential(*layers)
        self.output_size = conv_channels[-1] * in_freq

    def conv_out_len(self, size, dim=1):
        """ConvOutSize (cnn_utils.py:25-37): floor rule for every conv and pool."""
        for m in self.layers:
            if type(m) in (nn.Conv2d, nn.MaxPool2d):
                pad = m.padding[dim] if isinstance(m.padding, tuple) else m.padding
                k = m.kernel_size[dim] if isinstance(m.kernel_size, tuple) else m.kernel_size
                st = m.stride[dim] if isinstance(m.stride, tuple) else m.stride
                size = math.floor((size + 2 * pad - k) / st + 1)
        return size

    def forward(self, xs, x_lens):
        """xs: device tensor [B, T, F]; x_lens: host ints [B].  Returns
        (xs [B, T', F'*C] f32 device tensor, x_lens numpy int32 [B])."""
        if self.training and self.dropout_input_p > 0:
            xs = ops.dropout(xs, self.dropout_input_p)
        specs = []
        for conv, pool, bn in self._plan:
            pt, pf = (pool.kernel_size[1], pool.kernel_size[0]) if pool is not None else (0, 0)
            specs.append(dict(w=conv.weight, b=conv.bias, pt=pt, pf=pf,
                              ceil=int(bool(pool is not None and pool.ceil_mode)),
                              gamma=bn.weight if bn is not None else None,
                              beta=bn.bias if bn is not None else None,
                              run_mean=bn.running_mean if bn is not None else None,
                              run_var=bn.running_var if bn is not None else None,
                              momentum=bn.momentum if bn is not None else 0.1,
                              eps=bn.eps if bn is not None else 1e-5, bn=bn))
        out = ops.vgg_front(xs, specs, self.training, self.dropout_hidden_p)
        lens = np.array([self.conv_out_len(int(x), 1) for x in np.asarray(x_lens)], np.int32)
        return out, lens
