"""AttentionMechanism (reference models/pytorch_v3/attention/attention_layer.py).

Same constructor, submodule and parameter names (W_enc_head0, W_dec_head0,
W_conv_head0, conv_head0 [Conv2d 1->C, (1, K)], V_head0; content attention
without the two conv modules) and the same torch RNG consumption, so
state_dicts interchange.  In training the location-attention
step runs inside the fused HIP decoder loop (native_ops.att_decoder,
csrc/decoder.hip); ``forward`` is the same step as a standalone op
(native_ops.att_step: the loop's kernels launched for one step): conv over the
previous weights, energy V.tanh(W_enc h_enc + W_dec h_dec + W_conv f),
MULTIPLICATIVE length mask (:216-225), sharpening, softmax (or sigmoid
smoothing) and the context vector, with a HIP backward.
"""
import numpy as np
import torch
import torch.nn as nn

from .... import native_ops as ops

from ..linear import LinearND

ATTENTION_TYPE = ['content', 'location', 'dot_product', 'rnn_attention', 'coverage']


class AttentionMechanism(nn.Module):

    def __init__(self, encoder_num_units, decoder_num_units, attention_type, attention_dim,
                 sharpening_factor=1, sigmoid_smoothing=False, out_channels=10, kernel_size=201,
                 num_heads=1):
        super(AttentionMechanism, self).__init__()
        if attention_type not in ATTENTION_TYPE:
            raise TypeError('attention_type should be one of [%s], you provided %s.' %
                            (', '.join(ATTENTION_TYPE), attention_type))
        if attention_type not in ('location', 'content') or num_heads != 1:
            raise NotImplementedError('MI355X decoder: location / content attention, 1 head '
                                      '(dot_product / rnn_attention / coverage / multi-head '
                                      'are not provided)')
        self.attention_type = attention_type
        self.attention_dim = attention_dim
        self.sharpening_factor = sharpening_factor
        self.sigmoid_smoothing = sigmoid_smoothing
        self.num_heads = num_heads
        self.out_channels = out_channels
        self.kernel_size = kernel_size
        # registration order = attention_layer.py:66-98 (RNG parity)
        self.W_enc_head0 = LinearND(encoder_num_units, attention_dim, bias=True)
        self.W_dec_head0 = LinearND(decoder_num_units, attention_dim, bias=False)
        if attention_type == 'location':
            assert kernel_size % 2 == 1
            self.W_conv_head0 = LinearND(out_channels, attention_dim, bias=False)
            self.conv_head0 = nn.Conv2d(in_channels=1, out_channels=out_channels,
                                        kernel_size=(1, kernel_size), stride=1,
                                        padding=(0, kernel_size // 2), bias=False)
        self.V_head0 = LinearND(attention_dim, 1, bias=False)

    def conv_weights(self):
        """(W_conv [A, C], conv kernel [C, 1, 1, K]) of the location term.  For
        content attention (:145-153: the same energy without that term) one
        all-zero channel of width 1: W_conv f adds an exact 0.0 to every
        pre-activation, so the location kernels compute the content energy
        bit for bit, and d aw_prev is 0; the gradients the kernels accumulate
        into these constant tensors are never read."""
        if self.attention_type == 'location':
            return self.W_conv_head0.fc.weight, self.conv_head0.weight
        w = self.W_dec_head0.fc.weight
        z = self.__dict__.get('_zero_conv')
        if z is None or z[0].device != w.device:
            z = (torch.zeros(self.attention_dim, 1, device=w.device),
                 torch.zeros(1, 1, 1, 1, device=w.device))
            self.__dict__['_zero_conv'] = z
        return z

    def forward(self, enc_out, enc_out_a, x_lens, dec_out, aw_step):
        """attention_layer.py:123-251 (location, one head).
        enc_out [B, T, E]; enc_out_a [B, T, A, 1] = W_enc(enc_out) (the caller's
        hoisted projection, attention_seq2seq.py:735-739); x_lens [B] (tensor,
        list or array); dec_out [B, 1, D]; aw_step [B, T, 1] (the previous
        step's weights).  Returns (context_vec [B, 1, E], aw_step [B, T, 1])."""
        B, T, E = enc_out.shape
        dev = enc_out.device
        if torch.is_tensor(x_lens):
            lens = x_lens.reshape(-1).to(device=dev, dtype=torch.int32)
        else:
            lens = ops.h2d(np.asarray(x_lens, np.int32).reshape(-1), dev)
        w_conv, conv_w = self.conv_weights()
        ctx, aw = ops.att_step(enc_out, enc_out_a.reshape(B, T, -1), lens,
                               dec_out.reshape(B, -1), aw_step.reshape(B, T),
                               self.W_dec_head0.fc.weight, w_conv, conv_w,
                               self.V_head0.fc.weight, self.sharpening_factor,
                               self.sigmoid_smoothing)
        return ctx.unsqueeze(1), aw.unsqueeze(2)
