"""RNNDecoder (reference models/pytorch_v3/attention/rnn_decoder.py).

Same constructor, parameter names (``lstm_l{l}.weight_ih`` / ``gru_l{l}...``)
and RNG consumption.  In training the 1-layer LSTMCell step is fused into the HIP
decoder loop (csrc/decoder.hip cell_fwd / cell_bwd, AttentionSeq2seq);
``forward`` is the reference's layer API (rnn_decoder.py:63-113) on the HIP
GEMM (native_ops.linear2) + LSTM-cell kernels, for any number of layers,
residual / dense-residual connections and dropout.
"""
import torch
import torch.nn as nn

from .... import native_ops as ops


class RNNDecoder(nn.Module):

    def __init__(self, input_size, rnn_type, num_units, num_layers, dropout, residual=False,
                 dense_residual=False):
        super(RNNDecoder, self).__init__()
        if rnn_type not in ('lstm', 'gru'):
            raise ValueError('rnn_type must be "lstm" or "gru".')
        self.input_size = input_size
        self.rnn_type = rnn_type
        self.num_units = num_units
        self.num_layers = num_layers
        self.dropout = dropout
        self.residual = residual
        self.dense_residual = dense_residual
        cell = nn.LSTMCell if rnn_type == 'lstm' else nn.GRUCell
        for l in range(num_layers):
            din = input_size if l == 0 else num_units
            setattr(self, '%s_l%d' % (rnn_type, l), cell(input_size=din, hidden_size=num_units,
                                                         bias=True))
            setattr(self, 'dropout_l' + str(l), nn.Dropout(p=dropout))

    def forward(self, dec_in, dec_state):
        """rnn_decoder.py:63-113.  dec_in [B, 1, input_size]; dec_state =
        (hx_list, cx_list), lists of [B, num_units] per layer (updated in place
        like the reference).  Returns (dec_out [B, 1, num_units], dec_state)."""
        gru = self.rnn_type == 'gru'
        if gru:                                  # dec_state = hx_list (rnn_decoder.py:77-78)
            hx_list, cx_list = dec_state, None
            if torch.is_tensor(hx_list):
                hx_list = [hx_list]
        else:
            hx_list, cx_list = dec_state
            if torch.is_tensor(hx_list):
                hx_list, cx_list = [hx_list], [cx_list]
        x = dec_in.squeeze(1)
        for l in range(self.num_layers):
            cell = getattr(self, '%s_l%d' % (self.rnn_type, l))
            inp = x if l == 0 else hx_list[l - 1]
            if gru:
                hx_list[l] = ops.gru_cell(inp, hx_list[l], cell.weight_ih, cell.weight_hh,
                                          cell.bias_ih, cell.bias_hh)
            else:
                hx_list[l], cx_list[l] = ops.lstm_cell(inp, hx_list[l], cx_list[l],
                                                       cell.weight_ih, cell.weight_hh,
                                                       cell.bias_ih, cell.bias_hh)
            if self.training and self.dropout > 0:
                hx_list[l] = ops.dropout(hx_list[l], self.dropout)
            if l > 0 and self.residual or self.dense_residual:     # rnn_decoder.py:100-104
                if self.residual:
                    # the reference's ``hx_list[l] += sum(hx_list[l - 1])``: Python's
                    # sum over the lower layer's output runs over the batch rows
                    hx_list[l] = ops.add_batch_sum(hx_list[l], hx_list[l - 1])
                elif self.dense_residual:
                    for lower in hx_list[:l]:
                        hx_list[l] = ops.add(hx_list[l], lower)
        return hx_list[-1].unsqueeze(1), (hx_list if gru else (hx_list, cx_list))
