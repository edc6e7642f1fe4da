"""RNNDecoder (reference models/pytorch_v3/attention/rnn_decoder.py).

Parameter holder with the reference's names (``lstm_l{l}.weight_ih`` ...);
the LSTMCell step is fused into the HIP decoder loop (csrc/decoder.hip
cell_fwd / cell_bwd).
"""
import torch.nn as nn


class RNNDecoder(nn.Module):

    def __init__(self, input_size, rnn_type, num_units, num_layers, dropout, residual=False,
                 dense_residual=False):
        super(RNNDecoder, self).__init__()
        if rnn_type != 'lstm' or num_layers != 1 or residual or dense_residual:
            raise NotImplementedError('MI355X fused decoder: 1-layer LSTM decoder')
        self.input_size = input_size
        self.rnn_type = rnn_type
        self.num_units = num_units
        self.num_layers = num_layers
        self.dropout = dropout
        self.residual = residual
        self.dense_residual = dense_residual
        for l in range(num_layers):
            din = input_size if l == 0 else num_units
            setattr(self, 'lstm_l' + str(l), nn.LSTMCell(input_size=din, hidden_size=num_units,
                                                         bias=True))
            setattr(self, 'dropout_l' + str(l), nn.Dropout(p=dropout))

    def forward(self, dec_in, dec_state):
        raise NotImplementedError('the decoder cell runs inside the fused decoder loop')
