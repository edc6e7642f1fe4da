"""Encoder registry (reference models/pytorch_v3/encoders/load_encoder.py:15-35)."""
from .rnn import RNNEncoder

ENCODERS = {
    'lstm': RNNEncoder,
    'gru': RNNEncoder,
    'rnn': RNNEncoder,
}


def load(encoder_type):
    if encoder_type not in ENCODERS:
        raise TypeError('encoder_type should be one of [%s], you provided %s.' %
                        (', '.join(ENCODERS), encoder_type))
    return ENCODERS[encoder_type]
