"""LinearND / Embedding / Embedding_LS (reference models/pytorch_v3/linear.py).

Same constructor signatures and parameter names (``fc.weight``, ``fc.bias``,
``embed.weight``, ``embed.fc.weight``); the math runs in the HIP GEMM /
embedding kernels of libasr_hip.so.
"""
import torch
import torch.nn as nn

from ... import native_ops as ops


class LinearND(nn.Module):
    """linear.py:15-47: affine map on the last dim of an N-D tensor + dropout."""

    def __init__(self, *size, bias=True, dropout=0):
        super(LinearND, self).__init__()
        self.fc = nn.Linear(*size, bias=bias)
        self.dropout_p = float(dropout)

    def forward(self, xs, input_drop=None):
        """input_drop=(p, seed): the caller's dropout of xs (same mask as
        ops.dropout(xs, p, seed)), folded into this layer's product."""
        ys = ops.linear(xs, self.fc.weight, self.fc.bias, drop=input_drop)
        if self.training and self.dropout_p > 0:
            ys = ops.dropout(ys, self.dropout_p)
        return ys


class Embedding(nn.Module):
    """linear.py:50-77.  nn.Embedding(padding_idx=-1): the LAST row (the
    <sos>/<eos> index) receives no gradient, as in the reference."""

    def __init__(self, num_classes, embedding_dim, dropout=0, ignore_index=-1):
        super(Embedding, self).__init__()
        self.embed = nn.Embedding(num_classes, embedding_dim, padding_idx=ignore_index)
        self.padding_idx = self.embed.padding_idx
        self.dropout_p = float(dropout)

    def forward(self, y, y_host=None):
        e = ops.embedding(y, self.embed.weight, self.padding_idx, idx_host=y_host)
        if self.training and self.dropout_p > 0:
            e = ops.dropout(e, self.dropout_p)
        return e


class Embedding_LS(nn.Module):
    """linear.py:80-116: one-hot(y) @ W^T with W = embed.fc.weight [emb, V].
    The reference's label-smoothing line edits ``y`` instead of the one-hot
    (linear.py:138-140), so it is a no-op: this is an un-smoothed lookup of the
    columns of W (no padding row)."""

    def __init__(self, num_classes, embedding_dim, dropout=0, label_smoothing_prob=0.):
        super(Embedding_LS, self).__init__()
        self.num_classes = num_classes
        self.label_smoothing_prob = label_smoothing_prob
        self.embed = LinearND(num_classes, embedding_dim, bias=False, dropout=dropout)

    def forward(self, y, y_host=None):
        e = ops.embedding_t(y, self.embed.fc.weight, idx_host=y_host)
        if self.training and self.embed.dropout_p > 0:
            e = ops.dropout(e, self.embed.dropout_p)
        return e
