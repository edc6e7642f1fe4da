"""Label-smoothing cross entropy (reference models/pytorch_v3/criterion.py:51-80)
on the fused HIP softmax-xent kernel."""
from ... import native_ops as ops


def cross_entropy_label_smoothing(logits, y_lens, label_smoothing_prob, distribution='uniform',
                                  size_average=False):
    """sum_b sum_{t < y_lens[b]} sum_v -(ls/V) log_softmax(logits)[b,t,v]  (/B if
    size_average).  logits [B, T, V] device; y_lens int tensor [B] (device)."""
    if distribution != 'uniform':
        raise NotImplementedError
    B, T, V = logits.shape
    scale = label_smoothing_prob / (B if size_average else 1)
    # ls_scale * sum_rows -(1/V) sum_v (x - lse) == sum_rows sum_v -(ls/V) log p
    return ops.xent(logits, None, y_lens, T, ce_scale=0.0, ls_scale=scale)
