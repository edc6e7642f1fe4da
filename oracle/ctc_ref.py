"""numpy float64 CTC forward-backward + best-path decoder (oracle; test infra only).

Restates, in log space, the algorithm of the reference's numpy CTC
(models/chainer/ctc/ctc_loss_from_chainer.py: softmax :32-35, blank-interleaved
path :38-42, 3-way transition with the same-symbol skip ban :181-232, forward /
flipped backward recursions :234-264, loss :266-286, gradient = softmax - label
occupancy masked beyond the input length :288-304) under the warp-ctc contract
the reference actually calls (models/pytorch_v3/ctc/ctc.py:30-66):

  * activations are UNNORMALISED; softmax is applied inside,
  * blank index 0,
  * per-utterance cost = -log P(y | x); the caller sums and divides by B,
  * gradient is w.r.t. the unnormalised activations and zero for t >= T_b,
  * infeasible alignments (L + repeats > T_b): cost 0, gradient 0
    (zero_infinity semantics; SURVEY.md §8c decision).
"""
import numpy as np

NEG = -np.inf


def _lse(*xs):
    m = np.max(np.stack(xs), axis=0)
    with np.errstate(invalid='ignore'):
        out = m + np.log(sum(np.exp(x - m) for x in xs))
    return np.where(np.isneginf(m), NEG, out)


def ctc_single(acts, labels, blank=0):
    """One utterance.  acts: [T, V] unnormalised; labels: [L] ints (no blank).

    Returns (cost, grad[T, V]) in float64.
    """
    acts = np.asarray(acts, np.float64)
    T, V = acts.shape
    L = len(labels)
    S = 2 * L + 1
    path = np.full(S, blank, np.int64)                 # ctc_loss_from_chainer.py:38-42
    path[1::2] = labels
    m = acts.max(axis=1, keepdims=True)               # log-softmax (softmax :32-35)
    logz = m + np.log(np.exp(acts - m).sum(axis=1, keepdims=True))
    logp = acts - logz
    emit = logp[:, path]                               # [T, S]

    # skip transition s-2 -> s allowed only between different symbols (:198-202)
    skip = np.zeros(S, bool)
    skip[2:] = path[2:] != path[:-2]

    alpha = np.full((T, S), NEG)
    alpha[0, 0] = emit[0, 0]
    if S > 1:
        alpha[0, 1] = emit[0, 1]
    for t in range(1, T):
        a = alpha[t - 1]
        a1 = np.concatenate([[NEG], a[:-1]])
        a2 = np.concatenate([[NEG, NEG], a[:-2]])[:S]     # [:S]: S = 1 (empty label)
        a2 = np.where(skip, a2, NEG)
        alpha[t] = _lse(a, a1, a2) + emit[t]

    beta = np.full((T, S), NEG)
    beta[T - 1, S - 1] = emit[T - 1, S - 1]
    if S > 1:
        beta[T - 1, S - 2] = emit[T - 1, S - 2]
    skip_fwd = np.zeros(S, bool)                       # s -> s+2 allowed
    skip_fwd[:-2] = path[:-2] != path[2:]
    for t in range(T - 2, -1, -1):
        b = beta[t + 1]
        b1 = np.concatenate([b[1:], [NEG]])
        b2 = np.concatenate([b[2:], [NEG, NEG]])[:S]
        b2 = np.where(skip_fwd, b2, NEG)
        beta[t] = _lse(b, b1, b2) + emit[t]

    logP = _lse(alpha[T - 1, S - 1], alpha[T - 1, S - 2]) if S > 1 else alpha[T - 1, 0]
    if not np.isfinite(logP):
        return 0.0, np.zeros((T, V))
    gamma = alpha + beta - emit                        # occupancy log (:288-304)
    occ = np.exp(gamma - logP)                         # [T, S]
    grad = np.exp(logp)
    for s in range(S):
        grad[:, path[s]] -= occ[:, s]
    return float(-logP), grad


def ctc_batch(acts, labels_flat, label_lens, act_lens, blank=0, time_major=True):
    """warp-ctc style batch call (ctc.py:35-45): acts [T,B,V] (or [B,T,V])."""
    acts = np.asarray(acts, np.float64)
    if not time_major:
        acts = acts.transpose(1, 0, 2)
    T, B, V = acts.shape
    costs = np.zeros(B)
    grads = np.zeros((T, B, V))
    off = 0
    for b in range(B):
        L = int(label_lens[b])
        lab = np.asarray(labels_flat[off:off + L], np.int64)
        off += L
        Tb = int(act_lens[b])
        c, g = ctc_single(acts[:Tb, b], lab, blank)
        costs[b] = c
        grads[:Tb, b] = g
    if not time_major:
        grads = grads.transpose(1, 0, 2)
    return costs, grads


def greedy_best_path(logits, x_lens, blank=0):
    """CTC best path (greedy_decoder.py:19-47): argmax (first max on ties),
    collapse repeats, drop blank.  Returns a list of int arrays (ragged)."""
    out = []
    for b in range(logits.shape[0]):
        idx = np.argmax(logits[b, :int(x_lens[b])], axis=-1)
        keep = np.ones(len(idx), bool)
        keep[1:] = idx[1:] != idx[:-1]
        col = idx[keep]
        out.append(col[col != blank].astype(np.int64))
    return out
