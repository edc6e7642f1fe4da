"""CTC greedy (best path) decoder (reference greedy_decoder.py:19-47).

Device tensors go through the HIP best-path kernel (argmax with first-max
tie-breaking, collapse, blank removal on the GPU; only the compact hypotheses
cross PCIe).  numpy inputs (decode_from_probs) keep the reference's host
semantics.  Returns a list of int arrays (ragged; the reference's
``np.array(best_hyps)`` of ragged lists fails on numpy >= 1.24).
"""
import numpy as np
import torch

from ..... import native_ops as ops


class GreedyDecoder(object):

    def __init__(self, blank_index):
        self._blank = blank_index

    def __call__(self, logits, x_lens):
        if torch.is_tensor(logits) and logits.is_cuda:
            if not torch.is_tensor(x_lens):
                x_lens = torch.as_tensor(np.asarray(x_lens), dtype=torch.int32)
            lens = x_lens.to(logits.device).int()
            hyps, hl = ops.ctc_best_path(logits, lens, self._blank)
            hyps, hl = hyps.cpu().numpy(), hl.cpu().numpy()
            return [hyps[b, :hl[b]].astype(np.int64) for b in range(len(hl))]
        logits = np.asarray(logits)
        out = []
        for b in range(logits.shape[0]):
            idx = np.argmax(logits[b, :int(x_lens[b])], axis=-1)
            keep = np.ones(len(idx), bool)
            keep[1:] = idx[1:] != idx[:-1]
            col = idx[keep]
            out.append(col[col != self._blank].astype(np.int64))
        return out
