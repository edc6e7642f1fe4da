"""autograd wrappers over the C ABI (libasr_hip.so).

Each Function launches hand-written gfx950 kernels on torch's current stream
through ctypes; torch supplies only device memory, the stream and the autograd
tape.  No op here has a CPU path: CPU tensors raise NativeError.
"""
import torch

from . import _native as N


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


# ---------------------------------------------------------------------------
# CTC (warp-ctc replacement; models/pytorch_v3/ctc/ctc.py:30-66)
# ---------------------------------------------------------------------------
class CTCLossFn(torch.autograd.Function):
    """loss = loss_scale * sum_b CTC(logits_b, labels_b); logits [B, T, V] f32
    batch-major (no time-major transpose copy).  The gradient is produced in
    backward, already multiplied by grad_output * loss_scale, in one write."""

    @staticmethod
    def forward(ctx, logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale,
                blank=0, zero_infinity=True):
        N.require_device(logits, labels_flat, label_lens, act_lens)
        logits = logits.contiguous()
        B, T, V = logits.shape
        nbytes = N.query('asr_ctc_workspace_bytes', T, B, V, max_label_len)
        ws = _ws(nbytes, logits.device)
        costs = torch.empty(B, dtype=torch.float32, device=logits.device)
        loss = torch.empty(1, dtype=torch.float32, device=logits.device)
        N.call('asr_ctc_forward', N.ptr(logits), V, T * V, T, B, V, N.ptr(labels_flat),
               N.ptr(label_lens), N.ptr(act_lens), int(max_label_len), int(blank),
               int(bool(zero_infinity)), N.ptr(costs), N.ptr(loss), float(loss_scale), N.ptr(ws),
               nbytes, N.stream_handle(logits.device))
        ctx.save_for_backward(logits, labels_flat, label_lens, act_lens, ws)
        ctx.meta = (int(max_label_len), int(blank), float(loss_scale), nbytes)
        ctx.costs = costs
        ctx.mark_non_differentiable(costs)
        return loss, costs

    @staticmethod
    def backward(ctx, g_loss, g_costs):
        logits, labels_flat, label_lens, act_lens, ws = ctx.saved_tensors
        max_label_len, blank, loss_scale, nbytes = ctx.meta
        B, T, V = logits.shape
        grads = torch.empty_like(logits)
        g = g_loss.contiguous() if g_loss is not None else None
        N.call('asr_ctc_backward', N.ptr(logits), V, T * V, T, B, V, N.ptr(labels_flat),
               N.ptr(label_lens), N.ptr(act_lens), max_label_len, blank, N.ptr(g),
               loss_scale if g is not None else 0.0, N.ptr(grads), V, T * V, N.ptr(ws), nbytes,
               N.stream_handle(logits.device))
        return grads, None, None, None, None, None, None, None


def ctc_loss(logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale=1.0, blank=0,
             zero_infinity=True):
    """Returns (loss [1], costs [B])."""
    return CTCLossFn.apply(logits, labels_flat, label_lens, act_lens, max_label_len, loss_scale,
                           blank, zero_infinity)
