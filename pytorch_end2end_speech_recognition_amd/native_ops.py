"""autograd wrappers over the C ABI (libasr_hip.so).

Each Function launches hand-written gfx950 kernels on torch's current stream
through ctypes; torch supplies only device memory, the stream and the autograd
tape.  No op here has a CPU path: CPU tensors raise NativeError.

Weight gradients are accumulated by the kernels directly into ``param.grad``
(views into the model's flat gradient buffer, see models/pytorch_v3/base.py);
the Functions therefore return ``None`` for weights.
"""
import ctypes

import torch

from . import _native as N

F32 = N.ASR_DT_F32
BF16 = N.ASR_DT_BF16

_compute = {'dtype': F32}


def set_compute_dtype(name):
    """'fp32' (exact-f32 MFMA, parity mode) or 'bf16' (bf16 MFMA, f32 accumulate)."""
    if name not in ('fp32', 'bf16'):
        raise ValueError('compute dtype must be fp32 or bf16')
    _compute['dtype'] = BF16 if name == 'bf16' else F32


def compute_dtype():
    return _compute['dtype']


def _ws(nbytes, device):
    return torch.empty(max(int(nbytes), 1), dtype=torch.uint8, device=device)


def grad_buffer(p):
    """The gradient view a kernel accumulates into (allocated on first use)."""
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


# ---------------------------------------------------------------------------
# GEMM plumbing
# ---------------------------------------------------------------------------
def rowmap(stride_t, stride_b=0, rows_per_b=0, t_mul=1, t_add=0, t_limit=0, perm=None):
    return N.RowMap(int(stride_b), int(stride_t), int(rows_per_b), int(t_mul), int(t_add),
                    int(t_limit), perm.data_ptr() if perm is not None else None)


def operand(t, trans, rmap, offset=0):
    dt = BF16 if t.dtype == torch.bfloat16 else F32
    return N.Operand(t.data_ptr() + offset * t.element_size(), dt, int(trans), rmap)


def gemm_problem(a, b, c, c_map, M, N_, K, alpha=1.0, beta=0.0, bias=None, bias2=None, c_offset=0):
    return N.Gemm(a, b, c.data_ptr() + 4 * c_offset, c_map,
                  bias.data_ptr() if bias is not None else None,
                  bias2.data_ptr() if bias2 is not None else None, int(M), int(N_), int(K),
                  float(alpha), float(beta))


def run_gemm(problems, device):
    arr = (N.Gemm * len(problems))(*problems)
    N.call('asr_gemm', ctypes.cast(arr, ctypes.c_void_p), len(problems), compute_dtype(),
           N.stream_handle(device))


def colsum_accumulate(g2d, out0, out1=None, alpha=1.0):
    M, Nn = g2d.shape
    nb = N.query('asr_colsum_workspace_bytes', M, Nn)
    ws = _ws(nb, g2d.device)
    N.call('asr_colsum_accumulate', N.ptr(g2d), g2d.stride(0), M, Nn, float(alpha), N.ptr(out0),
           N.ptr(out1), N.ptr(ws), nb, N.stream_handle(g2d.device))


# ---------------------------------------------------------------------------
# Linear (LinearND, linear.py:15-47): y = x W^T + b on the last dim
# ---------------------------------------------------------------------------
class LinearFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias):
        N.require_device(x, weight)
        x = x.contiguous()
        K = x.shape[-1]
        Nout = weight.shape[0]
        M = x.numel() // K
        y = torch.empty(*x.shape[:-1], Nout, dtype=torch.float32, device=x.device)
        if M > 0:
            p = gemm_problem(operand(x, 0, rowmap(K)), operand(weight, 0, rowmap(K)), y,
                             rowmap(Nout), M, Nout, K, bias=bias)
            run_gemm([p], x.device)
        ctx.save_for_backward(x, weight)
        ctx.bias = bias
        return y

    @staticmethod
    def backward(ctx, dy):
        x, weight = ctx.saved_tensors
        dy = dy.contiguous()
        K = x.shape[-1]
        Nout = weight.shape[0]
        M = x.numel() // K
        dx = None
        if M == 0:
            return torch.zeros_like(x), None, None
        probs = []
        if ctx.needs_input_grad[0]:
            dx = torch.empty_like(x)
            probs.append(gemm_problem(operand(dy, 0, rowmap(Nout)), operand(weight, 1, rowmap(K)),
                                      dx, rowmap(K), M, K, Nout))
        gw = grad_buffer(weight)
        probs.append(gemm_problem(operand(dy, 1, rowmap(Nout)), operand(x, 1, rowmap(K)), gw,
                                  rowmap(K), Nout, K, M, beta=1.0))
        run_gemm(probs, x.device)
        if ctx.bias is not None:
            colsum_accumulate(dy.view(M, Nout), grad_buffer(ctx.bias))
        return dx, None, None


def linear(x, weight, bias=None):
    return LinearFn.apply(x, weight, bias)


# ---------------------------------------------------------------------------
# One bidirectional LSTM layer (nn.LSTM bidirectional + pack/pad, rnn.py)
# ---------------------------------------------------------------------------
class BLSTMLayerFn(torch.autograd.Function):
    """x_src [B, T_src, Din] f32; the layer input row (b, t) is
    x_src[perm[b] if perm else b, t*t_mul + t_add].  Parameters are passed as
    (w_ih [8H, Din], w_hh [8H, H], b_ih [8H], b_hh [8H]) where each is the
    forward-direction tensor immediately followed in memory by the reverse one
    (the flat layout of models/pytorch_v3/base.py)."""

    @staticmethod
    def forward(ctx, x_src, lens, T, perm, t_mul, t_add, gbufs, w_ih, w_hh, b_ih, b_hh):
        N.require_device(x_src, lens, w_ih, w_hh, b_ih, b_hh)
        x_src = x_src.contiguous()
        B, T_src, Din = x_src.shape
        H = w_hh.shape[1]
        dev = x_src.device
        a_map = rowmap(Din, stride_b=T_src * Din, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
        gx = torch.empty(B, T, 8 * H, dtype=torch.float32, device=dev)
        p = gemm_problem(operand(x_src, 0, a_map), operand(w_ih, 0, rowmap(Din)), gx,
                         rowmap(8 * H), B * T, 8 * H, Din, bias=b_ih, bias2=b_hh)
        run_gemm([p], dev)
        y = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        cst = torch.empty(B, T, 2 * H, dtype=torch.float32, device=dev)
        cd = compute_dtype()
        nb = N.query('asr_lstm_workspace_bytes', B, H, cd, 0)
        ws = _ws(nb, dev)
        whh_r = w_hh.data_ptr() + 4 * H * H * 4
        N.call('asr_lstm_forward', N.ptr(gx), N.ptr(w_hh), ctypes.c_void_p(whh_r), F32, N.ptr(lens),
               B, T, H, cd, N.ptr(y), N.ptr(cst), N.ptr(ws), nb, N.stream_handle(dev))
        ctx.save_for_backward(x_src, lens, w_ih, w_hh, b_ih, b_hh, gx, cst, y)
        ctx.meta = (T, perm, t_mul, t_add, gbufs)
        return y

    @staticmethod
    def backward(ctx, dy):
        x_src, lens, w_ih, w_hh, b_ih, b_hh, act, cst, y = ctx.saved_tensors
        T, perm, t_mul, t_add, gbufs = ctx.meta
        B, T_src, Din = x_src.shape
        H = w_hh.shape[1]
        dev = x_src.device
        dy = dy.contiguous()
        cd = compute_dtype()
        nb = N.query('asr_lstm_workspace_bytes', B, H, cd, 1)
        ws = _ws(nb, dev)
        whh_r = w_hh.data_ptr() + 4 * H * H * 4
        # the saved activations become the gate gradients dG in place
        N.call('asr_lstm_backward', N.ptr(dy), N.ptr(w_hh), ctypes.c_void_p(whh_r), F32,
               N.ptr(lens), B, T, H, cd, N.ptr(act), N.ptr(cst), N.ptr(ws), nb,
               N.stream_handle(dev))
        dg = act
        BT = B * T
        a_map = rowmap(Din, stride_b=T_src * Din, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                       t_limit=T_src, perm=perm)
        if gbufs is None:
            gbufs = tuple(grad_buffer(p) for p in (w_ih, w_hh, b_ih, b_hh))
        g_ih, g_hh, g_bih, g_bhh = gbufs
        probs = [
            # dW_ih [8H, Din] += dG^T x   (both directions in one problem)
            gemm_problem(operand(dg, 1, rowmap(8 * H)), operand(x_src, 1, a_map), g_ih,
                         rowmap(Din), 8 * H, Din, BT, beta=1.0),
        ]
        run_gemm(probs, dev)
        # dW_hh[dir] += dG_dir^T h_prev_dir ; h_prev = y[b, t-1, :H] (fwd), y[b, t+1, H:] (rev)
        hp_f = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=-1, t_limit=T)
        hp_r = rowmap(2 * H, stride_b=T * 2 * H, rows_per_b=T, t_add=1, t_limit=T)
        probs = [
            gemm_problem(operand(dg, 1, rowmap(8 * H)), operand(y, 1, hp_f), g_hh, rowmap(H),
                         4 * H, H, BT, beta=1.0),
            gemm_problem(operand(dg, 1, rowmap(8 * H), offset=4 * H),
                         operand(y, 1, hp_r, offset=H), g_hh, rowmap(H), 4 * H, H, BT, beta=1.0,
                         c_offset=4 * H * H),
        ]
        run_gemm(probs, dev)
        colsum_accumulate(dg.view(BT, 8 * H), g_bih, g_bhh)
        dx = None
        if ctx.needs_input_grad[0]:
            # dX [BT, Din] = dG [BT, 8H] W_ih [8H, Din], scattered back through the input map
            if perm is None and t_mul == 1 and t_add == 0 and T == T_src:
                dx = torch.empty_like(x_src)
            else:
                dx = torch.zeros_like(x_src)
            c_map = rowmap(Din, stride_b=T_src * Din, rows_per_b=T, t_mul=t_mul, t_add=t_add,
                           t_limit=T_src, perm=perm)
            p = gemm_problem(operand(dg, 0, rowmap(8 * H)), operand(w_ih, 1, rowmap(Din)), dx,
                             c_map, BT, Din, 8 * H)
            run_gemm([p], dev)
        return dx, None, None, None, None, None, None, None, None, None, None


def blstm_layer(x_src, lens, T, w_ih, w_hh, b_ih, b_hh, perm=None, t_mul=1, t_add=0, gbufs=None):
    """gbufs: optional (g_w_ih, g_w_hh, g_b_ih, g_b_hh) gradient views to accumulate
    into; default: the tensors' own .grad."""
    return BLSTMLayerFn.apply(x_src, lens, T, perm, t_mul, t_add, gbufs, w_ih, w_hh, b_ih, b_hh)


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
