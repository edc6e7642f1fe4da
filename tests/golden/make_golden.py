#!/usr/bin/env python
"""Generate the golden vectors under tests/golden/ from the REFERENCE itself.

Runs only in the build container (it imports /root/reference, which does not
exist on the GPU box).  The outputs are small .npz fixtures: inputs, the
reference's state_dict, and the reference's outputs / gradients.  Nothing from
the reference's source is stored -- only numbers.

The reference (torch-0.3 era code) needs a few harness-only shims to run on
torch 2.10 (SURVEY.md §8c "What makes the full hot path run here"):

  1. ``warpctc_pytorch`` is absent (external, unpinned SeanNaren/warp-ctc).  A
     stand-in module fills ``grads``/``costs`` exactly as warp-ctc's
     ``cpu_ctc`` contract says (softmax inside, blank 0, per-utterance costs,
     gradient w.r.t. the UNNORMALISED activations, zero for t >= act_len),
     computed with torch.nn.functional.ctc_loss in float64.  Infeasible
     alignments give cost 0 / grad 0 (zero_infinity), the documented choice.
     Its backward scales by grad_output (chain rule; SURVEY §8c decision).
  2. ``torch.nn.modules.loss._assert_no_grad`` is restored as a no-op.
  3. ``AttentionMechanism.forward`` and ``cross_entropy_label_smoothing`` index
     ``x_lens[b].data[0]``; 1-D length tensors are passed as ``[B, 1]``.
  4. ``compute_xe_loss`` returns a 0-dim tensor on torch 2.x; it is reshaped to
     ``[1]`` so ``loss += ctc_loss`` works (attention_seq2seq.py:547).

Usage (from the repo root, in the build container):
    python tests/golden/make_golden.py
"""
import json
import os
import sys
import types

import numpy as np
import torch
import torch.nn.functional as F

REF = '/root/reference'
OUT = os.path.dirname(os.path.abspath(__file__))


# --------------------------------------------------------------------------
# Shims (harness only; never shipped)
# --------------------------------------------------------------------------
def _install_shims():
    import torch.nn.modules.loss as L
    if not hasattr(L, '_assert_no_grad'):
        L._assert_no_grad = lambda v: None

    wc = types.ModuleType('warpctc_pytorch')

    class _CTC(torch.autograd.Function):
        @staticmethod
        def backward(ctx, grad_output):
            g = ctx.grads
            if hasattr(g, 'data'):
                g = g.data
            return g * grad_output.to(g.dtype).reshape(()), None, None, None, None

    def cpu_ctc(acts, grads, labels, label_lens, act_lens, minibatch, costs):
        a = acts.detach().double().clone().requires_grad_(True)
        with torch.enable_grad():
            lp = a.log_softmax(-1)
            c = F.ctc_loss(lp, labels.long(), act_lens.long(), label_lens.long(),
                           blank=0, reduction='none', zero_infinity=True)
            c.sum().backward()
        grads.copy_(a.grad.to(grads.dtype))
        costs.copy_(c.detach().to(costs.dtype))

    class CTCLoss(object):
        pass

    wc._CTC = _CTC
    wc.cpu_ctc = cpu_ctc
    wc.gpu_ctc = cpu_ctc
    wc.CTCLoss = CTCLoss
    sys.modules['warpctc_pytorch'] = wc

    sys.path.insert(0, REF)

    from models.pytorch_v3.attention import attention_layer as al
    orig_fwd = al.AttentionMechanism.forward

    def fwd(self, enc_out, enc_out_a, x_lens, dec_out, aw_step):
        if x_lens.dim() == 1:
            x_lens = x_lens.view(-1, 1)
        return orig_fwd(self, enc_out, enc_out_a, x_lens, dec_out, aw_step)
    al.AttentionMechanism.forward = fwd

    from models.pytorch_v3 import criterion as cr
    orig_ls = cr.cross_entropy_label_smoothing

    def ls(logits, y_lens, label_smoothing_prob, distribution='uniform',
           size_average=False):
        if y_lens.dim() == 1:
            y_lens = y_lens.view(-1, 1)
        return orig_ls(logits, y_lens, label_smoothing_prob, distribution, size_average)
    cr.cross_entropy_label_smoothing = ls

    from models.pytorch_v3.attention import attention_seq2seq as asq
    asq.cross_entropy_label_smoothing = ls
    from models.pytorch_v3.ctc import ctc as ctcmod
    ctcmod.cross_entropy_label_smoothing = ls
    orig_xe = asq.AttentionSeq2seq.compute_xe_loss

    def xe(self, *a, **k):
        return orig_xe(self, *a, **k).reshape(1)
    asq.AttentionSeq2seq.compute_xe_loss = xe


def _save(name, **arrays):
    path = os.path.join(OUT, name + '.npz')
    np.savez_compressed(path, **arrays)
    sz = os.path.getsize(path)
    print('wrote %s (%d bytes)' % (path, sz))


def _sd(model, prefix='sd/'):
    return {prefix + k: v.detach().cpu().numpy().copy() for k, v in model.state_dict().items()}


def _grads(model, prefix='grad/'):
    out = {}
    for k, p in model.named_parameters():
        g = p.grad
        out[prefix + k] = (np.zeros(p.shape, np.float32) if g is None
                           else g.detach().cpu().numpy().copy())
    return out


# --------------------------------------------------------------------------
# Case 1: CTC loss / gradient on raw activations (warp-ctc contract)
# --------------------------------------------------------------------------
def case_ctc():
    rng = np.random.RandomState(0)
    cases = []
    # (B, V, act_lens, label lists)
    # last utterance is infeasible (L + repeats = 5 > T = 3): cost 0, grad 0
    cases.append(('ctc_v6', 6, [30, 25, 20, 12, 3, 3],
                  [[1, 1, 2, 3], [4, 5, 5, 5, 1], [2], [1, 2, 1, 2, 1, 2, 1, 2], [3, 3],
                   [3, 3, 3]]))
    cases.append(('ctc_v29', 29, [50, 47, 40, 33],
                  [list(rng.randint(1, 29, 20)), list(rng.randint(1, 29, 15)),
                   [5, 5, 5, 5, 5, 5], list(rng.randint(1, 29, 12))]))
    cases.append(('ctc_v1000', 1000, [40, 37],
                  [list(rng.randint(1, 1000, 10)), list(rng.randint(1, 1000, 7))]))
    wc = sys.modules['warpctc_pytorch']
    for name, V, act_lens, labels in cases:
        B = len(act_lens)
        T = max(act_lens)
        acts = (rng.randn(T, B, V) * 2).astype(np.float32)
        lab_lens = np.array([len(l) for l in labels], np.int32)
        flat = np.concatenate([np.array(l, np.int32) for l in labels])
        grads = torch.zeros(T, B, V)
        costs = torch.zeros(B)
        wc.cpu_ctc(torch.from_numpy(acts), grads, torch.from_numpy(flat),
                   torch.from_numpy(lab_lens), torch.from_numpy(np.array(act_lens, np.int32)),
                   B, costs)
        _save(name, acts=acts, labels=flat, label_lens=lab_lens,
              act_lens=np.array(act_lens, np.int32), costs=costs.numpy(),
              grads=grads.numpy())


# --------------------------------------------------------------------------
# Case 2: BLSTM encoder (RNNEncoder) forward / backward
# --------------------------------------------------------------------------
def case_encoder():
    from models.pytorch_v3.encoders.rnn import RNNEncoder
    specs = [
        ('enc_fast', dict(input_size=7, rnn_type='lstm', bidirectional=True, num_units=5,
                          num_proj=0, num_layers=2, dropout_input=0, dropout_hidden=0,
                          subsample_list=[], subsample_type='drop', batch_first=True,
                          merge_bidirectional=False, pack_sequence=True)),
        ('enc_sub', dict(input_size=7, rnn_type='lstm', bidirectional=True, num_units=5,
                         num_proj=0, num_layers=3, dropout_input=0, dropout_hidden=0,
                         subsample_list=[False, True, False], subsample_type='drop',
                         batch_first=True, merge_bidirectional=False, pack_sequence=True)),
    ]
    for name, kw in specs:
        torch.manual_seed(1623)
        enc = RNNEncoder(**kw)
        for p in enc.parameters():
            torch.nn.init.uniform_(p, -0.3, 0.3)
        rng = np.random.RandomState(1)
        B, T = 4, 21
        x_lens = np.array([17, 21, 9, 13], np.int32)     # unsorted, distinct
        xs = rng.randn(B, T, kw['input_size']).astype(np.float32)
        for b in range(B):
            xs[b, x_lens[b]:] = 0
        xs_t = torch.from_numpy(xs).requires_grad_(True)
        out, out_lens, perm = enc(xs_t, torch.from_numpy(x_lens))
        R = torch.from_numpy(rng.randn(*out.shape).astype(np.float32))
        (out * R).sum().backward()
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, x_lens=x_lens,
              out=out.detach().numpy(), out_lens=out_lens.numpy().astype(np.int32),
              perm=perm.numpy().astype(np.int64), R=R.numpy(), dxs=xs_t.grad.numpy(),
              **_sd(enc), **_grads(enc))


# --------------------------------------------------------------------------
# Case 3: location-aware attention step forward / backward
# --------------------------------------------------------------------------
def case_attention_step():
    from models.pytorch_v3.attention.attention_layer import AttentionMechanism
    kw = dict(encoder_num_units=12, decoder_num_units=10, attention_type='location',
              attention_dim=8, sharpening_factor=2.0, sigmoid_smoothing=False,
              out_channels=3, kernel_size=7, num_heads=1)
    torch.manual_seed(1623)
    att = AttentionMechanism(**kw)
    for p in att.parameters():
        torch.nn.init.uniform_(p, -0.3, 0.3)
    rng = np.random.RandomState(2)
    B, T = 3, 15
    x_lens = np.array([15, 11, 15], np.int32)
    enc_out = torch.from_numpy(rng.randn(B, T, 12).astype(np.float32)).requires_grad_(True)
    enc_out_a = torch.from_numpy(rng.randn(B, T, 8, 1).astype(np.float32)).requires_grad_(True)
    dec_out = torch.from_numpy(rng.randn(B, 1, 10).astype(np.float32)).requires_grad_(True)
    aw = np.abs(rng.rand(B, T, 1)).astype(np.float32)
    aw /= aw.sum(1, keepdims=True)
    aw_t = torch.from_numpy(aw).requires_grad_(True)
    ctx, aw_out = att(enc_out, enc_out_a, torch.from_numpy(x_lens), dec_out, aw_t)
    Rc = torch.from_numpy(rng.randn(*ctx.shape).astype(np.float32))
    Ra = torch.from_numpy(rng.randn(*aw_out.shape).astype(np.float32))
    ((ctx * Rc).sum() + (aw_out * Ra).sum()).backward()
    _save('att_step', kwargs=np.array(json.dumps(kw)), x_lens=x_lens,
          enc_out=enc_out.detach().numpy(), enc_out_a=enc_out_a.detach().numpy(),
          dec_out=dec_out.detach().numpy(), aw_in=aw, ctx=ctx.detach().numpy(),
          aw_out=aw_out.detach().numpy(), Rc=Rc.numpy(), Ra=Ra.numpy(),
          d_enc_out=enc_out.grad.numpy(), d_enc_out_a=enc_out_a.grad.numpy(),
          d_dec_out=dec_out.grad.numpy(), d_aw_in=aw_t.grad.numpy(),
          **_sd(att), **_grads(att))


# --------------------------------------------------------------------------
# Case 4: whole CTC model: loss, grads, greedy best path
# --------------------------------------------------------------------------
def _batch(rng, B, T, F_, y_lens, num_classes, x_lens):
    xs = rng.randn(B, T, F_).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    L = max(y_lens)
    ys = np.full((B, L), -1, np.int32)
    for b in range(B):
        ys[b, :y_lens[b]] = rng.randint(0, num_classes, y_lens[b])
    return xs, ys


def _ctc_variant_specs():
    """Encoder variants of rnn.py:392-465: projection tanh(LinearND) between
    layers, 'concat' subsampling (successive frame pairs), residual and dense
    residual connections (from the last subsampling layer on)."""
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=3, fc_list=[],
                dropout_input=0, dropout_encoder=0, num_classes=5, parameter_init=0.1,
                subsample_list=[False, True, False], subsample_type='drop')
    return [
        ('model_ctc_proj', dict(base, encoder_num_proj=4)),
        ('model_ctc_concat', dict(base, subsample_list=[True, False, False],
                                  subsample_type='concat')),
        ('model_ctc_proj_concat', dict(base, encoder_num_proj=5, subsample_type='concat')),
        ('model_ctc_res', dict(base, encoder_num_layers=4,
                               subsample_list=[True, False, False, False],
                               encoder_residual=True)),
        ('model_ctc_dres', dict(base, encoder_num_layers=4, subsample_list=[],
                                encoder_dense_residual=True, encoder_num_proj=7)),
    ]


def _selected():
    """Case names given on the command line (default: every case)."""
    return set(a for a in sys.argv[1:] if not a.startswith('-'))


def case_ctc_model():
    from models.pytorch_v3.ctc.ctc import CTC
    from models.pytorch_v3.ctc.decoders.greedy_decoder import GreedyDecoder
    specs = [
        ('model_ctc_sub', dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                               encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=3,
                               fc_list=[], dropout_input=0, dropout_encoder=0, num_classes=5,
                               parameter_init=0.1, subsample_list=[False, True, False],
                               subsample_type='drop')),
        ('model_ctc_fast', dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2,
                                fc_list=[], dropout_input=0, dropout_encoder=0, num_classes=5,
                                parameter_init=0.1, subsample_list=[], subsample_type='drop')),
    ]
    specs += _ctc_variant_specs()
    # GRU encoders (rnn.py:173-191 fast nn.GRU, :226-233 per layer): fast path and
    # per-layer path with 'drop' subsampling
    specs += [
        ('model_ctc_gru_fast', dict(specs[1][1], encoder_type='gru')),
        ('model_ctc_gru_sub', dict(specs[0][1], encoder_type='gru')),
    ]
    only = _selected()
    for name, kw in specs:
        if only and name not in only:
            continue
        torch.manual_seed(1623)
        model = CTC(**kw)
        model.train()
        rng = np.random.RandomState(3)
        B, T = 4, 24
        x_lens = np.array([20, 24, 15, 11], np.int32)
        y_lens = np.array([5, 3, 4, 2], np.int32)
        xs, ys = _batch(rng, B, T, 8, y_lens, 5, x_lens)
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        # greedy decode: reference GreedyDecoder per utterance (ragged output)
        model.eval()
        with torch.no_grad():
            logits, out_lens, perm = model._encode(torch.from_numpy(xs),
                                                   torch.from_numpy(x_lens))
        dec = GreedyDecoder(blank_index=0)
        lg = logits.numpy()
        hyps = [dec(lg[b:b + 1], out_lens.numpy()[b:b + 1])[0] - 1 for b in range(B)]
        hyp_lens = np.array([len(h) for h in hyps], np.int32)
        hyp_flat = (np.concatenate(hyps).astype(np.int32) if hyp_lens.sum()
                    else np.zeros(0, np.int32))
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, loss=loss.detach().numpy().reshape(1), logits=lg,
              out_lens=out_lens.numpy().astype(np.int32), perm=perm.numpy().astype(np.int64),
              hyp_flat=hyp_flat, hyp_lens=hyp_lens, **_sd(model), **_grads(model))


# --------------------------------------------------------------------------
# Case 4b: VGG-BLSTM CTC (CNNEncoder front-end, models/pytorch_v3/encoders/cnn.py)
# --------------------------------------------------------------------------
def case_vgg_model():
    from models.pytorch_v3.ctc.ctc import CTC
    vgg = dict(input_size=16, encoder_type='lstm', encoder_bidirectional=True,
               encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2, fc_list=[],
               dropout_input=0, dropout_encoder=0, num_classes=5, parameter_init=0.1,
               subsample_list=[], subsample_type='drop', conv_channels=[4, 4, 16, 16],
               conv_kernel_sizes=[[3, 3]] * 4, conv_strides=[[1, 1]] * 4,
               poolings=[[], [2, 2], [], [2, 2]], activation='relu')
    specs = [('model_vgg_bn', dict(vgg, batch_norm=True)),
             ('model_vgg_nobn', dict(vgg, batch_norm=False, poolings=[[2, 2], [], [2, 2], []]))]
    for name, kw in specs:
        torch.manual_seed(1623)
        model = CTC(**kw)
        model.train()
        sd0 = _sd(model)                    # before the step (BN running stats move)
        rng = np.random.RandomState(5)
        B, T = 3, 23                        # odd T: the ceil-mode pool keeps a partial window
        x_lens = np.array([23, 17, 12], np.int32)
        y_lens = np.array([3, 2, 2], np.int32)
        xs, ys = _batch(rng, B, T, 16, y_lens, 5, x_lens)
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        after = {'after/' + k: v.detach().numpy().copy() for k, v in model.state_dict().items()
                 if 'running' in k}     # one training forward's running-stat update
        enc = model.encoder
        enc.conv.eval()                 # (eval: no second running-stat update)
        with torch.no_grad():
            conv_out, conv_lens = enc.conv(torch.from_numpy(xs), torch.from_numpy(x_lens))
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, loss=loss.detach().numpy().reshape(1),
              conv_lens=conv_lens.numpy().astype(np.int32), conv_T=np.int32(conv_out.shape[1]),
              **sd0, **after, **_grads(model))


# --------------------------------------------------------------------------
# Case 4c: hierarchical CTC (word CTC on top, char CTC on layer num_layers_sub)
# --------------------------------------------------------------------------
def case_hier_ctc_model():
    from models.pytorch_v3.ctc.hierarchical_ctc import HierarchicalCTC
    base = dict(input_size=16, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=3,
                encoder_num_layers_sub=2, fc_list=[], fc_list_sub=[], dropout_input=0,
                dropout_encoder=0, main_loss_weight=0.5, sub_loss_weight=0.5, num_classes=9,
                num_classes_sub=5, parameter_init=0.1, subsample_list=[], subsample_type='drop')
    specs = [('model_hier', base),
             ('model_hier_vgg', dict(base, main_loss_weight=0.7, sub_loss_weight=0.3,
                                     conv_channels=[4, 4, 16, 16],
                                     conv_kernel_sizes=[[3, 3]] * 4, conv_strides=[[1, 1]] * 4,
                                     poolings=[[], [2, 2], [], [2, 2]], batch_norm=True,
                                     activation='relu'))]
    for name, kw in specs:
        torch.manual_seed(1623)
        model = HierarchicalCTC(**kw)
        model.train()
        sd0 = _sd(model)
        rng = np.random.RandomState(6)
        B, T = 3, 26
        x_lens = np.array([26, 21, 13], np.int32)
        y_lens = np.array([2, 3, 1], np.int32)
        y_lens_sub = np.array([5, 4, 3], np.int32)
        xs, ys = _batch(rng, B, T, 16, y_lens, 9, x_lens)
        ys_sub = np.full((B, 5), -1, np.int32)
        for b in range(B):
            ys_sub[b, :y_lens_sub[b]] = rng.randint(0, 5, y_lens_sub[b])
        loss, loss_main, loss_sub = model(xs, ys, x_lens, y_lens, ys_sub, y_lens_sub)
        loss.backward()
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, ys_sub=ys_sub, y_lens_sub=y_lens_sub,
              loss=loss.detach().numpy().reshape(1),
              loss_main=loss_main.detach().numpy().reshape(1),
              loss_sub=loss_sub.detach().numpy().reshape(1), **sd0, **_grads(model))


# --------------------------------------------------------------------------
# Case 5: attention enc-dec (location, bahdanau) with / without auxiliary CTC
# --------------------------------------------------------------------------
def case_attention_model():
    from models.pytorch_v3.attention.attention_seq2seq import AttentionSeq2seq
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2,
                attention_type='location', attention_dim=7, decoder_type='lstm',
                decoder_num_units=9, decoder_num_layers=1, embedding_dim=4,
                dropout_input=0, dropout_encoder=0, dropout_decoder=0, dropout_embedding=0,
                num_classes=5, parameter_init=0.1, subsample_list=[False, True],
                subsample_type='drop', attention_conv_num_channels=3,
                attention_conv_width=5, bottleneck_dim=11, decoding_order='bahdanau')
    specs = [
        ('model_att', dict(base, init_dec_state='zero', ctc_loss_weight=0,
                           label_smoothing_prob=0)),
        ('model_att_hybrid', dict(base, init_dec_state='first', ctc_loss_weight=0.3,
                                  label_smoothing_prob=0, sharpening_factor=1.5)),
        ('model_att_ls', dict(base, init_dec_state='zero', ctc_loss_weight=0.3,
                              label_smoothing_prob=0.1)),
        ('model_att_mean', dict(base, init_dec_state='mean', ctc_loss_weight=0,
                                label_smoothing_prob=0)),
        # decoder / attention variants (attention_seq2seq.py:280-361, 704-799,
        # attention_layer.py:66-72, 145-153)
        ('model_att_content', dict(base, attention_type='content', init_dec_state='zero')),
        ('model_att_bwd', dict(base, init_dec_state='first', backward_loss_weight=0.4)),
        ('model_att_bwd_only', dict(base, init_dec_state='final', backward_loss_weight=1.0)),
        ('model_att_dec2', dict(base, init_dec_state='first', decoder_num_layers=2,
                                decoder_residual=True)),
        ('model_att_dec3_dres', dict(base, init_dec_state='zero', decoder_num_layers=3,
                                     decoder_dense_residual=True)),
        ('model_att_luong', dict(base, init_dec_state='zero', decoding_order='luong')),
        ('model_att_cond', dict(base, init_dec_state='first', decoding_order='conditional')),
        ('model_att_bridge', dict(base, init_dec_state='first', bridge_layer=True,
                                  ctc_loss_weight=0.2)),
        ('model_att_gru_enc', dict(base, encoder_type='gru', init_dec_state='first')),
        # TIMIT bgru_att_phone61 shape family: GRU encoder + bridge + GRU decoder
        ('model_att_gru', dict(base, encoder_type='gru', decoder_type='gru', bridge_layer=True,
                               init_dec_state='first')),
        ('model_att_gru_dec2', dict(base, decoder_type='gru', decoder_num_layers=2,
                                    init_dec_state='first', decoding_order='luong')),
    ]
    only = _selected()
    for name, kw in specs:
        if only and name not in only:
            continue
        torch.manual_seed(1623)
        model = AttentionSeq2seq(**kw)
        model.train()
        rng = np.random.RandomState(4)
        B, T = 3, 22
        x_lens = np.array([22, 19, 14], np.int32)
        y_lens = np.array([4, 6, 3], np.int32)
        xs, ys = _batch(rng, B, T, 8, y_lens, 5, x_lens)
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, loss=loss.detach().numpy().reshape(1),
              **_sd(model), **_grads(model))


# --------------------------------------------------------------------------
# Case 6b: hierarchical attention (word decoder on top, char decoder + CTC on
# layer encoder_num_layers_sub)
# --------------------------------------------------------------------------
def case_hier_attention_model():
    from models.pytorch_v3.attention.hierarchical_attention_seq2seq import \
        HierarchicalAttentionSeq2seq
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=3,
                encoder_num_layers_sub=2, attention_type='location', attention_dim=7,
                decoder_type='lstm', decoder_num_units=9, decoder_num_units_sub=7,
                decoder_num_layers=1, decoder_num_layers_sub=1, embedding_dim=4,
                embedding_dim_sub=3, dropout_input=0, dropout_encoder=0, dropout_decoder=0,
                dropout_embedding=0, num_classes=5, num_classes_sub=4, parameter_init=0.1,
                subsample_list=[False, True, False], subsample_type='drop',
                attention_conv_num_channels=3, attention_conv_width=5, bottleneck_dim=11,
                bottleneck_dim_sub=8, decoding_order='bahdanau')
    specs = [
        ('model_hatt', dict(base, init_dec_state='zero', main_loss_weight=0.5,
                            sub_loss_weight=0.5, ctc_loss_weight_sub=0)),
        ('model_hatt_ctc', dict(base, init_dec_state='first', sharpening_factor=1.5,
                                main_loss_weight=0.6, sub_loss_weight=0.2,
                                ctc_loss_weight_sub=0.3, label_smoothing_prob=0.1)),
    ]
    only = _selected()
    for name, kw in specs:
        if only and name not in only:
            continue
        torch.manual_seed(1623)
        model = HierarchicalAttentionSeq2seq(**kw)
        model.train()
        rng = np.random.RandomState(8)
        B, T = 3, 22
        x_lens = np.array([22, 19, 14], np.int32)
        y_lens = np.array([3, 4, 2], np.int32)
        y_lens_sub = np.array([6, 7, 4], np.int32)
        xs, ys = _batch(rng, B, T, 8, y_lens, 5, x_lens)
        ys_sub = np.full((B, int(y_lens_sub.max())), -1, np.int32)
        for b in range(B):
            ys_sub[b, :y_lens_sub[b]] = rng.randint(0, 4, y_lens_sub[b])
        loss, loss_main, loss_sub = model(xs, ys, x_lens, y_lens, ys_sub, y_lens_sub)
        loss.backward()
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, ys_sub=ys_sub, y_lens_sub=y_lens_sub,
              loss=loss.detach().numpy().reshape(1),
              loss_main=loss_main.detach().numpy().reshape(1),
              loss_sub=loss_sub.detach().numpy().reshape(1), **_sd(model), **_grads(model))


# --------------------------------------------------------------------------
# Case 5b: attention at the PRODUCTION attention shape (BASELINE configs[2]/[3],
# examples/librispeech/s5/conf/attention/char_blstm_att_100h.yml): location
# attention 128-dim, 10 conv channels x width 201, LSTM decoder 320, embedding
# 32, bottleneck 320, encoder 320 x 2 directions (E = 640), V = 28 + 2; T' =
# 161 frames (six 32-frame chunks of the attention kernels), ragged lengths.
# One encoder layer keeps the fixture small.  Weights are NOT stored (the
# model classes reproduce the reference's initial state_dict bit for bit under
# the same seed; per-tensor sums pin that); gradients of tensors above 64k
# values are stored as (first 2 rows, Frobenius norm, projection on a seeded
# N(0,1) tensor: np.random.RandomState(crc of the name)).
# --------------------------------------------------------------------------
PROD_ATT = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=320, encoder_num_proj=0, encoder_num_layers=1,
                attention_type='location', attention_dim=128, decoder_type='lstm',
                decoder_num_units=320, decoder_num_layers=1, embedding_dim=32,
                dropout_input=0, dropout_encoder=0, dropout_decoder=0, dropout_embedding=0,
                num_classes=28, parameter_init=0.1, subsample_list=[], subsample_type='drop',
                attention_conv_num_channels=10, attention_conv_width=201, bottleneck_dim=320,
                decoding_order='bahdanau', init_dec_state='zero')


def grad_digest(name, g, big=65536):
    """Compact gradient record (shared with tests/test_attention_prod.py)."""
    import zlib
    g = np.asarray(g, np.float32)
    if g.size <= big:
        return {'grad/' + name: g}
    r = np.random.RandomState(zlib.crc32(name.encode()) & 0x7fffffff).randn(*g.shape)
    return {'grad_rows/' + name: g.reshape(g.shape[0], -1)[:2].copy(),
            'grad_norm/' + name: np.array([np.linalg.norm(g.astype(np.float64))]),
            'grad_proj/' + name: np.array([np.sum(g.astype(np.float64) * r)])}


def case_attention_prod():
    from models.pytorch_v3.attention.attention_seq2seq import AttentionSeq2seq
    specs = [('model_att_prod', dict(PROD_ATT, ctc_loss_weight=0, label_smoothing_prob=0)),
             ('model_att_prod_hybrid', dict(PROD_ATT, ctc_loss_weight=0.3,
                                            label_smoothing_prob=0.1))]
    only = _selected()
    for name, kw in specs:
        if only and name not in only:
            continue
        torch.manual_seed(1623)
        model = AttentionSeq2seq(**kw)
        model.train()
        sums = {'sdsum/' + k: np.array([v.double().sum().item(), (v.double() ** 2).sum().item()])
                for k, v in model.state_dict().items()}
        rng = np.random.RandomState(11)
        B, T = 3, 161
        x_lens = np.array([161, 140, 97], np.int32)
        y_lens = np.array([23, 31, 17], np.int32)
        xs, ys = _batch(rng, B, T, 8, y_lens, 28, x_lens)
        loss = model(xs, ys, x_lens, y_lens)
        loss.backward()
        grads = {}
        for k, p in model.named_parameters():
            grads.update(grad_digest(k, np.zeros(p.shape, np.float32) if p.grad is None
                                     else p.grad.detach().numpy()))
        _save(name, kwargs=np.array(json.dumps(kw)), xs=xs, ys=ys, x_lens=x_lens,
              y_lens=y_lens, loss=loss.detach().numpy().reshape(1), **sums, **grads)


# --------------------------------------------------------------------------
# Case 8: the data path -- DatasetBase.sample_index / next / make_batch
# (utils/dataset/loader.py:29-157, base.py:76-201) with the LibriSpeech
# Dataset's filtering, sort and dynamic batching (load_dataset.py:104-142),
# and the frame stacking / splicing helpers.  The reference object is built
# with the attributes the corpus Dataset's __init__ sets (its label-file and
# CSV plumbing is corpus preparation, out of scope).
# --------------------------------------------------------------------------
def case_loader():
    import tempfile
    import pandas as pd
    from utils.dataset.loader import DatasetBase
    from utils.io.inputs.frame_stacking import stack_frame
    from utils.io.inputs.splicing import do_splice
    sys.path.insert(0, os.path.join(REF, 'examples', 'librispeech', 's5'))
    from exp.dataset.load_dataset import Dataset as LibriDataset

    rng = np.random.RandomState(12)
    n = 19
    frames = rng.randint(20, 1900, n)
    frames[3] = 35                                 # filtered (< min_frame_num 40)
    tmp = tempfile.mkdtemp()
    feats, trans = {}, []
    for i in range(n):
        # the features are at most 20 frames (the CSV's frame_num drives the
        # sort, the dynamic batch size and the padding) so the fixture stays small
        T = int(min(frames[i], 20))
        x = rng.randn(T, 3 * 41).astype(np.float32)                     # static | d | dd
        path = os.path.join(tmp, 'utt%03d.npy' % i)
        np.save(path, x)
        feats['feat/utt%03d' % i] = x
        trans.append(' '.join(str(v) for v in rng.randint(0, 29, rng.randint(1, 9))))
    df = pd.DataFrame({'frame_num': frames, 'input_path': [os.path.join(tmp, 'utt%03d.npy' % i)
                                                           for i in range(n)],
                       'transcript': trans})
    vocab = os.path.join(tmp, 'vocab.txt')
    open(vocab, 'w').write('\n'.join('c%d' % i for i in range(29)) + '\n')

    def make(batch_size, sort_utt, reverse, dynamic, input_freq, use_delta, use_dd,
             num_stack, num_skip, splice):
        ds = DatasetBase(vocab_file_path=vocab)
        d = df[df['frame_num'] >= 40]
        d = d.sort_values(by='frame_num', ascending=not reverse) if sort_utt else \
            d.sort_values(by='input_path', ascending=True)
        ds.df, ds.rest = d, set(list(d.index))
        ds.backend, ds.is_test, ds.batch_size, ds.max_epoch = 'pytorch', False, batch_size, 2
        ds.input_freq, ds.use_delta, ds.use_double_delta = input_freq, use_delta, use_dd
        ds.num_stack, ds.num_skip, ds.splice = num_stack, num_skip, splice
        ds.shuffle, ds.sort_utt, ds.sort_stop_epoch = False, sort_utt, None
        ds.num_enque, ds.dynamic_batching = None, dynamic
        ds.select_batch_size = types.MethodType(LibriDataset.select_batch_size, ds)
        return ds

    specs = {'a': (6, True, False, True, 41, True, True, 1, 1, 1),
             'b': (5, True, True, False, 40, False, False, 3, 2, 1),
             'c': (4, False, False, False, 41, True, True, 1, 1, 3)}
    out = {'df_frame_num': frames, 'df_transcript': np.array(trans)}
    out.update(feats)
    for tag, spec in specs.items():
        ds = make(*spec)
        out['spec/' + tag] = np.array(spec[:4] + spec[4:], dtype=np.int64)
        k = 0
        while True:
            try:
                batch, new_epoch = ds.next()
            except StopIteration:
                break
            names = [int(s_[3:]) for s_ in batch['input_names']]
            out['%s/%d/utts' % (tag, k)] = np.array(names, np.int64)
            out['%s/%d/new_epoch' % (tag, k)] = np.array([int(new_epoch)])
            for key in ('xs', 'ys', 'x_lens', 'y_lens'):
                out['%s/%d/%s' % (tag, k, key)] = np.asarray(batch[key])
            k += 1
        out['%s/n_batches' % tag] = np.array([k])
    x = rng.randn(37, 3 * 4 * 2).astype(np.float32)
    out['stack_in'] = x
    for st, sk in ((2, 1), (3, 2), (4, 3), (3, 3)):
        out['stack/%d_%d' % (st, sk)] = stack_frame(x, st, sk)
    for sp, ns in ((3, 1), (5, 2), (11, 1)):
        out['splice/%d_%d' % (sp, ns)] = do_splice(x[:, :12 * ns], sp, ns)
    _save('loader', **out)


# --------------------------------------------------------------------------
# Case 7: greedy attention decoding (attention_seq2seq.py:866-1036)
# --------------------------------------------------------------------------
def case_attention_decode():
    """AttentionSeq2seq.decode(beam_width=1) on random-init models (uniform
    +-1.5).  The init seed is the first of 1623, 1624, ... whose decode is not
    constant (at least three distinct tokens); in the 'eos' case it is the
    first whose all-<eos> early exit fires after more than one step."""
    from models.pytorch_v3.attention.attention_seq2seq import AttentionSeq2seq
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2,
                attention_type='location', attention_dim=7, decoder_type='lstm',
                decoder_num_units=9, decoder_num_layers=1, embedding_dim=4,
                dropout_input=0, dropout_encoder=0, dropout_decoder=0, dropout_embedding=0,
                num_classes=5, parameter_init=0.1, subsample_list=[False, True],
                subsample_type='drop', attention_conv_num_channels=3,
                attention_conv_width=5, bottleneck_dim=11, decoding_order='bahdanau',
                ctc_loss_weight=0, label_smoothing_prob=0)
    specs = [
        ('dec_att', dict(base, init_dec_state='zero'), False),
        ('dec_att_first', dict(base, init_dec_state='first', sharpening_factor=1.5), False),
        ('dec_att_eos', dict(base, init_dec_state='zero', num_classes=3), True),
    ]
    only = _selected()
    max_len = 12
    rng0 = np.random.RandomState(6)
    B, T = 4, 22
    x_lens = np.array([22, 17, 20, 11], np.int32)
    xs = rng0.randn(B, T, 8).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    for name, kw, want_exit in specs:
        if only and name not in only:
            continue
        for seed in range(1623, 1623 + 500):
            torch.manual_seed(seed)
            model = AttentionSeq2seq(**kw)
            for p in model.parameters():
                torch.nn.init.uniform_(p, -1.5, 1.5)
            hyps, aw, perm = model.decode(xs, x_lens, beam_width=1, max_decode_len=max_len)
            hyps = np.asarray(hyps)
            ok = (1 < hyps.shape[1] < max_len) if want_exit else len(np.unique(hyps)) >= 3
            if ok:
                break
        else:
            raise RuntimeError('no seed found for ' + name)
        _save(name, kwargs=np.array(json.dumps(kw)), seed=np.array([seed]), xs=xs,
              x_lens=x_lens, max_decode_len=np.array([max_len]),
              best_hyps=hyps.astype(np.int64), aw=np.asarray(aw, np.float32),
              perm=np.asarray(perm).astype(np.int64), **_sd(model))


def _install_beam_shims():
    """Harness-only shims for AttentionSeq2seq._decode_infer_beam (torch-0.3 /
    numpy < 1.24 era code on torch 2.10 / numpy 2.2):
      5. ``.data[0]`` on a 0-dim tensor (a scalar Variable's value in torch 0.3,
         attention_seq2seq.py:1072,1138) returns the tensor itself;
      6. ``np.array`` of ragged hypothesis lists returns an object array (numpy
         < 1.24 behaviour, attention_seq2seq.py:1235) instead of raising."""
    base_getitem = torch.Tensor.__getitem__

    def getitem(self, idx):
        if self.dim() == 0 and isinstance(idx, int) and idx == 0:
            return self
        return base_getitem(self, idx)
    torch.Tensor.__getitem__ = getitem

    from models.pytorch_v3.attention import attention_seq2seq as asq

    class _NP(types.ModuleType):
        def __getattr__(self, k):
            return getattr(np, k)

    npx = _NP('numpy_ragged')

    def array(obj, *a, **k):
        try:
            return np.array(obj, *a, **k)
        except ValueError:
            out = np.empty(len(obj), dtype=object)
            for i, o in enumerate(obj):
                out[i] = o
            return out
    npx.array = array
    asq.np = npx


def case_attention_beam():
    """AttentionSeq2seq.decode(beam_width > 1) (attention_seq2seq.py:1038-1237)
    on random-init models (uniform +-init): the seed is the first of 1623, ...
    whose beam output has at least three distinct tokens and hypotheses of
    different lengths (some complete with <eos> before max_decode_len)."""
    from models.pytorch_v3.attention.attention_seq2seq import AttentionSeq2seq
    _install_beam_shims()
    only = _selected()
    rng0 = np.random.RandomState(6)
    B, T = 4, 22
    x_lens = np.array([22, 17, 20, 11], np.int32)
    xs = rng0.randn(B, T, 8).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2,
                attention_type='location', attention_dim=7, decoder_type='lstm',
                decoder_num_units=9, decoder_num_layers=1, embedding_dim=4,
                dropout_input=0, dropout_encoder=0, dropout_decoder=0, dropout_embedding=0,
                num_classes=6, parameter_init=0.1, subsample_list=[False, True],
                subsample_type='drop', attention_conv_num_channels=3,
                attention_conv_width=5, bottleneck_dim=11, decoding_order='bahdanau',
                ctc_loss_weight=0, label_smoothing_prob=0, init_dec_state='zero')
    specs = [('beam_att', base, 0.6, dict(beam_width=3, max_decode_len=12)),
             ('beam_att_first', dict(base, init_dec_state='first', sharpening_factor=1.5), 0.6,
              dict(beam_width=4, max_decode_len=10, min_decode_len=3, length_penalty=0.1)),
             ('beam_att_wide', dict(base, num_classes=9), 0.8,
              dict(beam_width=5, max_decode_len=14, length_penalty=-0.05))]
    for name, kw, scale, opts in specs:
        if only and name not in only:
            continue
        for seed in range(1623, 1623 + 500):
            torch.manual_seed(seed)
            model = AttentionSeq2seq(**kw)
            for p in model.parameters():
                torch.nn.init.uniform_(p, -scale, scale)
            with torch.no_grad():   # torch-0.3 volatile decoding (deepcopy of non-leaf states)
                hyps, aw, perm = model.decode(xs, x_lens, **opts)
            hl = np.array([len(h) for h in hyps], np.int32)
            toks = np.concatenate([np.asarray(h, np.int64) for h in hyps])
            if len(np.unique(toks)) >= 3 and len(np.unique(hl)) >= 2:
                break
        else:
            raise RuntimeError('no seed found for ' + name)
        _save(name, kwargs=np.array(json.dumps(kw)), opts=np.array(json.dumps(opts)),
              seed=np.array([seed]), xs=xs, x_lens=x_lens, hyp_flat=toks, hyp_lens=hl,
              aw_flat=np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in aw]),
              perm=np.asarray(perm).astype(np.int64), **_sd(model))


def case_hier_attention_beam():
    """HierarchicalAttentionSeq2seq.decode(beam_width=3) for the word task
    (task_index 0, top layer) and the character task (task_index 1, layer
    encoder_num_layers_sub), random-init model as in case_attention_beam."""
    from models.pytorch_v3.attention.hierarchical_attention_seq2seq import \
        HierarchicalAttentionSeq2seq
    _install_beam_shims()
    if _selected() and 'beam_hatt' not in _selected():
        return
    kw = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
              encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=3,
              encoder_num_layers_sub=2, attention_type='location', attention_dim=7,
              decoder_type='lstm', decoder_num_units=9, decoder_num_units_sub=7,
              decoder_num_layers=1, decoder_num_layers_sub=1, embedding_dim=4,
              embedding_dim_sub=3, dropout_input=0, dropout_encoder=0, dropout_decoder=0,
              dropout_embedding=0, num_classes=7, num_classes_sub=6, parameter_init=0.1,
              subsample_list=[False, True, False], subsample_type='drop',
              attention_conv_num_channels=3, attention_conv_width=5, bottleneck_dim=11,
              bottleneck_dim_sub=8, decoding_order='bahdanau', init_dec_state='zero',
              main_loss_weight=0.5, sub_loss_weight=0.5, ctc_loss_weight_sub=0)
    rng0 = np.random.RandomState(9)
    B, T = 3, 22
    x_lens = np.array([22, 19, 14], np.int32)
    xs = rng0.randn(B, T, 8).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    opts = dict(beam_width=3, max_decode_len=10)
    for seed in range(1623, 1623 + 500):
        torch.manual_seed(seed)
        model = HierarchicalAttentionSeq2seq(**kw)
        for p in model.parameters():
            torch.nn.init.uniform_(p, -0.6, 0.6)
        out = {}
        with torch.no_grad():
            for task in (0, 1):
                out[task] = model.decode(xs, x_lens, task_index=task, **opts)
        ok, varied = True, False
        for task in (0, 1):
            hl = np.array([len(h) for h in out[task][0]])
            toks = np.concatenate([np.asarray(h, np.int64) for h in out[task][0]])
            ok &= len(np.unique(toks)) >= 2
            varied |= len(np.unique(hl)) >= 2
        ok &= varied
        if ok:
            break
    else:
        raise RuntimeError('no seed found for beam_hatt')
    arrays = {}
    for task in (0, 1):
        hyps, aw, perm = out[task]
        arrays['hyp_flat_%d' % task] = np.concatenate([np.asarray(h, np.int64) for h in hyps])
        arrays['hyp_lens_%d' % task] = np.array([len(h) for h in hyps], np.int32)
        arrays['aw_flat_%d' % task] = np.concatenate([np.asarray(a, np.float32).reshape(-1)
                                                      for a in aw])
        arrays['perm'] = np.asarray(perm).astype(np.int64)
    _save('beam_hatt', kwargs=np.array(json.dumps(kw)), opts=np.array(json.dumps(opts)),
          seed=np.array([seed]), xs=xs, x_lens=x_lens, **arrays, **_sd(model))


def case_decode_variants():
    """Greedy and beam decoding (attention_seq2seq.py:866-1237) of decoder
    variants: luong and conditional orders, a 2-layer residual decoder, the
    backward decoder alone (hypotheses reversed) and with a weaker forward one
    (decodes forward).  Random init uniform +-0.6; the seed is the first whose
    greedy output has at least three distinct tokens."""
    from models.pytorch_v3.attention.attention_seq2seq import AttentionSeq2seq
    _install_beam_shims()
    only = _selected()
    base = dict(input_size=8, encoder_type='lstm', encoder_bidirectional=True,
                encoder_num_units=6, encoder_num_proj=0, encoder_num_layers=2,
                attention_type='location', attention_dim=7, decoder_type='lstm',
                decoder_num_units=9, decoder_num_layers=1, embedding_dim=4,
                dropout_input=0, dropout_encoder=0, dropout_decoder=0, dropout_embedding=0,
                num_classes=6, parameter_init=0.1, subsample_list=[False, True],
                subsample_type='drop', attention_conv_num_channels=3,
                attention_conv_width=5, bottleneck_dim=11, ctc_loss_weight=0,
                label_smoothing_prob=0, init_dec_state='zero')
    specs = [('decv_luong', dict(base, decoding_order='luong')),
             ('decv_cond', dict(base, decoding_order='conditional', init_dec_state='first')),
             ('decv_dec2', dict(base, decoder_num_layers=2, decoder_residual=True)),
             ('decv_bwd', dict(base, backward_loss_weight=1.0, init_dec_state='final')),
             ('decv_content', dict(base, attention_type='content')),
             ('decv_gru', dict(base, encoder_type='gru', decoder_type='gru', bridge_layer=True,
                               init_dec_state='first'))]
    rng0 = np.random.RandomState(6)
    B, T = 4, 22
    x_lens = np.array([22, 17, 20, 11], np.int32)
    xs = rng0.randn(B, T, 8).astype(np.float32)
    for b in range(B):
        xs[b, x_lens[b]:] = 0
    for name, kw in specs:
        if only and name not in only:
            continue
        for seed in range(1623, 1623 + 500):
            torch.manual_seed(seed)
            model = AttentionSeq2seq(**kw)
            for p in model.parameters():
                torch.nn.init.uniform_(p, -0.6, 0.6)
            with torch.no_grad():
                g_hyps, g_aw, perm = model.decode(xs, x_lens, beam_width=1, max_decode_len=12)
            if len(np.unique(np.asarray(g_hyps))) >= 3:
                break
        else:
            raise RuntimeError('no seed found for ' + name)
        with torch.no_grad():
            b_hyps, b_aw, _ = model.decode(xs, x_lens, beam_width=3, max_decode_len=12)
        _save(name, kwargs=np.array(json.dumps(kw)), seed=np.array([seed]), xs=xs,
              x_lens=x_lens, greedy=np.asarray(g_hyps, np.int64),
              greedy_aw=np.asarray(g_aw, np.float32), perm=np.asarray(perm).astype(np.int64),
              beam_flat=np.concatenate([np.asarray(h, np.int64) for h in b_hyps]),
              beam_lens=np.array([len(h) for h in b_hyps], np.int32),
              beam_aw_flat=np.concatenate([np.asarray(a, np.float32).reshape(-1) for a in b_aw]),
              **_sd(model))


if __name__ == '__main__':
    _install_shims()
    if _selected():          # regenerate only the named model_ctc_* / dec_* cases
        case_ctc_model()
        case_attention_model()
        case_attention_decode()
        case_hier_attention_model()
        case_attention_prod()
        case_attention_beam()
        case_hier_attention_beam()
        case_decode_variants()
        if 'loader' in _selected():
            case_loader()
        sys.exit(0)
    case_ctc()
    case_encoder()
    case_attention_step()
    case_ctc_model()
    case_vgg_model()
    case_hier_ctc_model()
    case_attention_model()
    case_hier_attention_model()
    case_attention_prod()
    case_attention_decode()
    case_loader()
    case_attention_beam()
    case_hier_attention_beam()
    case_decode_variants()
