"""AttentionSeq2seq (reference models/pytorch_v3/attention/attention_seq2seq.py)
on the MI355X hot path: hybrid CTC + location-attention training step.

Drop-in: same constructor kwargs / defaults (:110-163), same submodule and
parameter names and the same torch RNG consumption at construction (state_dicts
interchange bit for bit), same ``forward(xs, ys, x_lens, y_lens, is_eval)``
contract and loss assembly (:422-562):

    loss = w_fwd * L_att + lambda * L_ctc                (NOT (1 - lambda) L_att)
    L_att = (1 - ls) * CE_sum / B + LS / B   (ls > 0)     else CE_sum / B
    L_ctc = sum_b cost_b / B

MI355X design: the teacher-forced decoder loop (bahdanau order) is ONE fused
op (native_ops.att_decoder): everything that does not depend on the
recurrence -- the input-embedding projection of every step, W_enc of the
encoder states, the W_d / W_c bottleneck, the output layer and the loss -- is
hoisted into full-batch GEMMs before / after the loop; per step only the
LSTMCell and the fused location-attention kernel run.
"""
import random

import numpy as np
import torch

from .... import native_ops as ops
from ..base import ModelBase, check_recurrences, eval_retry
from ..linear import LinearND, Embedding, Embedding_LS
from ..encoders.load_encoder import load
from .rnn_decoder import RNNDecoder
from .attention_layer import AttentionMechanism
from ..ctc.ctc import _concatenate_labels_np
from ..ctc.decoders.greedy_decoder import GreedyDecoder


class AttentionSeq2seq(ModelBase):

    def __init__(self, input_size, encoder_type, encoder_bidirectional, encoder_num_units,
                 encoder_num_proj, encoder_num_layers, attention_type, attention_dim,
                 decoder_type, decoder_num_units, decoder_num_layers, embedding_dim,
                 dropout_input, dropout_encoder, dropout_decoder, dropout_embedding, num_classes,
                 parameter_init_distribution='uniform', parameter_init=0.1,
                 recurrent_weight_orthogonal=False, init_forget_gate_bias_with_one=True,
                 subsample_list=[], subsample_type='drop', bridge_layer=False,
                 init_dec_state='first', sharpening_factor=1, logits_temperature=1,
                 sigmoid_smoothing=False, coverage_weight=0, ctc_loss_weight=0,
                 attention_conv_num_channels=10, attention_conv_width=201, num_stack=1,
                 splice=1, input_channel=1, conv_channels=[], conv_kernel_sizes=[],
                 conv_strides=[], poolings=[], activation='relu', batch_norm=False,
                 scheduled_sampling_prob=0, scheduled_sampling_max_step=0,
                 label_smoothing_prob=0, weight_noise_std=0, encoder_residual=False,
                 encoder_dense_residual=False, decoder_residual=False,
                 decoder_dense_residual=False, decoding_order='bahdanau', bottleneck_dim=256,
                 backward_loss_weight=0, num_heads=1):
        super(ModelBase, self).__init__()
        self.model_type = 'attention'
        self.input_size = input_size
        self.num_stack = num_stack
        self.encoder_type = encoder_type
        self.encoder_num_units = encoder_num_units * (2 if encoder_bidirectional else 1)
        self.encoder_num_proj = encoder_num_proj
        self.encoder_num_layers = encoder_num_layers
        self.subsample_list = subsample_list
        self.decoder_type = decoder_type
        self.decoder_num_units_0 = decoder_num_units
        self.decoder_num_layers_0 = decoder_num_layers
        self.embedding_dim = embedding_dim
        self._emb_dims = {0: embedding_dim}          # per task (hierarchical: task 1)
        self.num_classes = num_classes + 1
        self.sos_0 = num_classes
        self.eos_0 = num_classes
        self.decoding_order = decoding_order
        assert 0 <= backward_loss_weight <= 1
        self.fwd_weight_0 = 1 - backward_loss_weight
        self.bwd_weight_0 = backward_loss_weight
        if init_dec_state not in ['zero', 'mean', 'final', 'first']:
            raise ValueError('init_dec_state must be "zero" or "mean" or "final" or "first".')
        self.init_dec_state_0_fwd = init_dec_state
        self.sharpening_factor = sharpening_factor
        self.logits_temperature = logits_temperature
        self.sigmoid_smoothing = sigmoid_smoothing
        self.coverage_weight = coverage_weight
        self.num_heads_0 = num_heads
        self.weight_noise_injection = False
        self.weight_noise_std = float(weight_noise_std)
        if scheduled_sampling_prob > 0 and scheduled_sampling_max_step == 0:
            raise ValueError
        self.ss_prob = scheduled_sampling_prob
        self._ss_prob = scheduled_sampling_prob
        self.ss_max_step = scheduled_sampling_max_step
        self._step = 0
        self.ls_prob = label_smoothing_prob
        self.ctc_loss_weight = ctc_loss_weight
        self.dropout_decoder = float(dropout_decoder)
        self.dropout_embedding = float(dropout_embedding)

        self.init_dec_state_0_bwd = init_dec_state
        if backward_loss_weight > 0:                   # :187-191
            if init_dec_state == 'first':
                self.init_dec_state_0_bwd = 'final'
            elif init_dec_state == 'final':
                self.init_dec_state_0_bwd = 'first'
        if encoder_type != decoder_type:
            self.init_dec_state_0_fwd = 'zero'
            self.init_dec_state_0_bwd = 'zero'

        unsupported = []
        if decoding_order not in ('bahdanau', 'luong', 'conditional'):
            raise ValueError(decoding_order)
        if encoder_type == 'cnn':
            unsupported.append('cnn encoder')
        if coverage_weight != 0:
            unsupported.append('coverage')
        if unsupported:
            raise NotImplementedError('MI355X AttentionSeq2seq: not yet supported: ' +
                                      ', '.join(unsupported))

        self.encoder = load(encoder_type=encoder_type)(
            input_size=input_size, rnn_type=encoder_type, bidirectional=encoder_bidirectional,
            num_units=encoder_num_units, num_proj=encoder_num_proj,
            num_layers=encoder_num_layers, dropout_input=dropout_input,
            dropout_hidden=dropout_encoder, subsample_list=subsample_list,
            subsample_type=subsample_type, batch_first=True, merge_bidirectional=False,
            pack_sequence=True, num_stack=num_stack, splice=splice,
            input_channel=input_channel, conv_channels=conv_channels,
            conv_kernel_sizes=conv_kernel_sizes, conv_strides=conv_strides, poolings=poolings,
            activation=activation, batch_norm=batch_norm, residual=encoder_residual,
            dense_residual=encoder_dense_residual, nin=0)
        if bridge_layer:                               # :268-278
            self.bridge_0 = LinearND(self.encoder_num_units, decoder_num_units,
                                     dropout=dropout_encoder)
            self.encoder_num_units = decoder_num_units
            self.is_bridge = True
        else:
            self.is_bridge = False

        # :280-361 per direction (registration order = RNG order)
        directions = (['fwd'] if self.fwd_weight_0 > 0 else []) + \
            (['bwd'] if self.bwd_weight_0 > 0 else [])
        self._directions = directions
        for dir in directions:
            if getattr(self, 'init_dec_state_0_' + dir) != 'zero':
                setattr(self, 'W_dec_init_0_' + dir,
                        LinearND(self.encoder_num_units, decoder_num_units))
            if decoding_order == 'conditional':
                setattr(self, 'decoder_first_0_' + dir,
                        RNNDecoder(input_size=embedding_dim, rnn_type=decoder_type,
                                   num_units=decoder_num_units, num_layers=1,
                                   dropout=dropout_decoder, residual=False,
                                   dense_residual=False))
                setattr(self, 'decoder_second_0_' + dir,
                        RNNDecoder(input_size=self.encoder_num_units, rnn_type=decoder_type,
                                   num_units=decoder_num_units, num_layers=1,
                                   dropout=dropout_decoder, residual=False,
                                   dense_residual=False))
            else:
                setattr(self, 'decoder_0_' + dir,
                        RNNDecoder(input_size=self.encoder_num_units + embedding_dim,
                                   rnn_type=decoder_type, num_units=decoder_num_units,
                                   num_layers=decoder_num_layers, dropout=dropout_decoder,
                                   residual=decoder_residual,
                                   dense_residual=decoder_dense_residual))
            setattr(self, 'attend_0_' + dir, AttentionMechanism(
                encoder_num_units=self.encoder_num_units, decoder_num_units=decoder_num_units,
                attention_type=attention_type, attention_dim=attention_dim,
                sharpening_factor=sharpening_factor, sigmoid_smoothing=sigmoid_smoothing,
                out_channels=attention_conv_num_channels, kernel_size=attention_conv_width,
                num_heads=num_heads))
            setattr(self, 'W_d_0_' + dir,
                    LinearND(decoder_num_units, bottleneck_dim, dropout=dropout_decoder))
            setattr(self, 'W_c_0_' + dir,
                    LinearND(self.encoder_num_units, bottleneck_dim, dropout=dropout_decoder))
            setattr(self, 'fc_0_' + dir, LinearND(bottleneck_dim, self.num_classes))
        if label_smoothing_prob > 0:
            self.embed_0 = Embedding_LS(num_classes=self.num_classes,
                                        embedding_dim=embedding_dim, dropout=dropout_embedding,
                                        label_smoothing_prob=label_smoothing_prob)
        else:
            self.embed_0 = Embedding(num_classes=self.num_classes, embedding_dim=embedding_dim,
                                     dropout=dropout_embedding)
        if ctc_loss_weight > 0:
            self.fc_ctc_0 = LinearND(decoder_num_units if self.is_bridge
                                     else self.encoder_num_units, num_classes + 1)
            self._decode_ctc_greedy_np = GreedyDecoder(blank_index=0)

        # :397-420
        self.init_weights(parameter_init, distribution=parameter_init_distribution,
                          ignore_keys=['bias'])
        self.init_weights(0, distribution='constant', keys=['bias'])
        if recurrent_weight_orthogonal:
            self.init_weights(parameter_init, distribution='orthogonal',
                              keys=[encoder_type, 'weight'], ignore_keys=['bias'])
            self.init_weights(parameter_init, distribution='orthogonal',
                              keys=[decoder_type, 'weight'], ignore_keys=['bias'])
        if init_forget_gate_bias_with_one:
            self.init_forget_gate_bias_with_one()
        self.flatten_parameters_()
        self.encoder.__dict__['_owner'] = self

    # ------------------------------------------------------------------
    @eval_retry
    def forward(self, xs, ys, x_lens, y_lens, is_eval=False):
        """attention_seq2seq.py:422-562."""
        if is_eval:
            self.eval()
        else:
            self.train()
            if self.weight_noise_injection:
                with torch.no_grad():
                    self._flat_param.add_(torch.randn_like(self._flat_param) *
                                          self.weight_noise_std)
        B = len(xs)
        xs_d = self.np2var(xs, dtype='float')
        enc_out, enc_lens_d, perm_d = self._encode(xs_d, x_lens)
        perm = self.encoder.last_perm_np
        ys = np.asarray(ys)
        y_lens = np.asarray(y_lens).astype(np.int64)

        loss = None
        if self.fwd_weight_0 > 0:
            ys_in, ys_out = self._ys_in_out(ys, y_lens, self.eos_0, perm)
            self._ys_in_host = {0: ys_in}     # host copy: token-grouped embedding gradient
            loss = self.compute_xe_loss(enc_out, self.np2var(ys_in), self.np2var(ys_out),
                                        enc_lens_d, None, task=0, dir='fwd',
                                        weight=self.fwd_weight_0)
        if self.bwd_weight_0 > 0:             # :489-528: each label sequence reversed
            ys_rev = ys.copy()
            for b in range(B):
                ys_rev[b, :y_lens[b]] = ys[b, :y_lens[b]][::-1]
            ys_in, ys_out = self._ys_in_out(ys_rev, y_lens, self.eos_0, perm)
            self._ys_in_host = {0: ys_in}
            loss_bwd = self.compute_xe_loss(enc_out, self.np2var(ys_in), self.np2var(ys_out),
                                            enc_lens_d, None, task=0, dir='bwd',
                                            weight=self.bwd_weight_0)
            loss = loss_bwd if loss is None else ops.add(loss, loss_bwd)
        if self.ctc_loss_weight > 0:
            ys_ctc = (ys + 1)[perm]
            yl = y_lens[perm].astype(np.int32)
            loss = loss + self.compute_ctc_loss(enc_out, ys_ctc, enc_lens_d, yl,
                                                scale=self.ctc_loss_weight)
        if is_eval:
            check_recurrences(self)
            return float(loss.item())
        self._step += 1
        if self.ss_prob > 0:
            self._ss_prob = min(self.ss_prob, self.ss_prob / self.ss_max_step * self._step)
        return loss

    @staticmethod
    def _ys_in_out(ys, y_lens, eos, perm):
        """ys_in = [<sos>, y, <eos>...], ys_out = [y, <eos>, -1...] (:458-473; <sos> ==
        <eos>), host-side and vectorised, rows in the encoder's sorted order."""
        B, Lp = ys.shape
        pos = np.arange(Lp + 1)[None, :]
        ys_pad = np.concatenate([ys, np.full((B, 1), -1, ys.dtype)], axis=1)
        ys_out = np.where(pos < y_lens[:, None], ys_pad,
                          np.where(pos == y_lens[:, None], eos, -1)).astype(np.int64)
        ys_in = np.full((B, Lp + 1), eos, np.int64)
        ys_in[:, 1:] = np.where(pos[:, :-1] < y_lens[:, None], ys, eos)
        return ys_in[perm], ys_out[perm]

    def compute_xe_loss(self, enc_out, ys_in, ys_out, x_lens, y_lens, task, dir, weight=1.0):
        """:564-607 (forward decoder of `task`, loss already multiplied by `weight`)."""
        logits, _ = self._decode_train(enc_out, x_lens, ys_in, task, dir)
        if self.logits_temperature != 1:
            logits = logits * (1.0 / self.logits_temperature)
        B = enc_out.shape[0]
        ls = self.ls_prob
        ce = weight * (1 - ls) / B if ls > 0 else weight / B
        # LS rows are t < y_len + 1 == the rows whose target is not -1
        return ops.xent(logits, ys_out, None, 0, ce_scale=ce, ls_scale=weight * ls / B)

    def compute_ctc_loss(self, enc_out, ys_ctc, x_lens, y_lens, task=0, scale=1.0):
        """:609-653 on the HIP CTC kernel; ys_ctc already +1 (blank 0)."""
        fc = getattr(self, 'fc_ctc_%d' % task)
        labels = self.np2var(_concatenate_labels_np(ys_ctc, y_lens))
        yl_d = self.np2var(y_lens.astype(np.int32))
        B = enc_out.shape[0]
        max_l = int(y_lens.max()) if len(y_lens) else 0
        if not (self.training and fc.dropout_p > 0):
            # LinearND + CTC as one op (native_ops.linear_ctc_loss)
            loss, _ = ops.linear_ctc_loss(enc_out, fc.fc.weight, fc.fc.bias, labels, yl_d, x_lens,
                                          max_l, loss_scale=scale / B)
            return loss
        loss, _ = ops.ctc_loss(fc(enc_out), labels, yl_d, x_lens, max_l, loss_scale=scale / B)
        return loss

    def _encode(self, xs, x_lens, is_multi_task=False):
        """:655-698 (with num_layers_sub >= 1 the encoder returns the sub-task tap
        too: (xs, x_lens, xs_sub, x_lens_sub, perm_idx)); the bridge layer
        (:686-690) maps the main output to the decoder width."""
        out = self.encoder(xs, x_lens, volatile=not self.training)
        if getattr(self, 'is_bridge', False):
            out = (self.bridge_0(out[0]),) + tuple(out[1:])
        return out

    def _init_h0(self, enc_out, task=0, dir='fwd'):
        """_init_dec_state (:801-864): zero / mean (over all T, padding included,
        :832) / first / final, then tanh(W_dec_init(.))."""
        mode = getattr(self, 'init_dec_state_%d_%s' % (task, dir))
        if mode == 'zero':
            return None
        T = enc_out.shape[1]
        lin = getattr(self, 'W_dec_init_%d_%s' % (task, dir)).fc
        if mode == 'mean':
            return ops.tanh(ops.linear(ops.mean_time(enc_out), lin.weight, lin.bias))
        h = ops.linear_ex(enc_out, lin.weight, lin.bias, t_index=0 if mode == 'first' else T - 1)
        return ops.tanh(h)

    def _ss_steps(self, S):
        """Scheduled-sampling decisions of one decoder pass (attention_seq2seq.py:744):
        the reference draws ``random.random() < self._ss_prob`` at every step
        t > 0 once training has stepped (same Python RNG stream)."""
        if not (self.training and self.ss_prob > 0 and self._step > 0):
            return None
        flags = np.zeros(S, np.int32)
        for t in range(1, S):
            flags[t] = random.random() < self._ss_prob
        return flags if flags.any() else None

    def _fused_ok(self, task, dir):
        """The fused decoder op covers bahdanau order with a 1-layer decoder
        without residual connections (location or content attention)."""
        dec = getattr(self, 'decoder_%d_%s' % (task, dir), None)
        return (self.decoding_order == 'bahdanau' and dec is not None and dec.num_layers == 1
                and dec.rnn_type == 'lstm' and not dec.residual and not dec.dense_residual)

    @staticmethod
    def _run_dec(mod, inp, hx, cx):
        """RNNDecoder.forward with the (hx, cx) pair of either cell type (GRU
        decoders carry hx only)."""
        if mod.rnn_type == 'gru':
            out, hx = mod(inp, hx)
            return out, hx, cx
        out, (hx, cx) = mod(inp, (hx, cx))
        return out, hx, cx

    def _decode_train(self, enc_out, x_lens, ys, task=0, dir='fwd'):
        if not self._fused_ok(task, dir):
            return self._decode_train_steps(enc_out, x_lens, ys, task, dir)
        return self._decode_train_fused(enc_out, x_lens, ys, task, dir)

    def _decode_train_steps(self, enc_out, x_lens, ys, task=0, dir='fwd'):
        """:704-799 step by step for what the fused op does not cover: multi-layer
        and residual decoders (RNNDecoder.forward, HIP LSTM cells) and the luong
        / conditional decoding orders.  Each step is HIP autograd ops (the
        decoder cells, the attention step with its HIP backward); the W_d / W_c
        bottleneck and the output layer run once over all steps afterwards,
        except under scheduled sampling, which needs each step's logits."""
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        W_d, W_c = getattr(self, 'W_d_%d_%s' % (task, dir)), getattr(self, 'W_c_%d_%s' % (task, dir))
        fc = getattr(self, 'fc_%d_%s' % (task, dir))
        embed = getattr(self, 'embed_%d' % task)
        order = self.decoding_order
        if order == 'conditional':
            dec1 = getattr(self, 'decoder_first_%d_%s' % (task, dir))
            dec2 = getattr(self, 'decoder_second_%d_%s' % (task, dir))
            nl = 1
        else:
            dec1 = getattr(self, 'decoder_%d_%s' % (task, dir))
            nl = dec1.num_layers
        B, T, E = enc_out.shape
        S = ys.shape[1]
        D = getattr(self, 'decoder_num_units_%d' % task)
        dev = enc_out.device
        h0 = self._init_h0(enc_out, task, dir)
        zero = torch.zeros(B, D, dtype=torch.float32, device=dev)
        hx = [h0 if h0 is not None else zero for _ in range(nl)]
        cx = [zero for _ in range(nl)]
        dec_out = h0 if h0 is not None else zero
        aw = torch.zeros(B, T, dtype=torch.float32, device=dev)
        ctx = torch.zeros(B, E, dtype=torch.float32, device=dev)
        lens = x_lens if torch.is_tensor(x_lens) else torch.from_numpy(
            np.asarray(x_lens, np.int32)).to(dev)
        hosts = getattr(self, '_ys_in_host', None) or {}
        ys_host = hosts.pop(task, None)
        if ys_host is not None and tuple(ys_host.shape) != tuple(ys.shape):
            ys_host = None
        y_emb = embed(ys, ys_host)                                # [B, S, emb]
        enc_a = att.W_enc_head0(enc_out).unsqueeze(3)             # [B, T, A, 1]
        ss = self._ss_steps(S)

        def generate(d, c):
            return fc(ops.add_tanh(W_d(d), W_c(c)))

        decs, ctxs, aws, step_logits = [], [], [], []
        for t in range(S):
            if ss is not None and ss[t]:                          # :744-748
                prev = step_logits[-1].detach()
                y = embed(ops.row_argmax(prev).view(B, 1)).view(B, -1).detach()
            else:
                y = y_emb[:, t]
            if order == 'bahdanau':
                if t > 0:
                    d3, hx, cx = self._run_dec(dec1, torch.cat([y, ctx], dim=-1).unsqueeze(1),
                                               hx, cx)
                    dec_out = d3.squeeze(1)
                c3, a3 = att(enc_out, enc_a, lens, dec_out.unsqueeze(1), aw.unsqueeze(2))
            elif order == 'luong':
                d3, hx, cx = self._run_dec(dec1, torch.cat([y, ctx], dim=-1).unsqueeze(1), hx, cx)
                dec_out = d3.squeeze(1)
                c3, a3 = att(enc_out, enc_a, lens, dec_out.unsqueeze(1), aw.unsqueeze(2))
            else:                                                 # conditional
                d3, hx, cx = self._run_dec(dec1, y.unsqueeze(1), hx, cx)
                c3, a3 = att(enc_out, enc_a, lens, d3, aw.unsqueeze(2))
                d3, hx, cx = self._run_dec(dec2, c3, hx, cx)
                dec_out = d3.squeeze(1)
            ctx, aw = c3.squeeze(1), a3.squeeze(2)
            decs.append(dec_out)
            ctxs.append(ctx)
            aws.append(aw)
            if ss is not None:
                step_logits.append(generate(dec_out.unsqueeze(1), ctx.unsqueeze(1)))
        if ss is not None:
            logits = torch.cat(step_logits, dim=1)
        else:
            logits = generate(torch.stack(decs, dim=1), torch.stack(ctxs, dim=1))
        return logits, torch.stack(aws, dim=1)

    def _decode_train_fused(self, enc_out, x_lens, ys, task=0, dir='fwd'):
        """:704-799 as one fused op (bahdanau order).  Returns (logits [B,S,V], aw).

        Training mode: decoder dropout on h (rnn_decoder.py:97-98) inside the
        fused loop, dropout on the W_d / W_c bottleneck outputs (LinearND,
        linear.py:44-45), embedding dropout, and scheduled sampling -- sampled
        steps take embed(argmax logits_{t-1}) computed inside the loop from the
        same dropped bottleneck the loss sees (shared dropout seeds).

        With a BLSTM encoder, the decoder-side linear layers' weight gradients
        run beside that encoder's top backward recurrence
        (native_ops.wgrad_beside_encoder; ASR_DEC_WGRAD_SIDE=0: before it)."""
        bh = ops._produced_by_blstm(enc_out) if enc_out.dim() == 3 else None
        if bh is not None:
            with ops.wgrad_beside_encoder(*bh):
                return self._decode_train_fused_body(enc_out, x_lens, ys, task, dir)
        return self._decode_train_fused_body(enc_out, x_lens, ys, task, dir)

    def _decode_train_fused_body(self, enc_out, x_lens, ys, task=0, dir='fwd'):
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        cell = getattr(self, 'decoder_%d_%s' % (task, dir)).lstm_l0
        W_d, W_c = getattr(self, 'W_d_%d_%s' % (task, dir)), getattr(self, 'W_c_%d_%s' % (task, dir))
        fc = getattr(self, 'fc_%d_%s' % (task, dir))
        embed = getattr(self, 'embed_%d' % task)
        emb_dim = self._emb_dims[task]
        S = ys.shape[1]
        h0 = self._init_h0(enc_out, task, dir)
        enc_a = att.W_enc_head0(enc_out)                          # one GEMM for all frames
        hosts = getattr(self, '_ys_in_host', None) or {}
        ys_host = hosts.pop(task, None)                           # one use only
        if ys_host is not None and tuple(ys_host.shape) != tuple(ys.shape):
            ys_host = None
        y_emb = embed(ys, ys_host)                                # [B, S, emb] (+ dropout)
        pre_emb = ops.linear_ex(y_emb, cell.weight_ih, cell.bias_ih, cell.bias_hh, c0=0,
                                K=emb_dim)                        # all steps' input projection
        p_h = self.dropout_decoder if self.training else 0.0
        p_b = W_d.dropout_p if self.training else 0.0
        seed_d = ops.next_seed() if p_b > 0 else 0
        seed_c = ops.next_seed() if p_b > 0 else 0
        ss = self._ss_steps(S)
        train_opts = None
        if p_h > 0 or ss is not None:
            train_opts = dict(dropout_hidden=p_h, seed_hidden=ops.next_seed() if p_h > 0 else 0)
            if ss is not None:
                emb_ls = isinstance(embed, Embedding_LS)
                emb_w = embed.embed.fc.weight if emb_ls else embed.embed.weight
                p_e = self.dropout_embedding if self.training else 0.0
                train_opts.update(
                    ss_steps=ss, w_d=W_d.fc.weight, b_d=W_d.fc.bias, w_c=W_c.fc.weight,
                    b_c=W_c.fc.bias, w_fc=fc.fc.weight, b_fc=fc.fc.bias,
                    emb_w=emb_w, emb_trans=int(emb_ls), b_ih=cell.bias_ih, b_hh=cell.bias_hh,
                    drop_d=p_b, seed_d=seed_d, drop_c=p_b, seed_c=seed_c, drop_emb=p_e,
                    seed_emb=ops.next_seed() if p_e > 0 else 0)
        dec, ctx, aw = ops.att_decoder(enc_out, enc_a, x_lens, pre_emb, h0, emb_dim,
                                       self.sharpening_factor, self.sigmoid_smoothing,
                                       cell.weight_ih, cell.weight_hh, att.W_dec_head0.fc.weight,
                                       *att.conv_weights(),
                                       att.V_head0.fc.weight, train_opts)
        if p_b > 0:   # two LinearND with their own dropout masks, then tanh of the sum
            a = ops.dropout(ops.linear(dec, W_d.fc.weight, W_d.fc.bias), p_b, seed=seed_d)
            c = ops.dropout(ops.linear(ctx, W_c.fc.weight, W_c.fc.bias), p_b, seed=seed_c)
            z = ops.add_tanh(a, c)
        else:
            z = ops.tanh(ops.linear2(dec, W_d.fc.weight, W_d.fc.bias, ctx, W_c.fc.weight,
                                     W_c.fc.bias))
        logits = fc(z)
        return logits, aw

    @eval_retry
    @torch.no_grad()
    def decode_ctc(self, xs, x_lens, beam_width=1, task_index=0):
        """:1239-1289 (greedy; HIP best path)."""
        self.eval()
        if beam_width != 1:
            raise NotImplementedError
        xs_d = self.np2var(xs, dtype='float')
        enc_out, enc_lens_d, _ = self._encode(xs_d, x_lens)
        logits = self.fc_ctc_0(enc_out)
        check_recurrences(self)
        hyps = self._decode_ctc_greedy_np(logits, enc_lens_d)
        best = np.array([h - 1 for h in hyps] + [None], dtype=object)[:-1]
        return best, self.encoder.last_perm_np.copy()

    @eval_retry
    @torch.no_grad()
    def decode(self, xs, x_lens, beam_width, max_decode_len, min_decode_len=0,
               length_penalty=0, coverage_penalty=0, task_index=0, resolving_unk=False):
        """:866-915.  Returns (best_hyps int64 [B, T_out], aw [B, T_out, T_in],
        perm_idx), rows in the encoder's length-sorted order like the reference."""
        self.eval()
        xs_d = self.np2var(xs, dtype='float')
        enc_out, enc_lens_d, _ = self._encode(xs_d, x_lens)
        dir = 'fwd' if self.fwd_weight_0 >= self.bwd_weight_0 else 'bwd'   # :893
        if beam_width == 1:
            best_hyps, aw = self._decode_infer_greedy(enc_out, enc_lens_d, max_decode_len,
                                                      dir=dir)
        else:
            best_hyps, aw = self._decode_infer_beam(enc_out, self.encoder.last_lens_np, beam_width,
                                                    max_decode_len, min_decode_len,
                                                    length_penalty, coverage_penalty, dir=dir)
        check_recurrences(self)
        return best_hyps, aw, self.encoder.last_perm_np.copy()

    def _infer_step(self, task, dir, t, y_emb, st, enc, enc_a, lens):
        """One inference decoder step (:963-1001) on the HIP per-step ops, for any
        decoding order / decoder depth.  st = dict(h, c (lists per layer), dec,
        ctx, aw); y_emb [n, emb] (unused at t = 0 in bahdanau order).  Returns
        (new st, logits [n, V])."""
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        W_d, W_c = getattr(self, 'W_d_%d_%s' % (task, dir)), getattr(self, 'W_c_%d_%s' % (task, dir))
        fc = getattr(self, 'fc_%d_%s' % (task, dir))
        hx, cx, dec, ctx, aw = list(st['h']), list(st['c']), st['dec'], st['ctx'], st['aw']
        n = dec.shape[0]
        L = aw.shape[1]
        if self.decoding_order == 'conditional':
            d1 = getattr(self, 'decoder_first_%d_%s' % (task, dir))
            d2 = getattr(self, 'decoder_second_%d_%s' % (task, dir))
            dd, hx, cx = self._run_dec(d1, y_emb.unsqueeze(1), hx, cx)
            c3, a3 = att(enc, enc_a, lens, dd, aw.unsqueeze(2))
            d3, hx, cx = self._run_dec(d2, c3, hx, cx)
            dec = d3.squeeze(1)
        else:
            dm = getattr(self, 'decoder_%d_%s' % (task, dir))
            if self.decoding_order == 'luong' or t > 0:
                d3, hx, cx = self._run_dec(dm, torch.cat([y_emb, ctx], dim=-1).unsqueeze(1),
                                           hx, cx)
                dec = d3.squeeze(1)
            c3, a3 = att(enc, enc_a, lens, dec.unsqueeze(1), aw.unsqueeze(2))
        ctx, aw = c3.reshape(n, -1), a3.reshape(n, L)
        logits = fc(ops.tanh(ops.linear2(dec, W_d.fc.weight, W_d.fc.bias, ctx, W_c.fc.weight,
                                         W_c.fc.bias)))
        return dict(h=hx, c=cx, dec=dec, ctx=ctx, aw=aw), logits

    def _init_state(self, enc_out, task, dir):
        """_init_dec_state (:801-864) as the step state dict of _infer_step."""
        B, T, E = enc_out.shape
        D = getattr(self, 'decoder_num_units_%d' % task)
        dev = enc_out.device
        if self.decoding_order == 'conditional':
            nl = 1
        else:
            nl = getattr(self, 'decoder_%d_%s' % (task, dir)).num_layers
        h0 = self._init_h0(enc_out, task, dir)
        zero = torch.zeros(B, D, dtype=torch.float32, device=dev)
        h = h0 if h0 is not None else zero
        return dict(h=[h] * nl, c=[zero] * nl, dec=h,
                    ctx=torch.zeros(B, E, dtype=torch.float32, device=dev),
                    aw=torch.zeros(B, T, dtype=torch.float32, device=dev))

    @staticmethod
    def _reverse_bwd(best_hyps, y_lens):
        """:1027-1034 / :1231-1234: hypotheses of the backward decoder are
        reversed over their first y_lens tokens."""
        for b in range(len(best_hyps)):
            best_hyps[b][:y_lens[b]] = best_hyps[b][:y_lens[b]][::-1].copy()
        return best_hyps

    def _decode_infer_beam(self, enc_out, x_lens, beam_width, max_decode_len, min_decode_len,
                           length_penalty, coverage_penalty, task=0, dir='fwd'):
        """:1038-1237 (any decoding order / decoder depth).  Utterance by utterance like the
        reference, each over its own frames (enc_out[b, :x_len]); the live
        hypotheses of an utterance advance as ONE batch per step on the HIP ops
        (embedding, LSTMCell, the location-attention step, the bottleneck and
        output GEMMs), and the beam bookkeeping -- log-softmax, top-k, the
        min-length <eos> rule, length penalty, stable score sort, completion --
        runs on the host over the [n, V] log-probabilities of the step, as the
        reference does with its per-step reads.  Returns (best_hyps: an int64
        [B, L] array when every hypothesis has the same length, else an object
        array of int64 rows, each ending with <eos> when it completed; aw: list
        of [L_b, x_len_b] float32 arrays)."""
        if coverage_penalty > 0:
            raise NotImplementedError('coverage penalty (the reference raises too, :1150)')
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        embed = getattr(self, 'embed_%d' % task)
        sos, eos = getattr(self, 'sos_%d' % task), getattr(self, 'eos_%d' % task)
        dev = enc_out.device
        B, _, E = enc_out.shape
        lens = np.asarray(x_lens).reshape(-1).astype(np.int64)
        enc_a = att.W_enc_head0(enc_out)                            # [B, T, A]
        A = enc_a.shape[2]
        init = self._init_state(enc_out, task, dir)
        dm = getattr(self, 'decoder_%d_%s' % (task, dir), None)
        residual = dm is not None and dm.residual and dm.num_layers > 1

        def _rows(st, i):
            return {k: ([x[i:i + 1] for x in v] if isinstance(v, list) else v[i:i + 1])
                    for k, v in st.items()}
        best, aws = [], []
        for b in range(B):
            L = int(lens[b])
            enc_b = enc_out[b:b + 1, :L].contiguous()
            enc_a_b = enc_a[b:b + 1, :L].contiguous()
            state = dict(h=[x[b:b + 1] for x in init['h']], c=[x[b:b + 1] for x in init['c']],
                         dec=init['dec'][b:b + 1], ctx=init['ctx'][b:b + 1],
                         aw=init['aw'][b:b + 1, :L])
            beam = [dict(hyp=[sos], score=0.0, row=0, hist=[])]
            complete, step_aw = [], []
            for t in range(max_decode_len):
                n = len(beam)
                if n == 0:
                    break
                rows = torch.tensor([c['row'] for c in beam], dtype=torch.long, device=dev)
                st = {k: ([x.index_select(0, rows) for x in v] if isinstance(v, list)
                          else v.index_select(0, rows)) for k, v in state.items()}
                toks = np.array([c['hyp'][-1] for c in beam], np.int64).reshape(n, 1)
                y = embed(torch.from_numpy(toks).to(dev), toks).view(n, -1)
                if residual:
                    # the reference advances each hypothesis as a batch of one, and
                    # its residual decoder sums the lower layer over the batch
                    # (rnn_decoder.py:100-102): one step per hypothesis here too
                    outs = [self._infer_step(task, dir, t, y[i:i + 1], _rows(st, i), enc_b,
                                             enc_a_b.unsqueeze(3), [L]) for i in range(n)]
                    state = {k: ([torch.cat([o[0][k][l] for o in outs]) for l in range(len(v))]
                                 if isinstance(v, list) else torch.cat([o[0][k] for o in outs]))
                             for k, v in outs[0][0].items()}
                    logits = torch.cat([o[1] for o in outs])
                else:
                    state, logits = self._infer_step(
                        task, dir, t, y, st, enc_b.expand(n, L, E).contiguous(),
                        enc_a_b.expand(n, L, A).contiguous().unsqueeze(3), [L] * n)
                aw_t = state['aw']
                lg = logits.float().cpu().numpy()
                mx = lg.max(axis=1, keepdims=True)                          # log_softmax (f32)
                lp = lg - mx - np.log(np.exp(lg - mx).sum(axis=1, keepdims=True))
                k_top = min(beam_width, lp.shape[1])
                order = np.argsort(-lp, axis=1, kind='stable')[:, :k_top]   # topk, sorted
                step_aw.append(aw_t)
                new = []
                for i in range(n):
                    for k in range(k_top):
                        tok = int(order[i, k])
                        if tok == eos and len(beam[i]['hyp']) < min_decode_len:
                            continue
                        new.append(dict(hyp=beam[i]['hyp'] + [tok],
                                        score=beam[i]['score'] + float(lp[i, tok]) + length_penalty,
                                        row=i, hist=beam[i]['hist'] + [(t, i)]))
                new.sort(key=lambda c: c['score'], reverse=True)     # stable, as sorted()
                not_complete = []
                for cand in new[:beam_width]:
                    (complete if cand['hyp'][-1] == eos else not_complete).append(cand)
                if len(complete) >= beam_width:
                    complete = complete[:beam_width]
                    break
                beam = not_complete[:beam_width]
            if len(complete) == 0:
                complete = beam
            complete.sort(key=lambda c: c['score'], reverse=True)
            top = complete[0]
            best.append(np.array(top['hyp'][1:], dtype=np.int64))
            aw_rows = [step_aw[t][i] for t, i in top['hist']]
            aws.append(torch.stack(aw_rows).cpu().numpy() if aw_rows
                       else np.zeros((0, L), np.float32))
        if dir == 'bwd':                                  # :1231-1234
            best = self._reverse_bwd(best, [len(h) for h in best])
        if len(set(len(h) for h in best)) <= 1:
            return np.array(best), aws
        return np.array(best + [None], dtype=object)[:-1], aws

    def _decode_infer_greedy(self, enc_out, x_lens, max_decode_len, task=0, dir='fwd'):
        if self._fused_ok(task, dir):
            hyps, aw = self._decode_infer_greedy_fused(enc_out, x_lens, max_decode_len, task, dir)
        else:
            hyps, aw = self._decode_infer_greedy_steps(enc_out, x_lens, max_decode_len, task, dir)
        if dir == 'bwd':       # lengths counted up to the first <eos> (:1007-1014)
            eos = getattr(self, 'eos_%d' % task)
            y_lens = [int(np.argmax(h == eos)) if (h == eos).any() else len(h) for h in hyps]
            hyps = self._reverse_bwd(hyps, y_lens)
        return hyps, aw

    @torch.no_grad()
    def _decode_infer_greedy_steps(self, enc_out, x_lens, max_decode_len, task=0, dir='fwd'):
        """:917-1036 step by step (decoders the fused greedy op does not cover)."""
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        embed = getattr(self, 'embed_%d' % task)
        eos, sos = getattr(self, 'eos_%d' % task), getattr(self, 'sos_%d' % task)
        B = enc_out.shape[0]
        dev = enc_out.device
        enc_a = att.W_enc_head0(enc_out).unsqueeze(3)
        lens = x_lens if torch.is_tensor(x_lens) else torch.from_numpy(
            np.asarray(x_lens, np.int32)).to(dev)
        st = self._init_state(enc_out, task, dir)
        y = torch.full((B, 1), sos, dtype=torch.int64, device=dev)
        toks, aws = [], []
        for t in range(max_decode_len):
            st, logits = self._infer_step(task, dir, t, embed(y).view(B, -1), st, enc_out, enc_a,
                                          lens)
            y = ops.row_argmax(logits).view(B, 1)
            toks.append(y)
            aws.append(st['aw'])
            if bool((y == eos).all().item()):                     # :1017-1019
                break
        return (torch.cat(toks, dim=1).cpu().numpy(),
                torch.stack(aws, dim=1).cpu().numpy())

    def _decode_infer_greedy_fused(self, enc_out, x_lens, max_decode_len, task=0, dir='fwd'):
        """:917-1036 (bahdanau order, forward decoder): the whole loop is one
        fused decoder pass (native_ops.att_decode_greedy); the reference's early
        exit -- stop after the first step at which EVERY utterance emits <eos>
        -- becomes a truncation of the per-step tokens, which it does not change
        because later steps never feed back into earlier ones."""
        att = getattr(self, 'attend_%d_%s' % (task, dir))
        cell = getattr(self, 'decoder_%d_%s' % (task, dir)).lstm_l0
        W_d, W_c = getattr(self, 'W_d_%d_%s' % (task, dir)), getattr(self, 'W_c_%d_%s' % (task, dir))
        fc = getattr(self, 'fc_%d_%s' % (task, dir))
        embed = getattr(self, 'embed_%d' % task)
        emb_ls = isinstance(embed, Embedding_LS)
        emb_w = embed.embed.fc.weight if emb_ls else embed.embed.weight
        h0 = self._init_h0(enc_out, task, dir)
        enc_a = att.W_enc_head0(enc_out)
        gen = dict(w_d=W_d.fc.weight, b_d=W_d.fc.bias, w_c=W_c.fc.weight, b_c=W_c.fc.bias,
                   w_fc=fc.fc.weight, b_fc=fc.fc.bias, emb_w=emb_w,
                   emb_trans=int(emb_ls), b_ih=cell.bias_ih, b_hh=cell.bias_hh)
        toks, aw = ops.att_decode_greedy(enc_out, enc_a, x_lens, h0, self._emb_dims[task],
                                         self.sharpening_factor, self.sigmoid_smoothing,
                                         cell.weight_ih, cell.weight_hh,
                                         att.W_dec_head0.fc.weight, *att.conv_weights(),
                                         att.V_head0.fc.weight, gen,
                                         max_decode_len)
        toks = toks.cpu().numpy()
        all_eos = np.nonzero((toks == getattr(self, 'eos_%d' % task)).all(axis=0))[0]
        n = int(all_eos[0]) + 1 if len(all_eos) else toks.shape[1]   # :1017-1019
        return toks[:, :n], aw[:, :n].cpu().numpy()
