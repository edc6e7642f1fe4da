"""HierarchicalAttentionSeq2seq (reference
models/pytorch_v3/attention/hierarchical_attention_seq2seq.py) on the MI355X
hot path: a word-level attention decoder on the top encoder layer plus a
character-level attention decoder (and optionally a character CTC) on the
output of layer ``encoder_num_layers_sub`` (the CSJ /
Switchboard hierarchical recipes).

Construction follows the reference step by step (:24-422): the plain attention
model is built and initialised first, the encoder is rebuilt with the sub-task
tap, the sub-task modules are added in the reference's order
(``W_dec_init_1_fwd``, ``decoder_1_fwd``, ``attend_1_fwd``, ``W_d_1_fwd``,
``W_c_1_fwd``, ``fc_1_fwd``, ``embed_1``, ``fc_ctc_1``) and the initialisation
runs again -- so the same seed yields the same state_dict.

``forward(xs, ys, x_lens, y_lens, ys_sub, y_lens_sub, is_eval)`` (:424-567):

    loss = w_main * L_att(word) + w_sub * L_att(char) + w_ctc_sub * L_ctc(char)

returning (loss, loss_main, loss_sub) where loss_sub is the attention term
when ``sub_loss_weight > ctc_loss_weight_sub``, else the CTC term.  Both
decoders are the fused HIP decoder op of attention_seq2seq.py, the CTC term
the HIP CTC kernel.
"""
import numpy as np

from .attention_seq2seq import AttentionSeq2seq
from ..base import check_recurrences, eval_retry
from .attention_layer import AttentionMechanism
from .rnn_decoder import RNNDecoder
from ..encoders.load_encoder import load
from ..linear import LinearND, Embedding, Embedding_LS
from ..ctc.decoders.greedy_decoder import GreedyDecoder


class HierarchicalAttentionSeq2seq(AttentionSeq2seq):

    def __init__(self, input_size, encoder_type, encoder_bidirectional, encoder_num_units,
                 encoder_num_proj, encoder_num_layers, encoder_num_layers_sub, attention_type,
                 attention_dim, decoder_type, decoder_num_units, decoder_num_units_sub,
                 decoder_num_layers, decoder_num_layers_sub, embedding_dim, embedding_dim_sub,
                 dropout_input, dropout_encoder, dropout_decoder, dropout_embedding,
                 main_loss_weight, sub_loss_weight, num_classes, num_classes_sub,
                 parameter_init_distribution='uniform', parameter_init=0.1,
                 recurrent_weight_orthogonal=False, init_forget_gate_bias_with_one=True,
                 subsample_list=[], subsample_type='drop', bridge_layer=False,
                 init_dec_state='first', sharpening_factor=1, logits_temperature=1,
                 sigmoid_smoothing=False, coverage_weight=0, ctc_loss_weight_sub=0,
                 attention_conv_num_channels=10, attention_conv_width=201, num_stack=1,
                 splice=1, input_channel=1, conv_channels=[], conv_kernel_sizes=[],
                 conv_strides=[], poolings=[], activation='relu', batch_norm=False,
                 scheduled_sampling_prob=0, scheduled_sampling_max_step=0,
                 label_smoothing_prob=0, weight_noise_std=0, encoder_residual=False,
                 encoder_dense_residual=False, decoder_residual=False,
                 decoder_dense_residual=False, decoding_order='bahdanau', bottleneck_dim=256,
                 bottleneck_dim_sub=256, backward_sub=False, num_heads=1, num_heads_sub=1):
        # :87-138: the plain attention model first (its own initialisation included;
        # recurrent_weight_orthogonal / init_forget_gate_bias_with_one / activation stay
        # at their defaults there, as in the reference)
        super(HierarchicalAttentionSeq2seq, self).__init__(
            input_size=input_size, encoder_type=encoder_type,
            encoder_bidirectional=encoder_bidirectional, encoder_num_units=encoder_num_units,
            encoder_num_proj=encoder_num_proj, encoder_num_layers=encoder_num_layers,
            attention_type=attention_type, attention_dim=attention_dim,
            decoder_type=decoder_type, decoder_num_units=decoder_num_units,
            decoder_num_layers=decoder_num_layers, embedding_dim=embedding_dim,
            dropout_input=dropout_input, dropout_encoder=dropout_encoder,
            dropout_decoder=dropout_decoder, dropout_embedding=dropout_embedding,
            num_classes=num_classes, parameter_init=parameter_init,
            subsample_list=subsample_list, subsample_type=subsample_type,
            bridge_layer=bridge_layer, init_dec_state=init_dec_state,
            sharpening_factor=sharpening_factor, logits_temperature=logits_temperature,
            sigmoid_smoothing=sigmoid_smoothing, coverage_weight=coverage_weight,
            ctc_loss_weight=0, attention_conv_num_channels=attention_conv_num_channels,
            attention_conv_width=attention_conv_width, num_stack=num_stack, splice=splice,
            input_channel=input_channel, conv_channels=conv_channels,
            conv_kernel_sizes=conv_kernel_sizes, conv_strides=conv_strides, poolings=poolings,
            scheduled_sampling_prob=scheduled_sampling_prob,
            scheduled_sampling_max_step=scheduled_sampling_max_step,
            label_smoothing_prob=label_smoothing_prob, weight_noise_std=weight_noise_std,
            encoder_residual=encoder_residual, encoder_dense_residual=encoder_dense_residual,
            decoder_residual=decoder_residual, decoder_dense_residual=decoder_dense_residual,
            decoding_order=decoding_order, bottleneck_dim=bottleneck_dim,
            backward_loss_weight=0, num_heads=num_heads)
        self.model_type = 'hierarchical_attention'
        if backward_sub:
            raise NotImplementedError('MI355X HierarchicalAttentionSeq2seq: backward_sub '
                                      '(backward decoder)')
        if encoder_type not in ['lstm', 'gru', 'rnn']:
            raise NotImplementedError('encoder_type=%s' % encoder_type)

        # :140-176
        self.encoder_num_units_sub = self.encoder_num_units
        self.decoder_num_units_1 = decoder_num_units_sub
        self.decoder_num_layers_1 = decoder_num_layers_sub
        if decoder_num_layers_sub != 1:
            raise NotImplementedError('MI355X HierarchicalAttentionSeq2seq: multi-layer decoder '
                                      'in the fused training loop')
        self.num_classes_sub = num_classes_sub + 1
        self.sos_1 = num_classes_sub
        self.eos_1 = num_classes_sub
        self.backward_1 = backward_sub
        self.init_dec_state_1_fwd = init_dec_state
        if encoder_type != decoder_type:
            self.init_dec_state_1_fwd = 'zero'
        self.num_heads_1 = num_heads_sub
        self.main_loss_weight = main_loss_weight
        self.sub_loss_weight = sub_loss_weight
        self.ctc_loss_weight_sub = ctc_loss_weight_sub
        self._emb_dims[1] = embedding_dim_sub

        # :181-203: the encoder is rebuilt with the sub-task tap (same slot in _modules)
        self.encoder = load(encoder_type=encoder_type)(
            input_size=input_size, rnn_type=encoder_type, bidirectional=encoder_bidirectional,
            num_units=encoder_num_units, num_proj=encoder_num_proj,
            num_layers=encoder_num_layers, num_layers_sub=encoder_num_layers_sub,
            dropout_input=dropout_input, dropout_hidden=dropout_encoder,
            subsample_list=subsample_list, subsample_type=subsample_type, batch_first=True,
            merge_bidirectional=False, pack_sequence=True, num_stack=num_stack, splice=splice,
            input_channel=input_channel, conv_channels=conv_channels,
            conv_kernel_sizes=conv_kernel_sizes, conv_strides=conv_strides, poolings=poolings,
            activation=activation, batch_norm=batch_norm, residual=encoder_residual,
            dense_residual=encoder_dense_residual)

        self.is_bridge_sub = False
        if self.sub_loss_weight > 0:                              # :221-339
            if self.init_dec_state_1_fwd != 'zero':
                self.W_dec_init_1_fwd = LinearND(self.encoder_num_units_sub,
                                                 decoder_num_units_sub)
            self.decoder_1_fwd = RNNDecoder(
                input_size=self.encoder_num_units_sub + embedding_dim_sub,
                rnn_type=decoder_type, num_units=decoder_num_units_sub,
                num_layers=decoder_num_layers_sub, dropout=dropout_decoder,
                residual=decoder_residual, dense_residual=decoder_dense_residual)
            self.attend_1_fwd = AttentionMechanism(
                encoder_num_units=self.encoder_num_units_sub,
                decoder_num_units=decoder_num_units_sub, attention_type=attention_type,
                attention_dim=attention_dim, sharpening_factor=sharpening_factor,
                sigmoid_smoothing=sigmoid_smoothing, out_channels=attention_conv_num_channels,
                kernel_size=attention_conv_width, num_heads=num_heads_sub)
            self.W_d_1_fwd = LinearND(decoder_num_units_sub, bottleneck_dim_sub,
                                      dropout=dropout_decoder)
            self.W_c_1_fwd = LinearND(self.encoder_num_units_sub, bottleneck_dim_sub,
                                      dropout=dropout_decoder)
            self.fc_1_fwd = LinearND(bottleneck_dim_sub, self.num_classes_sub)
            if label_smoothing_prob > 0:
                self.embed_1 = Embedding_LS(num_classes=self.num_classes_sub,
                                            embedding_dim=embedding_dim_sub,
                                            dropout=dropout_embedding,
                                            label_smoothing_prob=label_smoothing_prob)
            else:
                self.embed_1 = Embedding(num_classes=self.num_classes_sub,
                                         embedding_dim=embedding_dim_sub,
                                         dropout=dropout_embedding)
        if ctc_loss_weight_sub > 0:                               # :344-351
            self.fc_ctc_1 = LinearND(self.encoder_num_units_sub, num_classes_sub + 1)
            self._decode_ctc_greedy_np = GreedyDecoder(blank_index=0)

        # :356-380
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

    @eval_retry
    def forward(self, xs, ys, x_lens, y_lens, ys_sub, y_lens_sub, is_eval=False):
        """:382-567."""
        if is_eval:
            self.eval()
        else:
            self.train()
            if self.weight_noise_injection:
                self.inject_weight_noise(mean=0, std=self.weight_noise_std)
        B = len(xs)
        xs_d = self.np2var(xs, dtype='float')
        enc_out, enc_lens_d, enc_sub, lens_sub_d, _ = self._encode(xs_d, x_lens,
                                                                   is_multi_task=True)
        perm = self.encoder.last_perm_np
        ys = np.asarray(ys)
        ys_sub = np.asarray(ys_sub)
        y_lens = np.asarray(y_lens).astype(np.int64)
        y_lens_sub = np.asarray(y_lens_sub).astype(np.int64)

        hosts = {}
        if self.main_loss_weight > 0:
            ys_in, ys_out = self._ys_in_out(ys, y_lens, self.eos_0, perm)
            hosts[0] = ys_in
            self._ys_in_host = hosts
            loss_main = self.compute_xe_loss(enc_out, self.np2var(ys_in), self.np2var(ys_out),
                                             enc_lens_d, None, task=0, dir='fwd',
                                             weight=self.main_loss_weight)
        else:
            loss_main = enc_out.new_zeros(1)
        loss = loss_main
        loss_sub = ctc_loss_sub = None
        if self.sub_loss_weight > 0:
            ys_in_s, ys_out_s = self._ys_in_out(ys_sub, y_lens_sub, self.eos_1, perm)
            self._ys_in_host = {1: ys_in_s}
            loss_sub = self.compute_xe_loss(enc_sub, self.np2var(ys_in_s), self.np2var(ys_out_s),
                                            lens_sub_d, None, task=1, dir='fwd',
                                            weight=self.sub_loss_weight)
            loss = loss + loss_sub
        if self.ctc_loss_weight_sub > 0:                         # :508-523
            ys_ctc = (ys_sub + 1)[perm]
            yl = y_lens_sub[perm].astype(np.int32)
            ctc_loss_sub = self.compute_ctc_loss(enc_sub, ys_ctc, lens_sub_d, yl, task=1,
                                                 scale=self.ctc_loss_weight_sub)
            loss = loss + ctc_loss_sub
        second = loss_sub if self.sub_loss_weight > self.ctc_loss_weight_sub else ctc_loss_sub
        if is_eval:
            check_recurrences(self)
            return (float(loss.item()), float(loss_main.item()),
                    float(second.item()) if second is not None else 0.0)
        self._step += 1
        if self.ss_prob > 0:
            self._ss_prob = min(self.ss_prob, self.ss_prob / self.ss_max_step * self._step)
        return loss, loss_main, second

    @eval_retry
    def decode(self, xs, x_lens, beam_width, max_decode_len, min_decode_len=0,
               length_penalty=0, coverage_penalty=0, task_index=0, **kwargs):
        """:569-648 (greedy or beam search; the joint word/char decodings
        are not provided): task_index 0 decodes words from the top layer, 1
        characters from layer encoder_num_layers_sub."""
        import torch
        if kwargs.get('joint_decoding') is not None:
            raise NotImplementedError('joint word/char decoding (:620-880)')
        with torch.no_grad():
            self.eval()
            xs_d = self.np2var(xs, dtype='float')
            enc_out, enc_lens_d, enc_sub, lens_sub_d, _ = self._encode(xs_d, x_lens,
                                                                       is_multi_task=True)
            if task_index == 0:
                enc, lens_d, lens_np = enc_out, enc_lens_d, self.encoder.last_lens_np
            else:
                enc, lens_d, lens_np = enc_sub, lens_sub_d, self.encoder.last_lens_sub_np
            if beam_width == 1:
                hyps, aw = self._decode_infer_greedy(enc, lens_d, max_decode_len, task=task_index)
            else:
                hyps, aw = self._decode_infer_beam(enc, lens_np, beam_width, max_decode_len,
                                                   min_decode_len, length_penalty,
                                                   coverage_penalty, task=task_index)
            check_recurrences(self)
            return hyps, aw, self.encoder.last_perm_np.copy()
