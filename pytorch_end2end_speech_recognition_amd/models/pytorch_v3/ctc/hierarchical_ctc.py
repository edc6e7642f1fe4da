"""HierarchicalCTC (reference models/pytorch_v3/ctc/hierarchical_ctc.py) on the
MI355X hot path: word-level CTC on the top encoder layer plus a character-level
CTC on the output of layer ``encoder_num_layers_sub`` (multi-task, SURVEY §8f
rank 3; the Switchboard / WSJ / CSJ hierarchical recipes).

Construction follows the reference step by step -- the plain CTC model is built
and initialised first, then the encoder is rebuilt with the sub-task tap, the
output layers are rebuilt and the sub-task head added, and the initialisation
runs again (hierarchical_ctc.py:83-265) -- so the same seed yields the same
state_dict.  ``forward(xs, ys, x_lens, y_lens, ys_sub, y_lens_sub, is_eval)``
returns (loss, loss_main, loss_sub) with
    loss = main_loss_weight * L_ctc(word) + sub_loss_weight * L_ctc(char)
(hierarchical_ctc.py:267-365); both CTC terms run on the HIP kernel.
"""
import numpy as np

from .ctc import CTC
from ..base import check_recurrences, eval_retry
from ..linear import LinearND
from ..encoders.load_encoder import load


class HierarchicalCTC(CTC):

    def __init__(self, input_size, encoder_type, encoder_bidirectional, encoder_num_units,
                 encoder_num_proj, encoder_num_layers, encoder_num_layers_sub, fc_list,
                 fc_list_sub, dropout_input, dropout_encoder, main_loss_weight, sub_loss_weight,
                 num_classes, num_classes_sub, parameter_init_distribution='uniform',
                 parameter_init=0.1, recurrent_weight_orthogonal=False,
                 init_forget_gate_bias_with_one=True, subsample_list=[], subsample_type='drop',
                 logits_temperature=1, num_stack=1, splice=1, input_channel=1, conv_channels=[],
                 conv_kernel_sizes=[], conv_strides=[], poolings=[], activation='relu',
                 batch_norm=False, label_smoothing_prob=0, weight_noise_std=0,
                 encoder_residual=False, encoder_dense_residual=False):
        # hierarchical_ctc.py:102-127: the plain CTC model first (same arguments;
        # recurrent_weight_orthogonal / init_forget_gate_bias_with_one stay at
        # their defaults there, as in the reference)
        super(HierarchicalCTC, self).__init__(
            input_size=input_size, encoder_type=encoder_type,
            encoder_bidirectional=encoder_bidirectional, encoder_num_units=encoder_num_units,
            encoder_num_proj=encoder_num_proj, encoder_num_layers=encoder_num_layers,
            dropout_input=dropout_input, dropout_encoder=dropout_encoder,
            num_classes=num_classes, parameter_init=parameter_init,
            subsample_list=subsample_list, subsample_type=subsample_type, fc_list=fc_list,
            num_stack=num_stack, splice=splice, input_channel=input_channel,
            conv_channels=conv_channels, conv_kernel_sizes=conv_kernel_sizes,
            conv_strides=conv_strides, poolings=poolings, logits_temperature=logits_temperature,
            batch_norm=batch_norm, label_smoothing_prob=label_smoothing_prob,
            weight_noise_std=weight_noise_std)
        self.model_type = 'hierarchical_ctc'
        self.encoder_num_layers_sub = encoder_num_layers_sub
        self.fc_list_sub = fc_list_sub
        self.num_classes_sub = num_classes_sub + 1
        self.main_loss_weight = main_loss_weight
        self.sub_loss_weight = sub_loss_weight

        if encoder_type not in ['lstm', 'gru', 'rnn']:
            raise NotImplementedError('encoder_type=%s' % encoder_type)
        self.encoder = load(encoder_type=encoder_type)(          # :141-170
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

        if len(fc_list) > 0:                                     # :185-207
            for i in range(len(fc_list)):
                din = self.encoder_num_units if i == 0 else fc_list[i - 1]
                setattr(self, 'fc_' + str(i), LinearND(din, fc_list[i], dropout=dropout_encoder))
            self.fc_out = LinearND(fc_list[-1], self.num_classes)
        else:
            self.fc_out = LinearND(self.encoder_num_units, self.num_classes)
        if len(fc_list_sub) > 0:                                 # :212-234
            for i in range(len(fc_list_sub)):
                din = self.encoder_num_units if i == 0 else fc_list_sub[i - 1]
                setattr(self, 'fc_sub_' + str(i),
                        LinearND(din, fc_list_sub[i], dropout=dropout_encoder))
            self.fc_out_sub = LinearND(fc_list_sub[-1], self.num_classes_sub)
        else:
            self.fc_out_sub = LinearND(self.encoder_num_units, self.num_classes_sub)

        self.init_weights(parameter_init, distribution=parameter_init_distribution,
                          ignore_keys=['bias'])                  # :240-259
        self.init_weights(0, distribution='constant', keys=['bias'])
        if recurrent_weight_orthogonal:
            self.init_weights(parameter_init, distribution='orthogonal',
                              keys=['lstm', 'weight'], ignore_keys=['bias'])
        if init_forget_gate_bias_with_one:
            self.init_forget_gate_bias_with_one()
        self.flatten_parameters_()
        self.encoder.__dict__['_owner'] = self

    @eval_retry
    def forward(self, xs, ys, x_lens, y_lens, ys_sub, y_lens_sub, is_eval=False):
        """hierarchical_ctc.py:267-365."""
        if is_eval:
            self.eval()
        else:
            self.train()
            if self.weight_noise_injection:
                self.inject_weight_noise(mean=0, std=self.weight_noise_std)
        B = len(xs)
        xs_d = self.np2var(xs, dtype='float')
        logits, lens_d, logits_sub, lens_sub_d, _ = self._encode(xs_d, x_lens,
                                                                 is_multi_task=True,
                                                                 defer_head=True)
        if self.logits_temperature != 1:
            logits = logits * (1.0 / self.logits_temperature)
            logits_sub = logits_sub * (1.0 / self.logits_temperature)
        perm = self.encoder.last_perm_np
        loss_main = self._ctc_term(logits, lens_d, ys, y_lens, perm, B) * self.main_loss_weight
        loss_sub = self._ctc_term(logits_sub, lens_sub_d, ys_sub, y_lens_sub, perm,
                                  B) * self.sub_loss_weight
        loss = loss_main + loss_sub
        if is_eval:
            check_recurrences(self)
            return float(loss.item()), float(loss_main.item()), float(loss_sub.item())
        return loss, loss_main, loss_sub
