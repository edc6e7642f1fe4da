"""Model parameter sets of the BASELINE.json workloads, as the ``params`` dicts
the reference's training script passes to ``models.load_model.load``
(examples/*/s5/exp/training/train.py:112).  Only the model / optimizer keys
load() reads are kept (data, annealing and logging keys are the recipe's own
business and not on the training step).

Sources:
  * timit2x320  -- examples/timit/s5/conf/ctc/blstm_ctc_phone61.yml with the
    BASELINE configs[0] encoder (2 x 320 BLSTM), F = 41 x 3 (delta, delta-delta),
    61 phones;
  * ctc5x512    -- examples/librispeech/s5/conf/ctc/char_blstm_ctc_100h.yml
    scaled to BASELINE configs[1] (5 x 512, no subsampling);
  * attention   -- examples/librispeech/s5/conf/attention/char_blstm_att_100h.yml
    (BASELINE configs[2]; configs[3] adds ctc_loss_weight 0.3);
  * vgg_hier    -- BASELINE configs[4]: VGG [64, 64, 128, 128] + BN in front of a
    4 x 320 BLSTM, hierarchical word (10k) / char CTC (Switchboard recipe shape).
"""

_COMMON = dict(
    use_delta=False, use_double_delta=False, input_channel=1, splice=1, num_stack=1,
    encoder_type='lstm', conv_channels=[], conv_kernel_sizes=[], conv_strides=[], poolings=[],
    activation='relu', batch_norm=False, encoder_bidirectional=True, encoder_residual=False,
    encoder_dense_residual=False, encoder_num_proj=0, subsample_type='drop', fc_list=[],
    optimizer='adam', learning_rate=1e-3, parameter_init_distribution='uniform',
    parameter_init=0.1, recurrent_weight_orthogonal=False, init_forget_gate_bias_with_one=True,
    char_init=False, clip_grad_norm=5.0, weight_decay=1e-6, logits_temperature=1,
    label_smoothing_prob=0, weight_noise_std=0)


def timit2x320():
    p = dict(_COMMON)
    p.update(model_type='ctc', input_freq=41, use_delta=True, use_double_delta=True,
             encoder_num_units=320, encoder_num_layers=2, subsample_list=[],
             dropout_input=0.2, dropout_encoder=0.5, num_classes=61)
    return p


def ctc5x512():
    p = dict(_COMMON)
    p.update(model_type='ctc', input_freq=80, encoder_num_units=512, encoder_num_layers=5,
             subsample_list=[], dropout_input=0, dropout_encoder=0.2, num_classes=28)
    return p


def attention4x320(ctc_loss_weight=0.0):
    p = dict(_COMMON)
    p.update(model_type='attention', input_freq=80, encoder_num_units=320, encoder_num_layers=4,
             subsample_list=[False, True, True, False], decoder_residual=False,
             decoder_dense_residual=False, bridge_layer=False, attention_type='location',
             attention_dim=128, decoder_type='lstm', decoder_num_units=320,
             decoder_num_layers=1, embedding_dim=32, attention_conv_num_channels=10,
             attention_conv_width=201, decoding_order='bahdanau', bottleneck_dim=320,
             num_heads=1, dropout_input=0, dropout_encoder=0.2, dropout_decoder=0.2,
             dropout_embedding=0.2, init_dec_state='zero', sharpening_factor=1.0,
             logits_temperature=1.0, sigmoid_smoothing=False, coverage_weight=0,
             scheduled_sampling_prob=0.2, scheduled_sampling_max_step=20000,
             label_smoothing_prob=0.1, backward_loss_weight=0, ctc_loss_weight=ctc_loss_weight,
             num_classes=28)
    return p


def vgg_hier():
    p = dict(_COMMON)
    p.update(model_type='hierarchical_ctc', input_freq=80, conv_channels=[64, 64, 128, 128],
             conv_kernel_sizes=[[3, 3]] * 4, conv_strides=[[1, 1]] * 4,
             poolings=[[], [2, 2], [], [2, 2]], batch_norm=True, encoder_num_units=320,
             encoder_num_layers=4, encoder_num_layers_sub=3, subsample_list=[], fc_list_sub=[],
             main_loss_weight=0.5, sub_loss_weight=0.5, dropout_input=0, dropout_encoder=0.2,
             num_classes=10000, num_classes_sub=28)
    return p
