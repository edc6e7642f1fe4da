"""CPU oracle for the hybrid CTC/attention training step -- TEST INFRASTRUCTURE ONLY.

This package is the checker, never the product.  Only ``tests/``,
``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
it.  The MI355X product path (``pytorch_end2end_speech_recognition_amd``) never
imports anything from here and fails loudly when its HIP library is missing.

Contents
--------
``ctc_ref``  numpy float64 restatement of the CTC forward-backward the reference
             delegates to warp-ctc, following the reference's own numpy CTC text
             (models/chainer/ctc/ctc_loss_from_chainer.py) and the warp-ctc
             contract at models/pytorch_v3/ctc/ctc.py:30-66; plus the CTC
             best-path decoder (models/pytorch_v3/ctc/decoders/greedy_decoder.py).
``asr_ref``  torch-CPU float32/float64 restatement of the model math: packed
             BLSTM encoder with pyramidal "drop" subsampling
             (models/pytorch_v3/encoders/rnn.py), LinearND, location attention
             (models/pytorch_v3/attention/attention_layer.py), the teacher-forced
             bahdanau decoder loop and loss assembly
             (models/pytorch_v3/attention/attention_seq2seq.py), the CTC model
             loss (models/pytorch_v3/ctc/ctc.py) and label smoothing
             (models/pytorch_v3/criterion.py).

Parity pinning
--------------
Both modules are pinned against golden vectors produced by running the
reference itself in the build container (``tests/golden/make_golden.py``; the
reference imports on torch 2.10 CPU with the harness shims documented there).
``tests/test_oracle_golden.py`` checks every fixture.  The warp-ctc binding is
external and unpinned upstream: its boundary behaviour is pinned
to ``torch.nn.functional.ctc_loss`` with warp-ctc conventions (softmax inside,
blank 0, cost 0 / grad 0 for infeasible alignments, gradient scaled by
``grad_output``).
"""
