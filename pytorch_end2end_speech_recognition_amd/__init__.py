"""MI355X-native (gfx950 / CDNA4) hybrid CTC/attention ASR training step.

Drop-in for the hot path of carolinebear/pytorch_end2end_speech_recognition:
``models.load_model.load`` and the ``models.pytorch_v3`` model classes are
mirrored under ``pytorch_end2end_speech_recognition_amd.models``; the per-step
compute runs in hand-written HIP kernels (``csrc/``, exported through the C ABI
in ``include/asr_hip.h`` as ``libasr_hip.so``).
"""
__version__ = '0.1.0'
